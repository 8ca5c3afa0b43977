#!/usr/bin/env python3
"""The operator-path companion alone (bench.operator_run).  Usage: python tools/op_bench.py [n]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
print(json.dumps(bench.operator_run(0, n)), flush=True)
