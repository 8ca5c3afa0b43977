#!/usr/bin/env python3
"""The radix-sort-at-scale companion alone (bench.sort_run).  Usage: python tools/sort_bench.py [n]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
eng = bench.skyline.SkylineEngine(8, 16, "mr-angle", 1000.0, 0)
r = bench.sort_run(eng, n, torch.device("cuda", 0))
print(json.dumps({k: r[k] for k in ("passes", "ms", "achieved", "frac")}), flush=True)
