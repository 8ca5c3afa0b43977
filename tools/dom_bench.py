#!/usr/bin/env python3
"""The dominance-bound companion alone (bench.dominance_run): std-anti 8D, MR-Angle P=16.
Usage: python tools/dom_bench.py [n] [steps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
D = int(os.environ.get("DOM_D", "8"))
r = bench.dominance_run(torch.device("cuda", 0), D, 16, n, 1234 + D, steps, 2)
print(json.dumps({k: r.get(k) for k in ("ms_per_query", "dominance_ms", "pair_tests_executed", "pair_tests_W", "frac",
                                        "W_rate", "path", "skyline_size", "tile_pairs_tested")}), flush=True)
