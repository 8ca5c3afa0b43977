#!/usr/bin/env python3
"""The dense all-pairs dominance kernel alone (bench.dominance_dense_run: k_brute16_pairs on
std-anti 8D rows with their MR-Angle keys, every row against every row).  For rocprofv3
kernel traces / PMC passes of that kernel by itself.
Usage: python tools/dense_bench.py [n ...]   (default 16384 65536)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

sizes = [int(x) for x in sys.argv[1:]] or [16384, 65536]
for n in sizes:
    r = bench.dominance_dense_run(torch.device("cuda", 0), 8, 16, n, 1234 + 8)
    print(json.dumps({k: r[k] for k in ("workload", "kernel", "pair_tests", "kernel_ms", "achieved", "frac",
                                        "frac_32bit", "rows_not_dominated")}), flush=True)
