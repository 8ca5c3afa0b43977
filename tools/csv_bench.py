#!/usr/bin/env python3
"""The CSV-ingest companion alone (bench.csv_ingest_run) on the C4 stream: decode time, per-kernel
times, CSV -> skyline.  Usage: python tools/csv_bench.py [n]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import skyline  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
D = 8
dev = torch.device("cuda", 0)
eng = skyline.SkylineEngine(D, 16, "mr-angle", 1000.0, 0)
vals, ids = bench.make_stream(eng, "anti_correlated", n, 1234 + D, 0, dev)
out_ids = torch.empty(n, dtype=torch.int64, device=dev)
out_org = torch.empty(n, dtype=torch.int32, device=dev)
r = bench.csv_ingest_run(eng, ids, vals, n, D, 3, out_ids, out_org)
print(json.dumps({k: r[k] for k in ("decode_ms", "kernels_ms", "kernel_ms", "csv_to_skyline_ms", "frac", "records")}),
      flush=True)
