#!/usr/bin/env python3
"""Where a small query's time goes (C1: MR-Dim 2D uniform 1M, P=8; or a config given by
CFG=C1|C2|C5T): per-kernel HIP-event means over 30 planned queries (profile level 2: every
timed kernel), the wall time per query with no timers, and the same with the measurement
build's SKY_FILTER_DBG modes when SKYLINE_HIP_LIB points at build_measure/ (results invalid
there; the timing of what is left is the point).  Prints one JSON line.
Usage: [SKY_FILTER_DBG=1] python tools/small_query_ab.py"""
import json
import os
import statistics
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "flink-skyline-qos_amd"))
import torch  # noqa: E402

import skyline  # noqa: E402

CFGS = {"C1": ("mr-dim", 2, 8, "uniform", 1_000_000), "C2": ("mr-grid", 4, 8, "correlated", 10_000_000),
        "C5T": ("mr-angle", 6, 8, "mixed", 1_000_000),
        "C4R": ("mr-angle", 8, 16, "anti_correlated", 12_500_000),   # one rank's shard of C4 on 8 GPUs
        "C3": ("mr-angle", 4, 8, "anti_correlated", 50_000_000), "C3R": ("mr-angle", 4, 8, "anti_correlated", 6_250_000),
        "C4H": ("mr-angle", 8, 16, "anti_correlated", 25_000_000)}
name = os.environ.get("CFG", "C1")
algo, D, P, dist, n = CFGS[name]
dev = torch.device("cuda", 0)
eng = skyline.SkylineEngine(D, P, algo, 1000.0, 0)
vals = torch.empty((n, D), dtype=torch.float64, device=dev)
ids = torch.empty(n, dtype=torch.int64, device=dev)
eng.synth_dev(dist, n, vals, ids, seed=1234 + D)
oi = torch.empty(n, dtype=torch.int64, device=dev)
oo = torch.empty(n, dtype=torch.int32, device=dev)
for _ in range(5):
    eng.query_dev(ids, vals, oi, oo, n)
eng.sync()
wall = []
for _ in range(50):
    t0 = time.perf_counter()
    eng.query_dev(ids, vals, oi, oo, n)
    eng.sync()
    wall.append((time.perf_counter() - t0) * 1e3)
# the C entry point alone (no torch stream ordering, no Python wrapper object): sky_query_dev
import ctypes  # noqa: E402
from skyline._abi import lib  # noqa: E402
cnt = ctypes.c_int64(0)
raw = []
args = (eng.h, ctypes.c_void_p(ids.data_ptr()), ctypes.c_void_p(vals.data_ptr()), n, ctypes.c_void_p(oi.data_ptr()),
        ctypes.c_void_p(oo.data_ptr()), n, ctypes.byref(cnt))
for _ in range(50):
    t0 = time.perf_counter()
    lib().sky_query_dev(*args)
    raw.append((time.perf_counter() - t0) * 1e3)
eng.profile(2)
eng.profile_reset()
for _ in range(30):
    eng.query_dev(ids, vals, oi, oo, n)
eng.sync()
kern = {}
for k in ("filter", "prefilter", "brute", "out", "outc", "outw", "mbr", "sfs_small"):
    ms, la, _ = eng.kernel_time(k)
    if la:
        kern[k] = ms / la
phases, counters = eng.phases()
eng.close()
print(json.dumps({"config": name, "filter_dbg": os.environ.get("SKY_FILTER_DBG"),
                  "filter_tpb": os.environ.get("SKY_FILTER_TPB"), "filter_pf": os.environ.get("SKY_FILTER_PF"),
                  "lib": os.path.basename(os.path.dirname(skyline._abi.LIB_PATH)),
                  "wall_p50_ms": statistics.median(wall), "wall_min_ms": min(wall),
                  "c_entry_p50_ms": statistics.median(raw), "c_entry_min_ms": min(raw),
                  "kernel_mean_ms_profiled": kern, "route_bits": int(counters[7]) & 0xff}), flush=True)
