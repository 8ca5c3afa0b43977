#!/usr/bin/env python3
"""The multi-GPU merge on the dominance-bound stream (std-anti 8D, MR-Angle P=16): W ranks
emulated on one GPU (one context per rank, tests/conftest.py dist_emulate), PER tuples each.
Reports each rank's own-vs-union time (HIP events around the union-fate pass: the bounding-box
pass of own tiles against union tiles) against the one-GPU bounding-box pass over the same
union (the union's vectors run as one query: k_mbr over all of them), and checks the
decomposition against the one-GPU query over the whole stream.
Usage: python tools/dist_union_bench.py [PER] [W]"""
import json
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "flink-skyline-qos_amd"))
sys.path.insert(0, os.path.join(R, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import skyline  # noqa: E402
from conftest import dist_emulate  # noqa: E402
from skyline.dist import unpack_blocks, block_words  # noqa: E402

per = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
W = int(sys.argv[2]) if len(sys.argv) > 2 else 4
D, P = 8, 16
n = per * W
eng = skyline.SkylineEngine(D, P, "mr-angle", 1000.0, 0)
vals = torch.empty((n, D), dtype=torch.float64, device="cuda")
ids = torch.empty(n, dtype=torch.int64, device="cuda")
eng.synth_dev("std_anti", n, vals, ids, seed=1234 + D)
oi = torch.empty(n, dtype=torch.int64, device="cuda")
oo = torch.empty(n, dtype=torch.int32, device="cuda")
g = eng.query_dev(ids, vals, oi, oo, n)
eng.sync()
t0 = time.perf_counter()
g = eng.query_dev(ids, vals, oi, oo, n)
eng.sync()
one_gpu_ms = (time.perf_counter() - t0) * 1e3
exp_ids = oi[:g].cpu().numpy()
exp_ls, exp_sv = eng.stats()

engs = [skyline.SkylineEngine(D, P, "mr-angle", 1000.0, 0) for _ in range(W)]
sh_i = [ids[r * per:(r + 1) * per] for r in range(W)]
sh_v = [vals[r * per:(r + 1) * per] for r in range(W)]
dist_emulate(engs, sh_i, sh_v)                        # learns the capacity and the route
for e in engs:
    e.profile(1)
    e.profile_reset()
t0 = time.perf_counter()
out = dist_emulate(engs, sh_i, sh_v, cap=1 << 22)[0]
step_ms = (time.perf_counter() - t0) * 1e3
ok = (np.array_equal(out["ids"], exp_ids) and np.array_equal(out["ls"], exp_ls) and
      np.array_equal(out["sv"], exp_sv))
union_ms = [e.kernel_time("union_fate")[0] for e in engs]
cnt = [e.phases()[1] for e in engs]
own = [int(c[3]) for c in cnt]
n_union = int(cnt[0][5])

# the same union on one GPU: its vectors (one row per distinct exported vector) as one query
send = [torch.empty(block_words(1 << 22, D), dtype=torch.int64, device="cuda") for _ in range(W)]
for r, e in enumerate(engs):
    e.dist_export_dev(sh_i[r], sh_v[r], send[r], 1 << 22)
blocks = unpack_blocks(torch.cat(send), W, 1 << 22, D)
urows = torch.cat([b[0] for b in blocks]).contiguous()
eng.profile(1)
eng.profile_reset()
uo = torch.empty(urows.shape[0], dtype=torch.int64, device="cuda")
uorg = torch.empty(urows.shape[0], dtype=torch.int32, device="cuda")
uid = torch.arange(urows.shape[0], dtype=torch.int64, device="cuda")
eng.query_dev(uid, urows, uo, uorg, urows.shape[0])
eng.sync()
eng.profile_reset()
eng.query_dev(uid, urows, uo, uorg, urows.shape[0])
eng.sync()
mbr_ms = eng.kernel_time("mbr")[0]
print(json.dumps({"workload": f"std_anti 8D, MR-Angle P=16, {W} emulated ranks x {per} tuples",
                  "exact_vs_one_gpu_query": ok, "one_gpu_query_ms": one_gpu_ms,
                  "dist_step_ms_emulated_serial": step_ms, "own_vectors": own, "union_vectors": n_union,
                  "union_route": int(cnt[0][6]), "per_rank_union_fate_ms": union_ms,
                  "one_gpu_mbr_pass_over_the_union_ms": mbr_ms,
                  "worst_rank_vs_one_gpu_union": max(union_ms) / mbr_ms if mbr_ms else None}), flush=True)
