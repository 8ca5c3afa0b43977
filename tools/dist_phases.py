#!/usr/bin/env python3
"""Per-rank phase table of the multi-GPU step, EMULATED ON ONE GPU (not a scaling curve).

W ranks run one after the other on the same device, one context per rank (as
tests/conftest.py dist_emulate does); the all-gather is a device concatenation of the
blocks and the all-reduce a device sum.  Each rank's export / merge / finish call is
timed alone (device synchronised before and after), so the per-rank numbers are what one
rank's GPU would spend on its own shard -- without the xGMI transfer, which RCCL adds.
The union-fate kernel time is the HIP-event pair around it (profile level 1).

Workloads (BASELINE.json configs[2], configs[3], and the labelled std-anti stream):
  c4_8way      MR-Angle 8D anti-correlated (reference formula) 100M, P=16, 8 ranks
  c3_{2,4,8}way MR-Angle 4D anti-correlated 50M, P=8
  std_anti_4x2M MR-Angle 8D std-anti 4 x 2M, P=16 (the dominance-bound union)
Every decomposition is checked against the one-GPU query (ids, origins, |L_k|, survivors_k).

Usage: python tools/dist_phases.py [--only c4_8way,...] [--out profiles/r06_dist_emulated_phases.json]
"""
import argparse
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
from skyline import _abi  # noqa: E402
from skyline.dist import block_words, stats_words  # noqa: E402


def now():
    torch.cuda.synchronize()
    return time.perf_counter()


def one_gpu(D, P, dist, n, seed, reps=3):
    eng = skyline.SkylineEngine(D, P, "mr-angle", 1000.0, 0)
    vals = torch.empty((n, D), dtype=torch.float64, device="cuda")
    ids = torch.empty(n, dtype=torch.int64, device="cuda")
    eng.synth_dev(dist, n, vals, ids, seed=seed)
    eng.sync()
    oi = torch.empty(n, dtype=torch.int64, device="cuda")
    oo = torch.empty(n, dtype=torch.int32, device="cuda")
    ms = []
    for _ in range(reps):
        t0 = now()
        g = eng.query_dev(ids, vals, oi, oo, n)
        eng.sync()
        ms.append((now() - t0) * 1e3)
    ls, sv = eng.stats()
    exp = (oi[:g].cpu().numpy(), oo[:g].cpu().numpy(), ls, sv)
    eng.close()
    return vals, ids, exp, float(np.median(ms))


def step(engs, di, dv, cap, timed):
    """One multi-GPU step; with timed=True every rank's calls are timed alone."""
    W = len(engs)
    D, K = engs[0].dims, engs[0].K
    oi = [torch.empty(max(v.shape[0], 1), dtype=torch.int64, device="cuda") for v in dv]
    oo = [torch.empty(max(v.shape[0], 1), dtype=torch.int32, device="cuda") for v in dv]
    rows = [dict() for _ in range(W)]
    export, attempts = True, 0
    while True:
        attempts += 1
        assert attempts <= 8
        send = [torch.empty(block_words(cap, D), dtype=torch.int64, device="cuda") for _ in range(W)]
        for r, e in enumerate(engs):
            t0 = now()
            if export:
                e.dist_export_dev(di[r], dv[r], send[r], cap)
            else:
                e.dist_reblock_dev(send[r], cap)
            e.sync()
            rows[r]["export_ms"] = (now() - t0) * 1e3
        recv = torch.cat(send)
        stats = [torch.empty(stats_words(K), dtype=torch.int64, device="cuda") for _ in range(W)]
        for r, e in enumerate(engs):
            u0 = e.kernel_time("union_fate")[0]
            t0 = now()
            e.dist_merge_dev(recv, W, r, cap, oi[r], oo[r], dv[r].shape[0], stats[r])
            e.sync()
            rows[r]["merge_ms"] = (now() - t0) * 1e3
            rows[r]["union_fate_kernel_ms"] = e.kernel_time("union_fate")[0] - u0
        tot = torch.stack(stats).sum(0)
        res = []
        for r, e in enumerate(engs):
            t0 = now()
            res.append(e.dist_finish(tot, dv[r].shape[0]))
            rows[r]["finish_ms"] = (now() - t0) * 1e3
        rc = {x[0] for x in res}
        assert len(rc) == 1, res
        rc = rc.pop()
        if rc == _abi.SKY_OK:
            break
        if rc == _abi.SKY_E_RETRY:
            export = True
        else:
            cap = max(x[2] for x in res) + 64
            export = False
    for r, e in enumerate(engs):
        cnt = e.phases()[1]
        rows[r]["own_vectors"] = int(cnt[3])
        rows[r]["union_vectors"] = int(cnt[5])
        rows[r]["route"] = "bounding_box" if int(cnt[6]) else "pair_kernel"
        rows[r]["host_syncs"] = None
    got = [(oi[r][:res[r][1]].cpu().numpy(), oo[r][:res[r][1]].cpu().numpy()) for r in range(W)]
    ls, sv = engs[0].stats()
    return rows, got, (ls, sv), cap, attempts


def run(name, D, P, dist, n, W, seed, steps=4):
    vals, ids, exp, one_ms = one_gpu(D, P, dist, n, seed)
    bounds = np.linspace(0, n, W + 1).astype(np.int64)
    sl = [slice(int(bounds[r]), int(bounds[r + 1])) for r in range(W)]
    di = [ids[x] for x in sl]
    dv = [vals[x] for x in sl]
    engs = [skyline.SkylineEngine(D, P, "mr-angle", 1000.0, 0) for _ in range(W)]
    for e in engs:
        e.profile(1)
    cap = 4096
    table = []
    ok = True
    for s in range(steps):
        h0 = [e.host_syncs() for e in engs]
        rows, got, (ls, sv), cap, attempts = step(engs, di, dv, cap, True)
        for r, e in enumerate(engs):
            rows[r]["host_syncs"] = e.host_syncs() - h0[r]
        ids_all = np.concatenate([g[0] for g in got])
        org_all = np.concatenate([g[1] for g in got])
        ok &= (np.array_equal(ids_all, exp[0]) and np.array_equal(org_all, exp[1]) and
               np.array_equal(ls, exp[2]) and np.array_equal(sv, exp[3]))
        table.append({"step": s, "attempts": attempts, "cap": cap, "ranks": rows})
        print(f"{name} step {s}: attempts {attempts} union_fate_ms "
              f"{[round(x['union_fate_kernel_ms'], 4) for x in rows]} "
              f"merge_ms {[round(x['merge_ms'], 3) for x in rows]}", flush=True)
    for e in engs:
        e.close()
    last = table[-1]["ranks"]
    out = {"workload": name, "dims": D, "partitions": P, "dist": dist, "tuples_total": n, "ranks": W,
           "exact_vs_one_gpu_query": bool(ok), "one_gpu_query_ms": one_ms,
           "last_step": {
               "worst_rank_union_fate_kernel_ms": max(x["union_fate_kernel_ms"] for x in last),
               "worst_rank_export_ms": max(x["export_ms"] for x in last),
               "worst_rank_merge_ms": max(x["merge_ms"] for x in last),
               "worst_rank_finish_ms": max(x["finish_ms"] for x in last),
               "worst_rank_sum_ms": max(x["export_ms"] + x["merge_ms"] + x["finish_ms"] for x in last)},
           "steps": table}
    del vals, ids, di, dv
    torch.cuda.empty_cache()
    return out


def std_anti_union(W=4, per=2_000_000):
    """std-anti 8D W x per: each rank's bounding-box own-vs-union pass against the one-GPU pass
    over the same union's vectors (tools/dist_union_bench.py's comparison)."""
    from skyline.dist import unpack_blocks
    D, P = 8, 16
    res = run(f"std_anti_{W}x{per // 1_000_000}M", D, P, "std_anti", W * per, W, 1234 + D, steps=3)
    # the same union on one GPU: its exported vectors as one query, the bounding-box pass timed
    n = W * per
    eng = skyline.SkylineEngine(D, P, "mr-angle", 1000.0, 0)
    vals = torch.empty((n, D), dtype=torch.float64, device="cuda")
    ids = torch.empty(n, dtype=torch.int64, device="cuda")
    eng.synth_dev("std_anti", n, vals, ids, seed=1234 + D)
    engs = [skyline.SkylineEngine(D, P, "mr-angle", 1000.0, 0) for _ in range(W)]
    cap = res["steps"][-1]["cap"]
    send = [torch.empty(block_words(cap, D), dtype=torch.int64, device="cuda") for _ in range(W)]
    for r, e in enumerate(engs):
        e.dist_export_dev(ids[r * per:(r + 1) * per], vals[r * per:(r + 1) * per], send[r], cap)
    blocks = unpack_blocks(torch.cat(send), W, cap, D)
    urows = torch.cat([b[0] for b in blocks]).contiguous()
    m = urows.shape[0]
    uo = torch.empty(m, dtype=torch.int64, device="cuda")
    uorg = torch.empty(m, dtype=torch.int32, device="cuda")
    uid = torch.arange(m, dtype=torch.int64, device="cuda")
    eng.profile(1)
    eng.query_dev(uid, urows, uo, uorg, m)
    eng.sync()
    eng.profile_reset()
    t = []
    for _ in range(3):
        a = eng.kernel_time("mbr")[0]
        eng.query_dev(uid, urows, uo, uorg, m)
        eng.sync()
        t.append(eng.kernel_time("mbr")[0] - a)
    for e in engs:
        e.close()
    eng.close()
    mbr_ms = float(np.median(t))
    res["one_gpu_mbr_pass_over_the_union_ms"] = mbr_ms
    res["worst_rank_union_fate_vs_one_gpu_union_pass"] = \
        res["last_step"]["worst_rank_union_fate_kernel_ms"] / mbr_ms if mbr_ms else None
    del vals, ids, urows
    torch.cuda.empty_cache()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="c4_8way,c3_2way,c3_4way,c3_8way,std_anti_4x2M")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    want = a.only.split(",")
    outs = []
    if "c4_8way" in want:
        outs.append(run("c4_8way", 8, 16, "anti_correlated", 100_000_000, 8, 1242))
    for W in (2, 4, 8):
        if f"c3_{W}way" in want:
            outs.append(run(f"c3_{W}way", 4, 8, "anti_correlated", 50_000_000, W, 1238))
    if "std_anti_4x2M" in want:
        outs.append(std_anti_union())
    doc = {"label": "emulated on one GPU, not a scaling curve: W ranks run one after the other on one MI355X, "
                    "each rank's calls timed alone; the all-gather is a device concatenation (no xGMI time)",
           "device": torch.cuda.get_device_name(0), "workloads": outs}
    s = json.dumps(doc, indent=1)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            f.write(s + "\n")
    for o in outs:
        print(json.dumps({k: o[k] for k in o if k != "steps"}), flush=True)


if __name__ == "__main__":
    main()
