#!/usr/bin/env python3
"""bench.py — skyline tuples/sec (+ p50 query latency) on MI355X.

Workload (BASELINE.json metric, config C4 on one GPU per rank): MR-Angle, 8D,
anti-correlated stream (the reference producer's formula,
python/unified_producer.py:89-123, counter RNG), P = 16 partitions, domain
[0,1000], N tuples per rank (default 100M) generated directly in HBM.

A step = one query over the whole landmark window (every tuple of the rank's
shard): partition keys -> local skylines of the P partitions -> global merge ->
stream-ordered skyline ids, with inputs already resident in HBM.  With N GPUs
(one process per GPU, launched by torch.distributed.run) every rank holds its
own N-tuple shard (weak scaling) and the ranks exchange their local skylines'
distinct vectors with one RCCL all-gather (skyline/dist.py).

Extra fields: "roofline" for the dominant kernel (k_filter, HBM-bound), timed
with HIP events on the stream it is launched on; "cpu_baseline" = the C
restatement of the reference BNL operators (oracle/, 1 thread) timed on a
bounded prefix of the same stream (rank 0, N=1 only).
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "flink-skyline-qos_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import skyline  # noqa: E402
from skyline import _abi  # noqa: E402
from skyline.dist import distributed_query  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X spec (MI355X_MICROARCH.md: 8.0 TB/s spec, 6.29 measured copy)
# VALU compare peak: 256 CU x 4 SIMD-32 x 32 lanes/clk x 2.4 GHz = one 32-bit compare per
# lane-cycle (MI355X_MICROARCH.md: SIMD-32, wave64 VALU op over 2 cycles; 157.3 TF fp32
# vector = 78.6 T FMA/s).  tools/probe/valu_probe measured 65 T v_add_f32 lane-ops/s.
VALU_PEAK_CMPS = 256 * 4 * 32 * 2.4e9


def dominance_run(dev, D, P, n, seed, steps, warmup):
    """Dominance-bound companion measurement (SURVEY §7 'std-anti'): the reference
    formula's 8D stream has ONE distinct skyline vector, so the pairwise phase is
    priced on the labelled standard anti-correlated generator instead.  achieved =
    D x W / (time of the dominance kernels), W = algorithmic pair tests over distinct
    vectors (sky_profile_dominance)."""
    eng = skyline.SkylineEngine(D, P, "mr-angle", 1000.0, dev.index or 0)
    vals = torch.empty((n, D), dtype=torch.float64, device=dev)
    ids = torch.empty(n, dtype=torch.int64, device=dev)
    eng.synth_dev("std_anti", n, vals, ids, seed=seed)
    out_ids = torch.empty(n, dtype=torch.int64, device=dev)
    out_org = torch.empty(n, dtype=torch.int32, device=dev)
    for _ in range(warmup):
        eng.query_dev(ids, vals, out_ids, out_org, n)
    eng.sync()
    eng.profile(True)
    eng.profile_reset()
    t0 = time.perf_counter()
    g = 0
    for _ in range(steps):
        g = eng.query_dev(ids, vals, out_ids, out_org, n)
    eng.sync()
    dt = (time.perf_counter() - t0) / steps
    eng.profile(False)
    w = eng.dominance_work()
    dom_ms, dom_launches, _ = eng.kernel_time("dom")
    phases, counters = eng.phases()
    dom_ms /= steps
    achieved = D * w / (dom_ms / 1e3) if dom_ms > 0 else 0.0
    eng.close()
    return {"bound": "valu", "kernel": "k_dom16 (+k_xcompact16), HIP events over every SFS round",
            "workload": f"std_anti (labelled extension generator) {D}D, {n} tuples, MR-Angle P={P}",
            "tuples_per_s": n / dt, "ms_per_query": dt * 1e3, "skyline_size": g,
            "pair_tests_W": w, "compares": D * w, "dominance_ms": dom_ms,
            "achieved": achieved, "peak": VALU_PEAK_CMPS, "unit": "compares/s",
            "frac": achieved / VALU_PEAK_CMPS, "path": "u16" if int(counters[7]) & 4 else "f32/f64",
            "local_sfs_ms": phases["local_sfs"], "global_sfs_ms": phases["global_sfs"],
            "sfs_rounds": int(counters[5])}


def csv_ingest_run(eng, ids, vals, n, D, steps, out_ids, out_org):
    """Bulk CSV -> SoA decode (ServiceTuple.fromString, ServiceTuple.java:89-104)
    on the same stream, formatted as the producer's payload (unified_producer.py:174) in HBM.
    Algorithmic bytes per record = its text bytes (read once) + 8 (id) + 8D (row) written.
    Also times decode + query together: skyline tuples/s from raw CSV bytes resident in HBM."""
    nb = eng.format_csv_dev(ids, vals, n)
    text = torch.empty(nb, dtype=torch.uint8, device=vals.device)
    eng.format_csv_dev(ids, vals, n, text, nb)
    pi = torch.empty_like(ids)
    pv = torch.empty_like(vals)
    eng.parse_csv_dev(text, nb, pi, pv, n)                 # warm-up
    eng.sync()
    assert torch.equal(pi, ids) and torch.equal(pv, vals), "CSV round trip differs"
    eng.profile(True)
    eng.profile_reset()
    t0 = time.perf_counter()
    for _ in range(steps):
        m, _ = eng.parse_csv_dev(text, nb, pi, pv, n)
    eng.sync()
    dt_parse = (time.perf_counter() - t0) / steps
    kt = {k: eng.kernel_time(k) for k in ("csv_count", "csv_lines", "csv_parse")}
    eng.profile(False)
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.parse_csv_dev(text, nb, pi, pv, n)
        g = eng.query_dev(pi, pv, out_ids, out_org, n)
    eng.sync()
    dt_e2e = (time.perf_counter() - t0) / steps
    alg = nb + n * (8 + 8 * D)
    p_ms = kt["csv_parse"][0] / max(kt["csv_parse"][1], 1)
    k_ms = sum(kt[k][0] / max(kt[k][1], 1) for k in kt)
    del text, pi, pv
    achieved = (nb + n * (8 + 8 * D)) / (p_ms / 1e3) / 1e9
    return {"bound": "hbm", "kernel": "k_csv_parse (+ k_csv_nl_count, k_csv_nl_write)",
            "workload": f"C4 stream as producer CSV text, {n} records, {nb} bytes",
            "text_bytes": nb, "records": m,
            "decode_ms": dt_parse * 1e3, "kernels_ms": k_ms,
            "kernel_ms": {k: kt[k][0] / max(kt[k][1], 1) for k in kt},
            "decode_records_per_s": n / dt_parse,
            "csv_to_skyline_tuples_per_s": n / dt_e2e, "csv_to_skyline_ms": dt_e2e * 1e3, "skyline_size": g,
            "alg_bytes_per_launch": alg,
            "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
            "all_passes_GBs": alg / (k_ms / 1e3) / 1e9}


def stream_run(dev_index, seed, triggers=20, per_trigger=1_000_000, batch=50_000, window=0):
    """Config C5: continuous queries over a 6D mixed stream (65536-tuple blocks
    cycling the producer's uniform / correlated / anti-correlated formulas), MR-Angle, P = 8
    (Flink parallelism 4).  Micro-batches of `batch` tuples arrive from pinned host memory
    (H2D included); a query_trigger every `per_trigger` tuples.  Latency = trigger -> global
    skyline ids in host memory.  window=0: the reference's landmark window; window=W:
    the count-based sliding window extension."""
    import numpy as np
    D, P = 6, 8
    n = triggers * per_trigger
    vals_np, ids_np = skyline.synth_host(_abi.DISTS["mixed"], D, n, seed=seed)
    vals = torch.from_numpy(vals_np).pin_memory().numpy()
    ids = torch.from_numpy(ids_np).pin_memory().numpy()
    eng = skyline.SkylineEngine(D, P, "mr-angle", 1000.0, dev_index)
    st = skyline.SkylineStream(eng, window)
    lat, sizes = [], []
    t_start = time.perf_counter()
    for t in range(triggers):
        base = t * per_trigger
        for b0 in range(base, base + per_trigger, batch):
            st.append(ids[b0:b0 + batch], vals[b0:b0 + batch])
        tq = time.perf_counter()
        g = st.query_host_view()
        lat.append((time.perf_counter() - tq) * 1e3)
        sizes.append(g)
    total = time.perf_counter() - t_start
    resident, _ = st.size()
    st.close()
    eng.close()
    rate = n / total
    return {"workload": (f"C5: 6D mixed stream, MR-Angle P={P}, {batch}-tuple micro-batches from pinned host "
                         f"memory, query_trigger every {per_trigger} tuples, {triggers} triggers, "
                         + ("landmark window (reference semantics)" if window == 0
                            else f"count-based sliding window W={window} (extension)")),
            "ingest_tuples_per_s": rate, "sustains_10M_per_s": rate >= 1e7,
            "p50_query_latency_ms": statistics.median(lat), "max_query_latency_ms": max(lat),
            "skyline_size_last": sizes[-1], "resident_tuples_last": resident}


def sort_run(eng, n, dev, steps=3):
    """Sort phase at scale (HBM GB/s of the sort): the pipeline's radix sort
    (k_radix.hip) alone on n pairs keyed like its candidate keys (4-bit partition | 32-bit
    score | 16-bit hash, 52 varying bits -> 7 onesweep passes).  Algorithmic bytes =
    passes x n x 24 (read + write a u64 key and a u32 value per pass)."""
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    part = torch.randint(0, 16, (n,), device=dev, dtype=torch.int64, generator=g)
    score = torch.randint(0, 1 << 32, (n,), device=dev, dtype=torch.int64, generator=g)
    hsh = torch.randint(0, 1 << 16, (n,), device=dev, dtype=torch.int64, generator=g)
    keys0 = (part << 56) | (score << 24) | hsh
    del part, score, hsh
    vals0 = torch.arange(n, device=dev, dtype=torch.int32)
    kor = torch.zeros((), dtype=torch.int64, device=dev)
    kand = torch.full((), -1, dtype=torch.int64, device=dev)
    for b in range(64):   # varying key bits / bytes, to cross-check the library's pass count
        bit = (keys0 >> b) & 1
        kor |= bit.max() << b
        kand &= (bit.min() << b) | ~(torch.ones((), dtype=torch.int64, device=dev) << b)
    varying = int((kor ^ kand).item())
    var_bytes = sum(1 for byte in range(8) if (varying >> (8 * byte)) & 0xff)
    best, passes = None, 0
    for i in range(steps + 1):
        keys = keys0.clone()
        vals = vals0.clone()
        passes, ms = eng.profile_sort_dev(keys, vals)
        if i > 0:
            best = ms if best is None else min(best, ms)
    # the result is sorted (as unsigned: keys are non-negative) and a permutation
    assert bool((keys[1:] >= keys[:-1]).all()), "radix sort output not sorted"
    assert torch.equal(keys0[vals.long()], keys), "radix sort values do not follow their keys"
    alg = passes * n * 24
    achieved = alg / (best / 1e3) / 1e9
    del keys0, vals0, keys, vals
    return {"bound": "hbm", "kernel": "k_rs_onesweep (+ k_rs_hist_all, k_rs_scan_all)",
            "workload": f"{n} (u64 key, u32 value) pairs, {bin(varying & ((1 << 64) - 1)).count('1')} varying "
                        f"key bits in {var_bytes} bytes", "passes": passes,
            "ms": best, "keys_per_s": n / (best / 1e3), "alg_bytes": alg,
            "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS}


def cpu_baseline(d, P, dist_name, seed, sample, domain):
    """Reference algorithm restated in C (per-key BNL, buffer 5000, single-threaded
    global BNL), one thread, on the first `sample` tuples of the same stream."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from conftest import Oracle   # test infrastructure: the checker / CPU baseline only
    orc = Oracle()
    vals = orc.synth(_abi.DISTS[dist_name], d, sample, seed=seed)
    ids = np.arange(sample, dtype=np.int64)
    t0 = time.perf_counter()
    g, _, _, _ = orc.query_bnl("angle", vals, ids, P, domain)
    dt = time.perf_counter() - t0
    # one thread per Flink subtask for the local phase (keys round-robin), single-threaded merge
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    threads = max(1, min(16, cores, P))
    t0 = time.perf_counter()
    g2, _, _, _ = orc.query_bnl_mt("angle", vals, ids, P, threads, domain)
    dt2 = time.perf_counter() - t0
    assert sorted(g.tolist()) == sorted(g2.tolist())
    return sample / dt, dt, len(g), sample / dt2, dt2, threads


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--tuples", type=int, default=100_000_000, help="tuples per rank (GPU)")
    ap.add_argument("--dims", type=int, default=8)
    ap.add_argument("--partitions", type=int, default=16)
    ap.add_argument("--dist", default="anti_correlated")
    ap.add_argument("--seed", type=int, default=1242)
    ap.add_argument("--cpu-sample", type=int, default=60000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dom-n", type=int, default=2_000_000, help="tuples of the dominance-bound companion run")
    ap.add_argument("--no-dominance", action="store_true")
    ap.add_argument("--no-csv", action="store_true", help="skip the CSV-ingest companion measurement")
    ap.add_argument("--no-stream", action="store_true", help="skip the C5 continuous-query companion measurement")
    ap.add_argument("--no-sort", action="store_true", help="skip the radix-sort-at-scale companion measurement")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL over xGMI, the measured path) or gloo (rehearsing ranks on one GPU)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    dev_index = local_rank % max(torch.cuda.device_count(), 1)   # > 1 rank per GPU only with gloo
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    red_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")

    D, P, n = args.dims, args.partitions, args.tuples
    eng = skyline.SkylineEngine(D, P, "mr-angle", 1000.0, dev_index)
    vals = torch.empty((n, D), dtype=torch.float64, device=dev)
    ids = torch.empty(n, dtype=torch.int64, device=dev)
    eng.synth_dev(args.dist, n, vals, ids, seed=args.seed, id0=rank * n)
    eng.sync()
    out_ids = torch.empty(n, dtype=torch.int64, device=dev)
    out_org = torch.empty(n, dtype=torch.int32, device=dev)

    def step():
        if distributed:
            return distributed_query(eng, ids, vals, out_ids, out_org, n)
        return eng.query_dev(ids, vals, out_ids, out_org, n)

    for _ in range(args.warmup):
        step()
    eng.sync()
    torch.cuda.synchronize()
    eng.profile(True)
    eng.profile_reset()
    step_ms = []
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g = 0
    for _ in range(args.steps):
        ts = time.perf_counter()
        g = step()
        eng.sync()
        step_ms.append((time.perf_counter() - ts) * 1e3)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    eng.profile(False)
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        gt = torch.tensor([g], dtype=torch.int64, device=red_dev)
        dist.all_reduce(gt)
        g = int(gt.item())
    phases, counters = eng.phases()
    f_ms, f_launch, f_units = eng.kernel_time("filter")

    if rank == 0:
        ms_per_step = elapsed * 1e3 / args.steps
        total = n * world
        value = total / (ms_per_step / 1e3)
        bytes_per_tuple = D * 8 + 2            # read the f64 row once, write the u16 status word
        avg_ms = f_ms / max(f_launch, 1)
        achieved = (bytes_per_tuple * (f_units / max(f_launch, 1))) / (avg_ms / 1e3) / 1e9 if f_launch else 0.0
        traffic = None
        tf = os.path.join(REPO, "profiles", "traffic_filter.json")
        if os.path.exists(tf):
            try:
                tj = json.load(open(tf))
                if tj.get("n") == n and tj.get("dims") == D and tj.get("dist") == args.dist:
                    traffic = tj.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            rate, dt, gs, rate_mt, dt_mt, thr = cpu_baseline(D, P, args.dist, args.seed, args.cpu_sample, 1000.0)
            cpu = {"value": rate_mt, "unit": "tuples/s", "cores": thr, "kind": "port",
                   "sample": f"first {args.cpu_sample} tuples of the same stream, oracle/ C restatement of the "
                             f"reference per-key BNL (buffer 5000), one thread per subtask ({thr}), then the "
                             f"single-threaded global BNL: {dt_mt:.1f} s, skyline {gs}",
                   "single_thread": {"value": rate, "cores": 1, "seconds": dt}}
        csvr = None
        if world == 1 and not args.no_csv:
            csvr = csv_ingest_run(eng, ids, vals, n, D, 3, out_ids, out_org)
        sortr = None
        if world == 1 and not args.no_sort:
            sortr = sort_run(eng, n, dev)
        streamr = None
        if world == 1 and not args.no_stream:
            streamr = {"landmark": stream_run(dev_index, args.seed),
                       "sliding_10M": stream_run(dev_index, args.seed, window=10_000_000)}
        domr = None
        if world == 1 and not args.no_dominance:
            domr = dominance_run(dev, D, P, args.dom_n, args.seed, 2, 1)
        line = {
            "metric": "skyline tuples/sec + p50 query latency, 8D anti-corr, 1/2/4/8 MI355X",
            "value": value,
            "unit": "tuples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "p50_query_latency_ms": statistics.median(step_ms),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (reference anti-correlated formula, counter RNG, generated in HBM)",
            "config": {"workload": "C4: MR-Angle 8D anti-correlated, P=16, landmark-window query",
                       "tuples_per_gpu": n, "dims": D, "partitions": P, "algo": "mr-angle",
                       "dist": args.dist, "domain": [0, 1000], "compare_dtype": "f32 (values exact)",
                       "parallelism": f"shards{world}", "skyline_size": g},
            "roofline": {"bound": "hbm", "kernel": "k_filter", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "alg_bytes_per_unit": bytes_per_tuple, "units_per_launch": f_units / max(f_launch, 1),
                         "avg_launch_ms": avg_ms, "launches": f_launch},
            "phases_ms_last_step": phases,
            "counters_last_step": {"n": int(counters[0]), "candidates": int(counters[1]),
                                   "distinct_reps": int(counters[2]), "global_candidates": int(counters[3]),
                                   "output": int(counters[4]), "sfs_rounds": int(counters[5])},
            "cpu_baseline": cpu,
            "dominance_roofline": domr,
            "csv_ingest": csvr,
            "stream_c5": streamr,
            "sort_roofline": sortr,
        }
        print(json.dumps(line), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
