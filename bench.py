#!/usr/bin/env python3
"""bench.py — skyline tuples/sec (+ p50 query latency) on MI355X.

Headline workload (BASELINE.json metric; config C4 on one GPU per rank): MR-Angle, 8D,
anti-correlated stream (the reference producer's formula, python/unified_producer.py:89-123,
counter RNG), P = 16 partitions, domain [0,1000], 100M tuples per rank generated in HBM.

A step = one query over the whole landmark window (every tuple of the rank's shard):
partition keys -> local skylines of the P partitions -> global merge -> stream-ordered
skyline ids, inputs already resident in HBM.  With N GPUs (one process per GPU, launched
by torch.distributed.run) every rank owns a shard; the ranks exchange their local
skylines' distinct vectors with one RCCL all-gather and each rank filters ITS OWN
vectors against the union (skyline/dist.py).  --scaling strong (default, as BASELINE states
C4: 100M tuples on 8 GPUs): 100M tuples in total, split over the ranks; --scaling weak: N x
100M tuples.  With N > 1 the other mode is measured as well ("<mode>_scaling_companion").

--config C1..C5 runs one BASELINE configuration as the headline line instead:
  C1 MR-Dim 2D uniform 1M P=8 | C2 MR-Grid 4D correlated 10M P=8 | C3 MR-Angle 4D anti 50M P=8
  C4 MR-Angle 8D anti 100M P=16 | C5 6D mixed continuous queries, MR-Angle P=8.
The default run (C4) also carries every other configuration as a sub-line under
"configs" (each with its own roofline and cpu_baseline), the end-to-end C4 rates with the
host->device transfer (rows, or CSV text) inside the timed region, and the companion
rooflines of the dominance, CSV-decode and sort kernels.

"roofline": the dominant kernel (k_filter, HBM-bound), HIP events on the stream it is
launched on.  "cpu_baseline": the C restatement of the reference operators (oracle/,
test infrastructure) on a bounded sample of the same stream, rank 0, N=1 only, with the
extrapolation to the full size from the committed sweep (tools/cpu_baseline_sweep.py).
"""
import argparse
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

METRIC = "skyline tuples/sec + p50 query latency, 8D anti-corr, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0   # MI355X spec (MI355X_MICROARCH.md: 8.0 TB/s spec, 6.29 measured copy)
PCIE_PEAK_GBS = 64.0    # PCIe 5.0 x16, one direction (the host link the ingest-inclusive rate crosses)
# VALU compare peaks: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz = 78.6 T 32-bit lane-ops/s; k_dom16
# compares packed u16 pairs (v_pk_sub_u16: 2 compares per lane-op) -> 157.3 T compares/s
VALU_PEAK_32 = 256 * 4 * 32 * 2.4e9
VALU_PEAK_PK16 = 2 * VALU_PEAK_32

CONFIGS = {
    "C1": dict(algo="mr-dim", dims=2, dist="uniform", tuples=1_000_000, partitions=8, cpu_sample=1_000_000,
               workload="C1: MR-Dim 2D independent (uniform), P=8 (Flink parallelism 4), landmark-window query"),
    "C2": dict(algo="mr-grid", dims=4, dist="correlated", tuples=10_000_000, partitions=8, cpu_sample=1_000_000,
               workload="C2: MR-Grid 4D correlated, P=8, landmark-window query"),
    "C3": dict(algo="mr-angle", dims=4, dist="anti_correlated", tuples=50_000_000, partitions=8, cpu_sample=100_000,
               workload="C3: MR-Angle 4D anti-correlated, P=8, landmark-window query"),
    "C4": dict(algo="mr-angle", dims=8, dist="anti_correlated", tuples=100_000_000, partitions=16, cpu_sample=60_000,
               workload="C4: MR-Angle 8D anti-correlated, P=16, landmark-window query"),
}
# the one published reference number for a configured workload: MR-Dim, 2D, 1M tuples,
# TotalTime 19,544 ms (python/graph_paper_figures.py:29; hardware unstated)
C1_PUBLISHED_MS = 19544.0


def host_cores():
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def filter_roofline(eng, D, kt=None):
    """k_filter over the timed launches: algorithmic bytes = the f64 row read once + the u16
    status word written (8D + 2 per tuple), / its HIP-event time."""
    f_ms, f_launch, f_units = kt if kt is not None else eng.kernel_time("filter")
    if not f_launch:
        return None
    bpt = D * 8 + 2
    avg_ms = f_ms / f_launch
    units = f_units / f_launch
    achieved = bpt * units / (avg_ms / 1e3) / 1e9
    return {"bound": "hbm", "kernel": "k_filter", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": None, "alg_bytes_per_unit": bpt,
            "units_per_launch": units, "avg_launch_ms": avg_ms, "launches": f_launch}


def traffic_for(n, D, dist_name):
    """HBM bytes per k_filter launch from the PMC passes (tools/gpu_pmc.sh: FETCH_SIZE and
    WRITE_SIZE in separate rocprofv3 runs, gfx950 correction), reported only when they were
    measured on THIS build (hash of k_filter's sources) and workload; else None."""
    tf = os.path.join(REPO, "profiles", "traffic_filter.json")
    try:
        sys.path.insert(0, os.path.join(REPO, "tools"))
        from src_hash import kernel_src_sha
        tj = json.load(open(tf))
        if (tj.get("n") == n and tj.get("dims") == D and tj.get("dist") == dist_name and
                tj.get("kernel_src_sha") == kernel_src_sha("k_filter")):
            return tj.get("hbm_bytes_per_launch")
    except Exception:
        pass
    return None


def sweep_alpha(cfg_name):
    """Exponent of t = a * N^alpha from the committed CPU sweep (None if absent)."""
    for f in ("r02_cpu_baseline_sweep.json",):
        p = os.path.join(REPO, "profiles", f)
        try:
            sw = json.load(open(p))
            fit = sw["configs"][cfg_name]["fit"]
            return max(float(v["alpha"]) for v in fit.values()), f
        except Exception:
            continue
    return None, None


def cpu_baseline(cfg_name, cfg, seed):
    """The reference operators restated in C (oracle/, test infrastructure: the checker and
    this baseline only): per-key BNL with 5000-tuple buffers, one thread per Flink subtask
    (keys round-robin over p = Flink parallelism = P/2 threads), then the single-threaded
    global BNL merge, on the first `sample` tuples of the same stream."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from conftest import Oracle
    orc = Oracle()
    n_s = cfg["cpu_sample"]
    D, P = cfg["dims"], cfg["partitions"]
    vals = orc.synth(_abi.DISTS[cfg["dist"]], D, n_s, seed=seed)
    ids = np.arange(n_s, dtype=np.int64)
    algo = cfg["algo"][3:]
    p = max(1, min(P // 2, host_cores()))
    t0 = time.perf_counter()
    g, _, _, _ = orc.query_bnl_mt(algo, vals, ids, P, p)
    dt = time.perf_counter() - t0
    t0 = time.perf_counter()
    g1, _, _, _ = orc.query_bnl(algo, vals, ids, P)
    dt1 = time.perf_counter() - t0
    assert sorted(g.tolist()) == sorted(g1.tolist())
    out = {"value": n_s / dt, "unit": "tuples/s", "cores": p, "kind": "port",
           "sample": f"first {n_s} tuples of the same {cfg['dist']} stream (seed {seed}); oracle/ C restatement of "
                     f"the reference operators: per-key BNL (buffer 5000) on {p} subtask threads, single-threaded "
                     f"global BNL: {dt:.2f} s, skyline {len(g)}",
           "single_thread": {"value": n_s / dt1, "cores": 1, "seconds": dt1}}
    N = cfg["tuples"]
    if n_s < N:
        alpha, src = sweep_alpha(cfg_name)
        if alpha is not None:
            t_full = dt * (N / n_s) ** alpha
            out["extrapolated_full"] = {"tuples": N, "seconds": t_full, "tuples_per_s": N / t_full,
                                        "alpha": alpha, "fit_source": "profiles/" + src,
                                        "note": "EXTRAPOLATION t(N) = t(sample) * (N/sample)^alpha, alpha fitted "
                                                "over the N-sweep; the reference BNL is quadratic in the "
                                                "duplicate all-zero tuples (SURVEY §3)"}
    return out


def make_stream(eng, dist_name, n, seed, id0, dev):
    vals = torch.empty((n, eng.dims), dtype=torch.float64, device=dev)
    ids = torch.empty(n, dtype=torch.int64, device=dev)
    eng.synth_dev(dist_name, n, vals, ids, seed=seed, id0=id0)
    eng.sync()
    return vals, ids


def time_steps(step, eng, steps, warmup, distributed):
    """W untimed steps, then K timed steps with the light kernel timers on (HIP events around
    the timed kernels only: the roofline), then one untimed step with the phase events on."""
    for _ in range(warmup):
        step()
    eng.sync()
    torch.cuda.synchronize()
    eng.profile(1)
    eng.profile_reset()
    step_ms = []
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g = 0
    for _ in range(steps):
        ts = time.perf_counter()
        g = step()
        eng.sync()
        step_ms.append((time.perf_counter() - ts) * 1e3)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kt = eng.kernel_time("filter")   # the timed launches only
    eng.profile(2)                   # phase split of one more (untimed) step
    step()
    eng.sync()
    eng.profile(False)
    return elapsed, step_ms, g, kt


def config_line(name, dev, dev_index, steps, warmup, with_cpu):
    """One BASELINE configuration on one GPU (sub-line of the default run, or --config)."""
    cfg = CONFIGS[name]
    D, P, n = cfg["dims"], cfg["partitions"], cfg["tuples"]
    seed = 1234 + D
    eng = skyline.SkylineEngine(D, P, cfg["algo"], 1000.0, dev_index)
    eng.use_torch_stream()
    vals, ids = make_stream(eng, cfg["dist"], n, seed, 0, dev)
    out_ids = torch.empty(n, dtype=torch.int64, device=dev)
    out_org = torch.empty(n, dtype=torch.int32, device=dev)
    step = lambda: eng.query_dev(ids, vals, out_ids, out_org, n)   # noqa: E731
    elapsed, step_ms, g, kt = time_steps(step, eng, steps, warmup, False)
    phases, counters = eng.phases()
    roof = filter_roofline(eng, D, kt)
    if roof:
        roof["traffic"] = traffic_for(n, D, cfg["dist"])
    # the same steps again with no profiler event in the stream: a HIP-event pair around k_filter
    # puts ~10 us of gap into a query whose kernels take tens of microseconds (C1, C2); the
    # roofline above comes from the timed steps with the events
    eng.sync()
    t0 = time.perf_counter()
    bare_ms = []
    for _ in range(max(steps, 20)):
        ts = time.perf_counter()
        step()
        eng.sync()
        bare_ms.append((time.perf_counter() - ts) * 1e3)
    bare_elapsed = time.perf_counter() - t0
    ms = bare_elapsed * 1e3 / len(bare_ms)
    ms_timed = elapsed * 1e3 / steps
    line = {"metric": METRIC, "value": n / (ms / 1e3), "unit": "tuples/s", "n_gpus": 1, "steps": len(bare_ms),
            "warmup": warmup, "ms_per_step": ms, "p50_query_latency_ms": statistics.median(bare_ms),
            "with_kernel_timers": {"steps": steps, "ms_per_step": ms_timed, "p50_query_latency_ms":
                                   statistics.median(step_ms), "note": "HIP events around k_filter in every "
                                   "step (the roofline's measurement)"},
            "dtype": "f64", "config": {"workload": cfg["workload"], "tuples": n, "dims": D, "partitions": P,
                                       "algo": cfg["algo"], "dist": cfg["dist"], "seed": seed, "skyline_size": g},
            "roofline": roof, "phases_ms_last_step": phases,
            "counters_last_step": {"candidates": int(counters[1]), "distinct_reps": int(counters[2]),
                                   "global_candidates": int(counters[3]), "output": int(counters[4])}}
    if name == "C1":
        ref_rate = 1e6 / (C1_PUBLISHED_MS / 1e3)
        line["vs_published"] = {"reference_total_ms": C1_PUBLISHED_MS, "reference_tuples_per_s": ref_rate,
                                "ratio": line["value"] / ref_rate,
                                "source": "python/graph_paper_figures.py:29 (MR-Dim 2D 1M TotalTime, includes "
                                          "Kafka ingest; hardware unstated)"}
    if with_cpu:
        line["cpu_baseline"] = cpu_baseline(name, cfg, seed)
    eng.close()
    del vals, ids, out_ids, out_org
    torch.cuda.empty_cache()
    return line


def end_to_end_c4(eng, vals, ids, n, D, steps, out_ids, out_org):
    """C4 with the host->device transfer inside the timed region (the reference's
    total_processing_time_ms spans first tuple to emission, FlinkSkyline.java:581-587):
    (a) f64 rows + i64 ids from pinned host memory -> HBM -> query;
    (b) the producers' CSV text (unified_producer.py:174) from pinned host memory -> HBM ->
        device CSV decode (k_csv.hip) -> query."""
    dev = vals.device
    h_vals = torch.empty(vals.shape, dtype=vals.dtype, pin_memory=True)
    h_ids = torch.empty(ids.shape, dtype=ids.dtype, pin_memory=True)
    h_vals.copy_(vals)
    h_ids.copy_(ids)
    d_vals = torch.empty_like(vals)
    d_ids = torch.empty_like(ids)
    res = {}

    def rows_step():
        d_vals.copy_(h_vals, non_blocking=True)
        d_ids.copy_(h_ids, non_blocking=True)
        return eng.query_dev(d_ids, d_vals, out_ids, out_org, n)

    for _ in range(1):
        rows_step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        g = rows_step()
    eng.sync()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    t1 = time.perf_counter()
    for _ in range(steps):
        d_vals.copy_(h_vals, non_blocking=True)
        d_ids.copy_(h_ids, non_blocking=True)
    torch.cuda.synchronize()
    h2d = (time.perf_counter() - t1) / steps
    byts = n * (8 * D + 8)
    res["rows_h2d"] = {"workload": f"C4, {n} f64 rows + i64 ids from pinned host memory, H2D + query per step",
                       "tuples_per_s": n / dt, "ms_per_step": dt * 1e3, "skyline_size": g,
                       "h2d_ms": h2d * 1e3, "h2d_GBs": byts / h2d / 1e9, "h2d_bytes": byts}
    del h_vals, h_ids
    nb = eng.format_csv_dev(ids, vals, n)
    text = torch.empty(nb, dtype=torch.uint8, device=dev)
    eng.format_csv_dev(ids, vals, n, text, nb)
    h_text = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
    h_text.copy_(text)

    def csv_step():
        text.copy_(h_text, non_blocking=True)
        eng.parse_csv_dev(text, nb, d_ids, d_vals, n)
        return eng.query_dev(d_ids, d_vals, out_ids, out_org, n)

    csv_step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        g = csv_step()
    eng.sync()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    res["csv_h2d"] = {"workload": f"C4 as producer CSV text ({nb} bytes) from pinned host memory: H2D + device "
                                  f"decode + query per step", "tuples_per_s": n / dt, "ms_per_step": dt * 1e3,
                      "skyline_size": g, "text_bytes": nb}
    del text, h_text, d_vals, d_ids
    torch.cuda.empty_cache()
    return res


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
    eng.profile(1)                        # light timers only (dom / mbr) inside the timed queries
    eng.profile_reset()
    t0 = time.perf_counter()
    g = 0
    for _ in range(steps):
        g = eng.query_dev(ids, vals, out_ids, out_org, n)
    eng.sync()
    dt = (time.perf_counter() - t0) / steps
    w = eng.dominance_work()
    dom16_ms, _, _ = eng.kernel_time("dom")
    mbr_ms, mbr_launches, _ = eng.kernel_time("mbr")
    eng.profile(2)                        # the phase split from one more (untimed) query
    eng.query_dev(ids, vals, out_ids, out_org, n)
    eng.sync()
    eng.profile(False)
    phases, counters = eng.phases()
    dom_ms = (dom16_ms + mbr_ms) / steps
    executed = int(counters[6])           # pair tests the last query executed (pruned pass) / upper bound (SFS)
    mbr = mbr_launches > 0
    achieved = D * executed / (dom_ms / 1e3) if dom_ms > 0 and mbr else D * w / (dom_ms / 1e3) if dom_ms > 0 else 0.0
    eng.close()
    return {"bound": "valu",
            "kernel": ("k_mbr_pairs (+ Morton key, sort, tiles: the whole bounding-box pruned pass), HIP events"
                       if mbr else "k_dom16 (+k_xcompact16), HIP events over every SFS round"),
            "workload": f"std_anti (labelled extension generator) {D}D, {n} tuples, MR-Angle P={P}",
            "tuples_per_s": n / dt, "ms_per_query": dt * 1e3, "skyline_size": g,
            "pair_tests_W": w, "compares_W": D * w, "pair_tests_executed": executed if mbr else None,
            "dominance_ms": dom_ms,
            "achieved": achieved, "peak": VALU_PEAK_PK16, "unit": "compares/s",
            "frac": achieved / VALU_PEAK_PK16,
            "achieved_note": ("compares the pruned pass executed (D x pair tests counted on the device) / its time"
                              if mbr else "D x W (algorithmic SFS pair tests over distinct vectors) / SFS time"),
            "W_rate": D * w / (dom_ms / 1e3) if dom_ms > 0 else None,
            "frac_W": (D * w / (dom_ms / 1e3)) / VALU_PEAK_PK16 if dom_ms > 0 else None,
            "W_rate_note": ("D x W / time with W = SURVEY §8d's algorithmic pair count (the quadratic SFS/BNL over "
                            "distinct vectors): the compare rate a pair-by-pair algorithm would need to finish in "
                            "this time; above the VALU peak because the bounding-box pass skips most pairs"),
            "peak_note": "packed-u16 compare peak (2 compares per v_pk_sub_u16 lane-op); the 32-bit lane-op "
                         "peak is half of it",
            "peak_32bit": VALU_PEAK_32, "frac_32bit": achieved / VALU_PEAK_32,
            "path": ("mbr-" if mbr else "sfs-") + ("u16" if int(counters[7]) & 4 else "f32/f64"),
            "local_sfs_ms": phases["local_sfs"], "global_sfs_ms": phases["global_sfs"],
            "sfs_rounds": int(counters[5]),
            "tile_pairs_tested": int(counters[7]) >> 8 if mbr else None}


def dominance_dense_run(dev, D, P, n, seed, steps=3):
    """The dense all-pairs dominance kernel alone (sky_profile_pairs_dev: k_brute16_pairs, the
    small-set route's pair pass, every row against every row -- the pairs of the BNL loops
    FlinkSkyline.java:424-441 without any pruning) on n rows of the labelled std-anti generator
    with their MR-Angle keys: D x n^2 compares / the kernel's HIP-event time, against the
    packed-u16 compare peak.  n = 16384 is the brute route's slot ceiling."""
    eng = skyline.SkylineEngine(D, P, "mr-angle", 1000.0, dev.index or 0)
    vals = torch.empty((n, D), dtype=torch.float64, device=dev)
    ids = torch.empty(n, dtype=torch.int64, device=dev)
    eng.synth_dev("std_anti", n, vals, ids, seed=seed)
    keys = torch.empty(n, dtype=torch.int32, device=dev)
    eng.partition_keys_dev(vals, keys)
    fates = torch.empty(n, dtype=torch.int32, device=dev)
    eng.profile_pairs_dev(vals, keys, fates)              # warm-up
    ms = []
    kind = 0
    for _ in range(steps):
        kind, t = eng.profile_pairs_dev(vals, keys, fates)
        ms.append(t)
    eng.sync()
    in_g = int(((fates & 2) == 0).sum().item())
    eng.close()
    t = statistics.median(ms)
    pairs = n * n
    achieved = D * pairs / (t / 1e3)
    return {"bound": "valu", "kernel": "k_brute16_pairs (dense all-pairs, packed u16, HIP events)"
            if kind == 0 else "k_brute_pairs (f32/f64)",
            "workload": f"std_anti {D}D, {n} rows, MR-Angle P={P} keys, every row against every row",
            "pair_tests": pairs, "compares": D * pairs, "kernel_ms": t, "achieved": achieved,
            "peak": VALU_PEAK_PK16, "unit": "compares/s", "frac": achieved / VALU_PEAK_PK16,
            "peak_32bit": VALU_PEAK_32, "frac_32bit": achieved / VALU_PEAK_32,
            "rows_not_dominated": in_g,
            "peak_note": "packed-u16 compare peak: 2 compares per v_pk_sub_u16 lane-op at 128 lanes/clk/CU; "
                         "the kernel issues 4 v_pk_sub_u16 + 1 v_sub_u32 + 2 v_or3 + 1 v_min (+2 v_mov per 4 "
                         "rows) per 8D pair test, so issue-bound it tops out near 8/8.5/2 = 0.47 of it"}


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
    eng.profile(1)                                          # light timers only (csv_*)
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
    achieved = alg / (p_ms / 1e3) / 1e9
    return {"bound": "hbm", "kernel": "k_csv_fields (+ k_csv_nl_count, its scan, k_csv_group_pos)",
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
    D, P = 6, 8
    n = triggers * per_trigger
    vals_np, ids_np = skyline.synth_host(_abi.DISTS["mixed"], D, n, seed=seed)
    vals = torch.from_numpy(vals_np).pin_memory().numpy()
    ids = torch.from_numpy(ids_np).pin_memory().numpy()
    eng = skyline.SkylineEngine(D, P, "mr-angle", 1000.0, dev_index)
    if not os.environ.get("BENCH_OWN_STREAM"):   # (A/B: the library on its own stream)
        eng.use_torch_stream()
    eng.warmup()                                  # first launches / allocations, before the stream starts

    def run_stream(timers):
        st = skyline.SkylineStream(eng, window)
        st.reserve(window if window else n)      # result buffers pinned once, before the stream starts
        lat_int, lat_ids, copy_ms, sizes = [], [], [], []
        eng.profile(1 if timers else 0)          # light timers only (the k_filter roofline)
        eng.profile_reset()
        t_start = time.perf_counter()
        for t in range(triggers):
            base = t * per_trigger
            for b0 in range(base, base + per_trigger, batch):
                st.append(ids[b0:b0 + batch], vals[b0:b0 + batch])
                if b0 == base and t:
                    # the last trigger's ids reached host memory while this micro-batch went in
                    cm = st.wait()
                    copy_ms.append(cm)
                    lat_ids.append(lat_int[-1] + cm)
            tq = time.perf_counter()
            g = st.query_async_host_view()        # returns with the integers (skyline size, stats)
            lat_int.append((time.perf_counter() - tq) * 1e3)
            sizes.append(g)
        cm = st.wait()
        copy_ms.append(cm)
        lat_ids.append(lat_int[-1] + cm)
        total = time.perf_counter() - t_start
        eng.profile(False)
        resident, _ = st.size()
        vectors = st.vectors()
        st.close()
        return lat_int, lat_ids, copy_ms, sizes, total, resident, vectors

    # the stream as measured: no profiler event in it (an event pair around k_filter adds ~10 us
    # to a trigger of ~0.3 ms); then the same stream again with the light timers, for the roofline
    lat_int, lat_ids, copy_ms, sizes, total, resident, vectors = run_stream(False)
    t_lat = run_stream(True)[0]
    roof = filter_roofline(eng, D)
    eng.close()
    rate = n / total
    lat = lat_ids
    return {"workload": (f"C5: 6D mixed stream, MR-Angle P={P}, {batch}-tuple micro-batches from pinned host "
                         f"memory, query_trigger every {per_trigger} tuples, {triggers} triggers, "
                         + ("landmark window (reference semantics)" if window == 0
                            else f"count-based sliding window W={window} (extension)")),
            "ingest_tuples_per_s": rate, "sustains_10M_per_s": rate >= 1e7,
            "latency_note": ("p50_query_latency_ms = trigger -> the reference's result integers (skyline_size, "
                             "|L_k|, survivors_k: FlinkSkyline.java:593-608) on the host "
                             "(sky_stream_query_async returns); ids_* = trigger -> every skyline id + origin in "
                             "host memory = the integers' latency + the D2H copy's device time, the copy "
                             "overlapping the next micro-batch's append"),
            "p50_query_latency_ms": statistics.median(lat_int),
            "p90_query_latency_ms": sorted(lat_int)[int(0.9 * len(lat_int))],
            "max_query_latency_ms": max(lat_int), "latencies_ms": [round(x, 3) for x in lat_int],
            "ids_p50_latency_ms": statistics.median(lat), "ids_p90_latency_ms": sorted(lat)[int(0.9 * len(lat))],
            "ids_max_latency_ms": max(lat), "ids_latencies_ms": [round(x, 3) for x in lat],
            "copy_ms": [round(x, 3) for x in copy_ms],
            "with_kernel_timers_p50_query_latency_ms": statistics.median(t_lat),
            "skyline_size_last": sizes[-1], "resident_tuples_last": resident,
            "resident_vectors_last": vectors,
            "resident_note": ("landmark: the local-skyline tuples kept (ids, arrival order) and the distinct "
                              "vectors the next query runs over" if window == 0 else "the window's tuples"),
            "roofline": roof}


def operator_run(dev_index, n=10_000_000, buf=5000, micro=80_000):
    """The drop-in operator path (FlinkSkyline.java:265-316, :417-444,
    :515-569) on the first n tuples of the C4 stream, from host memory as the JNI shim passes
    it.  Tuples are routed to per-key 5000-tuple buffers in stream order; after every micro-batch
    of `micro` tuples (Kafka poll granularity) the keys whose buffers are full are flushed in ONE
    sky_parts_insert call (asynchronous: no host read).  At the trigger: the partial buffers are
    flushed, every key's snapshot taken (the one synchronisation), and sky_global_merge run over
    the P local skylines.  Reported: tuples/s end to end, per-call latency (p50 / p99, host time
    of one sky_parts_insert), and the same stream with one sky_part_insert per full buffer."""
    import numpy as np
    from skyline.operators import _LocalPart
    D, P = 8, 16
    vals, ids = skyline.synth_host(_abi.DISTS["anti_correlated"], D, n, seed=1234 + D)
    eng = skyline.SkylineEngine(D, P, "mr-angle", 1000.0, dev_index)
    eng.warmup()
    keys = eng.partition_keys(vals)
    order = np.argsort(keys, kind="stable")
    starts = np.searchsorted(keys[order], np.arange(P + 1))
    per_key = {k: order[starts[k]:starts[k + 1]] for k in range(P)}    # stream order within a key
    batches = {k: (np.ascontiguousarray(ids[per_key[k]]), np.ascontiguousarray(vals[per_key[k]])) for k in range(P)}
    # the flush schedule: after micro-batch m, the buffers that filled up during it, one call per
    # round (a key whose buffer filled r times in the micro-batch appears in the first r calls)
    sched = []
    done = {k: 0 for k in range(P)}
    for m0 in range(0, n, micro):
        lim = m0 + micro
        full = {}
        for k in range(P):
            nfull = int(np.searchsorted(per_key[k], lim)) // buf
            full[k] = list(range(done[k], nfull))
            done[k] = nfull
        for r in range(max(len(v) for v in full.values())):
            call = [(k, f[r] * buf, (f[r] + 1) * buf) for k, f in full.items() if r < len(f)]
            if call:
                sched.append(call)

    import ctypes
    from skyline._abi import check, lib

    def run(batched, device_merge=True):
        parts = {k: _LocalPart(eng, k) for k in range(P)}
        lat = []
        # the calls' argument arrays (part handles, pointers into the per-key buffers, counts) are
        # what the JNI shim receives from the operator directly: built before the timed loop, so
        # that the loop times the library calls, not Python list building
        args = []
        if batched:
            for call in sched:
                nc = len(call)
                ph = (ctypes.c_void_p * nc)(*[parts[k].h.value for k, _, _ in call])
                ip = (ctypes.c_void_p * nc)(*[batches[k][0].ctypes.data + lo * 8 for k, lo, _ in call])
                vp = (ctypes.c_void_p * nc)(*[batches[k][1].ctypes.data + lo * D * 8 for k, lo, _ in call])
                cn = (ctypes.c_int64 * nc)(*[hi - lo for _, lo, hi in call])
                args.append((nc, ph, ip, vp, cn))
        f_ins = lib().sky_parts_insert
        t0 = time.perf_counter()
        for ci, call in enumerate(sched):
            ts = time.perf_counter()
            if batched:
                check(f_ins(*args[ci]))
            else:
                for k, lo, hi in call:
                    parts[k].insert(batches[k][0][lo:hi], batches[k][1][lo:hi])
            lat.append((time.perf_counter() - ts) * 1e3)
        t_ins = time.perf_counter() - t0
        tq = time.perf_counter()
        rest = [k for k in range(P) if len(batches[k][0]) % buf]
        _LocalPart.insert_many([parts[k] for k in rest],
                               [(batches[k][0][done[k] * buf:], batches[k][1][done[k] * buf:]) for k in rest])
        if device_merge:
            # co-located aggregator: the local skylines never leave the device
            gids, _ = _LocalPart.global_merge_many(eng, [parts[k] for k in range(P)], list(range(P)))
            local_sizes = [int(x) for x in eng.stats()[0]]
        else:
            snaps = [parts[k].snapshot() for k in range(P)]     # processQuery: the one synchronisation
            gids, _ = eng.global_merge(list(range(P)), [sn[0] for sn in snaps], [sn[1] for sn in snaps])
            local_sizes = [len(sn[0]) for sn in snaps]
        t_q = time.perf_counter() - tq
        total = time.perf_counter() - t0
        for pt in parts.values():
            pt.close()
        lat.sort()
        nflush = sum(len(cl) for cl in sched)
        return {"calls": len(lat), "flushes": nflush, "insert_phase_s": t_ins, "query_phase_s": t_q,
                "tuples_per_s": n / total, "ingest_tuples_per_s": (nflush * buf) / t_ins if t_ins else None,
                "p50_call_ms": lat[len(lat) // 2] if lat else None,
                "p99_call_ms": lat[min(len(lat) - 1, int(len(lat) * 0.99))] if lat else None,
                "max_call_ms": lat[-1] if lat else None,
                "skyline_size": int(len(gids)), "local_sizes": local_sizes, "skyline_ids": gids}

    # ---- the Java operators' exact call sequence (HipSkylineOperators, java/org/main): full buffers
    #      in arrival order wait until FLUSH_GROUP = 8 are pending, then drainFull issues rounds (the
    #      first waiting buffer of every key, one sky_parts_insert per round); the trigger: per key
    #      drainFull + the partial buffer's sky_part_insert + sky_part_sizes + sky_part_snapshot_reps
    #      (the LocalSkyline message), then sky_global_merge_reps over the P messages
    done_pos = []
    for k in range(P):
        for j in range(len(per_key[k]) // buf):
            done_pos.append((int(per_key[k][(j + 1) * buf - 1]), k, j))
    done_pos.sort()
    jsched, fifo = [], []

    def drain():
        nonlocal fifo
        while fifo:
            seen, rnd, later = set(), [], []
            for kj in fifo:
                (later if kj[0] in seen else rnd).append(kj)
                seen.add(kj[0])
            jsched.append(rnd)
            fifo = later
    for _, k, j in done_pos:
        fifo.append((k, j))
        if len(fifo) >= 8:
            drain()
    drain()

    def java_sequence():
        parts = {k: _LocalPart(eng, k) for k in range(P)}
        args = []
        for rnd in jsched:
            nc = len(rnd)
            args.append((nc, (ctypes.c_void_p * nc)(*[parts[k].h.value for k, _ in rnd]),
                         (ctypes.c_void_p * nc)(*[batches[k][0].ctypes.data + j * buf * 8 for k, j in rnd]),
                         (ctypes.c_void_p * nc)(*[batches[k][1].ctypes.data + j * buf * D * 8 for k, j in rnd]),
                         (ctypes.c_int64 * nc)(*([buf] * nc))))
        f_ins = lib().sky_parts_insert
        lat = []
        t0 = time.perf_counter()
        for a in args:
            ts = time.perf_counter()
            check(f_ins(*a))
            lat.append((time.perf_counter() - ts) * 1e3)
        t_ins = time.perf_counter() - t0
        tq = time.perf_counter()
        msgs = []
        for k in range(P):                       # processQuery on every key (the trigger's broadcast)
            nf = len(per_key[k]) // buf
            if len(per_key[k]) > nf * buf:
                parts[k].insert(batches[k][0][nf * buf:], batches[k][1][nf * buf:])
            m = parts[k].snapshot_reps()
            msgs.append((m.ids, m.rep_idx, m.reps, m.rep_counts))
        t_snap = time.perf_counter() - tq
        gids, _ = eng.global_merge_reps(list(range(P)), msgs)   # GlobalAggregator, last arrival
        t_q = time.perf_counter() - tq
        total = time.perf_counter() - t0
        for pt in parts.values():
            pt.close()
        lat.sort()
        return {"calls": len(lat), "flushes": sum(len(r) for r in jsched), "insert_phase_s": t_ins,
                "query_phase_s": t_q, "snapshot_s": t_snap, "merge_s": t_q - t_snap, "tuples_per_s": n / total,
                "p50_call_ms": lat[len(lat) // 2] if lat else None,
                "p99_call_ms": lat[min(len(lat) - 1, int(len(lat) * 0.99))] if lat else None,
                "message_bytes": int(sum(m[0].nbytes + m[1].nbytes + m[2].nbytes + m[3].nbytes for m in msgs)),
                "message_tuples": int(sum(len(m[0]) for m in msgs)), "message_vectors": int(sum(len(m[2]) for m in msgs)),
                "skyline_size": int(len(gids)), "skyline_ids": gids}

    run(True)                                          # first launches / allocations
    b = run(True)
    s1 = run(False, device_merge=False)
    java_sequence()
    js = java_sequence()
    exp = eng.query(vals, ids)[0]
    exact = bool(np.array_equal(np.sort(b.pop("skyline_ids")), exp) and
                 np.array_equal(np.sort(s1.pop("skyline_ids")), exp) and
                 np.array_equal(np.sort(js.pop("skyline_ids")), exp))
    eng.close()
    return {"workload": f"C4 stream prefix, {n} tuples, MR-Angle P={P}, per-key {buf}-tuple buffers from host memory; "
                        f"the full buffers flushed after every {micro}-tuple micro-batch in one sky_parts_insert "
                        f"call, then the co-located global merge of the device-resident states "
                        f"(sky_parts_global_merge); 'one_call_per_buffer': one sky_part_insert per buffer, then "
                        f"snapshots through host memory + sky_global_merge",
            "java_sequence_workload": "the Java operators' calls exactly (HipSkylineOperators): drainFull rounds of "
                                      "sky_parts_insert every 8 full buffers, per key sky_part_sizes + "
                                      "sky_part_snapshot_reps at the trigger, sky_global_merge_reps",
            "exact_vs_whole_stream_query": exact, "batched": b, "one_call_per_buffer": s1, "java_sequence": js,
            "tuples_per_s": b["tuples_per_s"], "p50_call_ms": b["p50_call_ms"], "p99_call_ms": b["p99_call_ms"]}


def sort_run(eng, n, dev, steps=3):
    """Sort phase at scale (HBM GB/s of the sort): the pipeline's radix sort
    (k_radix.hip) alone on n pairs keyed like its candidate keys (4-bit partition | 32-bit
    score | 16-bit hash, 52 varying bits).  Algorithmic bytes = passes x n x 24 (read +
    write a u64 key and a u32 value per pass)."""
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    part = torch.randint(0, 16, (n,), device=dev, dtype=torch.int64, generator=g)
    score = torch.randint(0, 1 << 32, (n,), device=dev, dtype=torch.int64, generator=g)
    hsh = torch.randint(0, 1 << 16, (n,), device=dev, dtype=torch.int64, generator=g)
    keys0 = (part << 56) | (score << 24) | hsh
    del part, score, hsh
    vals0 = torch.arange(n, device=dev, dtype=torch.int32)
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
            "workload": f"{n} (u64 key, u32 value) pairs, 4-bit partition | 32-bit score | 16-bit hash",
            "passes": passes, "ms": best, "keys_per_s": n / (best / 1e3), "alg_bytes": alg,
            "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS}


def spawn_ranks(n):
    """`bench.py --gpus N` (N > 1) run directly: start N rank processes through
    torch.distributed.run as a CHILD process (this parent never initialises the GPU and never
    exec()s) with the same arguments, and return its exit status.  Rank 0 prints the line."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C4", choices=["C1", "C2", "C3", "C4", "C5"])
    ap.add_argument("--scaling", default="strong", choices=["weak", "strong"],
                    help="strong (default: BASELINE states each configuration's tuples in total, e.g. C4 = "
                         "100M tuples on 8 GPUs): --tuples in total, split over the ranks; weak: --tuples per "
                         "rank.  With N > 1 the other one is measured too, as a labelled companion key")
    ap.add_argument("--no-companion-scaling", action="store_true",
                    help="N > 1: skip the companion measurement of the other scaling mode")
    ap.add_argument("--tuples", type=int, default=None, help="override the config's tuple count")
    ap.add_argument("--dist", default=None, help="override the config's distribution (e.g. std_anti)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dom-n", type=int, default=2_000_000, help="tuples of the dominance-bound companion run")
    ap.add_argument("--dom-n-large", type=int, default=10_000_000,
                    help="tuples of the second dominance-bound companion run (0: skip)")
    ap.add_argument("--dom-n-huge", type=int, default=100_000_000,
                    help="tuples of the north_star-size dominance run (std-anti 8D; 0: skip)")
    ap.add_argument("--no-dominance", action="store_true")
    ap.add_argument("--no-csv", action="store_true", help="skip the CSV-ingest companion measurement")
    ap.add_argument("--no-stream", action="store_true", help="skip the C5 continuous-query companion measurement")
    ap.add_argument("--no-sort", action="store_true", help="skip the radix-sort-at-scale companion measurement")
    ap.add_argument("--no-configs", action="store_true", help="skip the C1/C2/C3 sub-lines")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (H2D inside) C4 rates")
    ap.add_argument("--no-operator", action="store_true", help="skip the per-key operator-path companion")
    ap.add_argument("--dist-backend", default="auto", choices=["auto", "nccl", "gloo"],
                    help="nccl (= RCCL over xGMI, the measured path), gloo (rehearsing several ranks on one "
                         "GPU), auto: nccl when every rank has a GPU of its own")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: start the ranks from here, before anything touches the GPU
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"WORLD_SIZE={world} but --gpus {args.gpus}: launch one rank per GPU")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    n_dev = max(torch.cuda.device_count(), 1)
    backend = args.dist_backend
    if backend == "auto":
        backend = "nccl" if n_dev >= world else "gloo"
    dev_index = local_rank % n_dev   # > 1 rank per GPU only when rehearsing with gloo
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    # one non-default stream for everything this process issues; the engines run ON it
    # (use_torch_stream: no cross-stream events per call), and the collectives order after it
    torch.cuda.set_stream(torch.cuda.Stream(device=dev))
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    red_dev = dev if backend == "nccl" else torch.device("cpu")

    if args.config == "C5":
        if rank == 0:
            lm = stream_run(dev_index, 1234 + 6)
            sl = stream_run(dev_index, 1234 + 6, window=10_000_000)
            line = {"metric": METRIC, "value": lm["ingest_tuples_per_s"], "unit": "tuples/s", "n_gpus": 1,
                    "steps": 20, "warmup": 0, "ms_per_step": lm["p50_query_latency_ms"],
                    "p50_query_latency_ms": lm["p50_query_latency_ms"], "higher_is_better": True,
                    "scaling": "weak", "vs_baseline": None, "dtype": "f64",
                    "data": "synthetic (6D mixed blocks of the reference formulas)",
                    "config": {"workload": lm["workload"]}, "roofline": lm["roofline"],
                    "cpu_baseline": None, "landmark": lm, "sliding_10M": sl}
            print(json.dumps(line), flush=True)
        if distributed:
            dist.barrier()
            dist.destroy_process_group()
        return

    cfg = dict(CONFIGS[args.config])
    if args.dist:
        cfg["dist"] = args.dist
    D, P = cfg["dims"], cfg["partitions"]
    n_cfg = args.tuples or cfg["tuples"]
    seed = 1234 + D
    eng = skyline.SkylineEngine(D, P, cfg["algo"], 1000.0, dev_index)
    eng.use_torch_stream()

    def shard(mode):
        """(tuples on this rank, first id, tuples in the whole job) of a scaling mode."""
        if mode == "strong":
            lo, hi = rank * n_cfg // world, (rank + 1) * n_cfg // world
            return hi - lo, lo, n_cfg
        return n_cfg, rank * n_cfg, n_cfg * world

    def measure(mode):
        """W + K steps of one scaling mode; every rank's elapsed / p50 reduced by MAX."""
        n, id0, total = shard(mode)
        vals, ids = make_stream(eng, cfg["dist"], n, seed, id0, dev)
        out_ids = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        out_org = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        dist_phase_log = []

        def step():
            if distributed:
                g = distributed_query(eng, ids, vals, out_ids, out_org, n)
                dist_phase_log.append(eng.last_dist_phases)     # export / all-gather / merge / finish split
                return g
            return eng.query_dev(ids, vals, out_ids, out_org, n)

        elapsed, step_ms, g, kt = time_steps(step, eng, args.steps, args.warmup, distributed)
        p50 = statistics.median(step_ms)
        if distributed:
            t = torch.tensor([elapsed, p50], dtype=torch.float64, device=red_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed, p50 = float(t[0].item()), float(t[1].item())
            gt = torch.tensor([g], dtype=torch.int64, device=red_dev)
            dist.all_reduce(gt)
            g = int(gt.item())
        dist_stats = getattr(eng, "last_dist_stats", None) if distributed else None
        if dist_stats is not None:
            # the timed steps' phase split (warm-up steps come first, the profiled step last), with
            # the own-vs-union pass's kernel time on its own (union_pass_kernel_ms)
            dist_stats = dict(dist_stats, phases_per_step=dist_phase_log[args.warmup:args.warmup + args.steps])
        return dict(n=n, total=total, elapsed=elapsed, step_ms=step_ms, p50=p50, g=g, kt=kt, dist_stats=dist_stats,
                    vals=vals, ids=ids, out_ids=out_ids, out_org=out_org)

    companion = None
    if distributed and not args.no_companion_scaling:
        other = "weak" if args.scaling == "strong" else "strong"
        c = measure(other)
        ms_c = c["elapsed"] * 1e3 / args.steps
        companion = {"scaling": other, "value": c["total"] / (ms_c / 1e3), "unit": "tuples/s",
                     "ms_per_step": ms_c, "p50_query_latency_ms": c["p50"], "tuples_per_gpu": c["n"],
                     "tuples_total": c["total"], "skyline_size": c["g"], "dist_exchange": c["dist_stats"]}
        del c
        torch.cuda.empty_cache()
    m = measure(args.scaling)
    n, total, elapsed, step_ms, p50, g, kt = (m[k] for k in ("n", "total", "elapsed", "step_ms", "p50", "g", "kt"))
    vals, ids, out_ids, out_org = m["vals"], m["ids"], m["out_ids"], m["out_org"]
    dist_stats = m["dist_stats"]
    phases, counters = eng.phases()
    roof = filter_roofline(eng, D, kt)

    if rank == 0:
        ms_per_step = elapsed * 1e3 / args.steps
        value = total / (ms_per_step / 1e3)
        if roof:
            roof["traffic"] = traffic_for(n, D, cfg["dist"])
        solo = world == 1
        cpu = None
        if solo and not args.no_cpu_baseline:
            c = dict(cfg)
            c["tuples"] = n_cfg
            cpu = cpu_baseline(args.config, c, seed)
        extra = {}
        if solo and args.config == "C4" and n_cfg == CONFIGS["C4"]["tuples"] and not args.dist:
            if not args.no_e2e:
                extra["end_to_end"] = end_to_end_c4(eng, vals, ids, n, D, 3, out_ids, out_org)
            if not args.no_csv:
                extra["csv_ingest"] = csv_ingest_run(eng, ids, vals, n, D, 3, out_ids, out_org)
            if not args.no_sort:
                extra["sort_roofline"] = sort_run(eng, n, dev)
            if not args.no_operator:
                extra["operator_path"] = operator_run(dev_index)
            if not args.no_configs:
                extra["configs"] = {nm: config_line(nm, dev, dev_index, args.steps, args.warmup,
                                                    not args.no_cpu_baseline)
                                    for nm in ("C1", "C2", "C3")}
                if not args.no_stream:
                    extra["configs"]["C5"] = {"landmark": stream_run(dev_index, 1234 + 6),
                                              "sliding_10M": stream_run(dev_index, 1234 + 6, window=10_000_000)}
            if not args.no_dominance:
                extra["dominance_roofline"] = dominance_run(dev, D, P, args.dom_n, seed, 3, 2)
                if args.dom_n_large:
                    extra["dominance_roofline_large"] = dominance_run(dev, D, P, args.dom_n_large, seed, 3, 2)
                extra["dominance_dense_roofline"] = dominance_dense_run(dev, D, P, 16384, seed)
                extra["dominance_dense_roofline_64k"] = dominance_dense_run(dev, D, P, 65536, seed)
                if args.dom_n_huge:
                    # north_star's size: the std-anti 8D stream at 100M tuples through the whole query
                    extra[f"dominance_roofline_{args.dom_n_huge // 1_000_000}M"] = dominance_run(
                        dev, D, P, args.dom_n_huge, seed, 1, 1)
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "tuples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "p50_query_latency_ms": p50,
            "step_ms": [round(x, 3) for x in step_ms],
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (reference generator formulas, counter RNG, generated in HBM)",
            "config": {"workload": cfg["workload"], "tuples_per_gpu": n, "tuples_total": total, "dims": D,
                       "partitions": P, "algo": cfg["algo"], "dist": cfg["dist"], "domain": [0, 1000],
                       "seed": seed, "compare_dtype": "f32 / packed u16 when the values are exact",
                       "parallelism": f"shards{world}", "skyline_size": g,
                       "transport": (None if world == 1 else
                                     "RCCL over xGMI (nccl)" if backend == "nccl" else
                                     f"gloo rehearsal: {world} ranks on {min(n_dev, world)} GPU(s)")},
            "roofline": roof,
            "phases_ms_last_step": phases,
            "counters_last_step": {"n": int(counters[0]), "candidates": int(counters[1]),
                                   "distinct_reps": int(counters[2]), "global_candidates": int(counters[3]),
                                   "output": int(counters[4]), "sfs_rounds": int(counters[5])},
            "dist_exchange": dist_stats,
            "cpu_baseline": cpu,
        }
        if companion is not None:
            line[f"{companion['scaling']}_scaling_companion"] = companion
        e2e = extra.get("end_to_end")
        if e2e:
            # tuples INGESTED and reflected per second -- with the host->device copy inside
            # the step (never `value`, which is the HBM-resident re-query rate); bound: PCIe 5.0 x16
            rh = e2e["rows_h2d"]
            line["value_end_to_end"] = {
                "value": rh["tuples_per_s"], "unit": "tuples/s", "bound": "pcie",
                "workload": rh["workload"], "ms_per_step": rh["ms_per_step"],
                "h2d_GBs": rh["h2d_GBs"], "peak_GBs": PCIE_PEAK_GBS, "frac_of_pcie": rh["h2d_GBs"] / PCIE_PEAK_GBS,
                "csv_text_tuples_per_s": e2e["csv_h2d"]["tuples_per_s"]}
        line.update(extra)
        print(json.dumps(line), flush=True)
    eng.close()
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
