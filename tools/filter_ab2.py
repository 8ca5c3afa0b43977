"""Interleaved A/B of engine variants (environment knobs read per launch) in ONE
process on one synthetic 8D stream (box-to-box clock differences cancel):
VARIANTS="SKY_DOM_R=4;SKY_DOM_R=64,..." (';' between variants, ',' between the
variables of one), ALGO (default mr-angle), DIST, N.  Prints per variant the median
over REPS rounds of each kernel timer in KERNELS (default filter) and of the whole
query (host wall clock, synchronised)."""
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flink-skyline-qos_amd"))
import torch  # noqa: E402
import skyline  # noqa: E402

n, D, P = int(os.environ.get("N", 100_000_000)), 8, 16
algo = os.environ.get("ALGO", "mr-angle")
reps = int(os.environ.get("REPS", 5))
variants = [v for v in os.environ.get("VARIANTS", "").split(";") if v]
dev = torch.device("cuda", 0)
vals = torch.empty((n, D), dtype=torch.float64, device=dev)
ids = torch.empty(n, dtype=torch.int64, device=dev)
oi = torch.empty(n, dtype=torch.int64, device=dev)
oo = torch.empty(n, dtype=torch.int32, device=dev)
eng = skyline.SkylineEngine(D, P, algo, 1000.0, 0)
eng.synth_dev(os.environ.get("DIST", "anti_correlated"), n, vals, ids, seed=1242)
eng.query_dev(ids, vals, oi, oo, n)
eng.sync()
ref = oi[:10].clone()
kernels = os.environ.get("KERNELS", "filter").split(",")
times = {v: {k: [] for k in kernels + ["query"]} for v in variants}
for _ in range(reps):
    for v in variants:
        for kv in v.split(","):
            k, x = kv.split("=")
            os.environ[k] = x
        eng.profile(True)
        eng.profile_reset()
        t0 = time.perf_counter()
        for _ in range(2):
            g = eng.query_dev(ids, vals, oi, oo, n)
        eng.sync()
        times[v]["query"].append((time.perf_counter() - t0) * 500.0)
        for kn in kernels:
            ms, la, _ = eng.kernel_time(kn)
            times[v][kn].append(ms / max(la, 1) if kn == "filter" else ms / 2)
        eng.profile(False)
        for kv in v.split(","):
            os.environ.pop(kv.split("=")[0])
# the box's streaming reference: torch's own reduction over the same 6.4 GB
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
flat = vals.view(-1)
tsum = []
for _ in range(5):
    st.record()
    flat.sum()
    en.record()
    torch.cuda.synchronize()
    tsum.append(st.elapsed_time(en))
res = {v: {k: round(statistics.median(t), 4) for k, t in kt.items()} for v, kt in times.items()}
for v in res:
    if "filter" in res[v]:
        res[v]["filter_GBps"] = round(n * 66 / res[v]["filter"] / 1e6)
res["torch_sum_ref"] = {"ms_median": statistics.median(tsum), "GBps": n * D * 8 / statistics.median(tsum) / 1e6}
print(json.dumps(res, indent=1))
