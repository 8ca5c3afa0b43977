"""A/B of the k_filter stream: the same 100M-tuple 8D stream under each partitioner
(MR-Dim / MR-Grid keys are a few VALU ops; MR-Angle carries the angle estimate), so
the difference isolates the key's VALU cost from the HBM stream."""
import os
import sys
import json
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flink-skyline-qos_amd"))
import torch  # noqa: E402
import skyline  # noqa: E402

n, D, P = int(os.environ.get("N", 100_000_000)), 8, 16
dev = torch.device("cuda", 0)
vals = torch.empty((n, D), dtype=torch.float64, device=dev)
ids = torch.empty(n, dtype=torch.int64, device=dev)
oi = torch.empty(n, dtype=torch.int64, device=dev)
oo = torch.empty(n, dtype=torch.int32, device=dev)
res = {}
for algo in ("mr-dim", "mr-grid", "mr-angle"):
    eng = skyline.SkylineEngine(D, P, algo, 1000.0, 0)
    if algo == "mr-dim":
        eng.synth_dev("anti_correlated", n, vals, ids, seed=1242)
    eng.query_dev(ids, vals, oi, oo, n)
    eng.sync()
    eng.profile(True)
    eng.profile_reset()
    for _ in range(3):
        eng.query_dev(ids, vals, oi, oo, n)
    eng.sync()
    ms, la, un = eng.kernel_time("filter")
    ph, cnt = eng.phases()
    res[algo] = {"filter_ms": ms / la, "GBps": n * 66 / (ms / la) / 1e6, "phases": ph}
    eng.profile(False)
    eng.close()
print(json.dumps(res))
