"""Box calibration: achievable HBM stream rates on this GPU (torch kernels), to read the
k_filter time against what the box itself sustains (boxes of the pool differ)."""
import json
import torch

dev = torch.device("cuda", 0)
n = 800_000_000                       # 6.4 GB of f64, the C4 row bytes
x = torch.ones(n, dtype=torch.float64, device=dev)
y = torch.empty_like(x)
res = {}
for name, fn, nbytes in (("read_sum", lambda: x.sum(), 8 * n), ("copy", lambda: y.copy_(x), 16 * n)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    res[name] = {"ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1)}
print(json.dumps(res))
