import sys; sys.path.insert(0, "flink-skyline-qos_amd")
import torch, skyline
dev = torch.device("cuda", 0)
n = 10_000_000
g = torch.Generator(device=dev); g.manual_seed(7)
part = torch.randint(0, 16, (n,), device=dev, dtype=torch.int64, generator=g)
score = torch.randint(0, 1 << 32, (n,), device=dev, dtype=torch.int64, generator=g)
hsh = torch.randint(0, 1 << 16, (n,), device=dev, dtype=torch.int64, generator=g)
keys0 = (part << 56) | (score << 24) | hsh
var = [b for b in range(64) if bool(((keys0 >> b) & 1).any()) and not bool(((keys0 >> b) & 1).all())]
print("varying bits", len(var), var[:5], var[-5:])
eng = skyline.SkylineEngine(8, 16, "mr-angle", 1000.0, 0)
for m in (n, 100_000_000):
    if m != n:
        part = torch.randint(0, 16, (m,), device=dev, dtype=torch.int64, generator=g)
        score = torch.randint(0, 1 << 32, (m,), device=dev, dtype=torch.int64, generator=g)
        hsh = torch.randint(0, 1 << 16, (m,), device=dev, dtype=torch.int64, generator=g)
        keys0 = (part << 56) | (score << 24) | hsh
    k = keys0.clone(); v = torch.arange(m, device=dev, dtype=torch.int32)
    print(m, eng.profile_sort_dev(k, v))
