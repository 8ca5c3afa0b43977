"""A/B timing of the CSV decoder on the C4 stream formatted as producer CSV (tools only)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "flink-skyline-qos_amd"))
import torch
import skyline
n, D = int(os.environ.get("N", "100000000")), 8
eng = skyline.SkylineEngine(D, 16, "mr-angle", 1000.0, 0)
vals = torch.empty((n, D), dtype=torch.float64, device="cuda")
ids = torch.empty(n, dtype=torch.int64, device="cuda")
eng.synth_dev(os.environ.get("DIST", "anti_correlated"), n, vals, ids, seed=1242)
nb = eng.format_csv_dev(ids, vals, n)
text = torch.empty(nb, dtype=torch.uint8, device="cuda")
eng.format_csv_dev(ids, vals, n, text, nb)
pi = torch.empty_like(ids); pv = torch.empty_like(vals)
for mode in os.environ.get("MODES", "0,1,2,3,0").split(","):
    os.environ["SKY_CSV_STOP"] = mode
    _, cnt = eng.parse_csv_dev(text, nb, pi, pv, n)
    print(f"stop={mode} counts {list(cnt)}", flush=True)
    eng.profile(True); eng.profile_reset()
    for _ in range(3):
        eng.parse_csv_dev(text, nb, pi, pv, n)
    eng.sync()
    ms, la, _ = eng.kernel_time("csv_parse")
    eng.profile(False)
    print(f"stop={mode} parse {ms/la:.3f} ms  ({nb/(ms/la)/1e6:.0f} GB/s text)", flush=True)
