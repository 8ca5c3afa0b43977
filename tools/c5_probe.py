#!/usr/bin/env python3
"""C5 tail-latency probe: the C5 stream (6D mixed, MR-Angle P=8, 1M tuples per trigger) twice on
ONE engine; per trigger: the query latency, the rep count, the route bits (counters[7]: 8 planned,
16 plan miss, mbr tile pairs << 8) and the phase times (profile level 2).  A spike only in the
first pass is an allocation.  Usage: python tools/c5_probe.py [W]   (W=0: landmark window)"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "flink-skyline-qos_amd"))
import torch  # noqa: E402,F401

import skyline  # noqa: E402
from skyline import _abi  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 10_000_000
D, P, per, batch, triggers = 6, 8, 1_000_000, 50_000, 20
vals, ids = skyline.synth_host(_abi.DISTS["mixed"], D, per * triggers, seed=1240)
eng = skyline.SkylineEngine(D, P, "mr-angle", 1000.0, 0)
eng.warmup()
for rnd in range(2):
    st = skyline.SkylineStream(eng, W)
    st.reserve(W if W else per * triggers)
    lat, rows = [], []
    for t in range(triggers):
        for b0 in range(t * per, (t + 1) * per, batch):
            st.append(ids[b0:b0 + batch], vals[b0:b0 + batch])
        eng.profile(2 if "--phases" in sys.argv else 0)
        t0 = time.perf_counter()
        g = st.query_host_view()
        lat.append(round((time.perf_counter() - t0) * 1e3, 3))
        ms, cnt = eng.phases()
        res, _ = st.size()
        rows.append({"t": t, "ms": lat[-1], "n": int(cnt[0]), "cand": int(cnt[1]), "reps": int(cnt[2]),
                     "greps": int(cnt[3]), "out": int(g), "rounds": int(cnt[5]), "bits": int(cnt[7]) & 255,
                     "mbr_tiles": int(cnt[7]) >> 8, "resident": int(res),
                     "phases": {k: round(v, 3) for k, v in ms.items() if v}})
    print(f"pass {rnd}: {lat}", flush=True)
    for r in rows:
        print(json.dumps(r), flush=True)
    st.close()
eng.close()
