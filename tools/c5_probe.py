#!/usr/bin/env python3
"""C5 tail-latency probe: two sliding-window streams back to back on ONE engine; prints the
per-trigger query latencies of both (a spike only in the first pass is an allocation)."""
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
if "--warmup" in sys.argv:
    eng.warmup()
for rnd in range(2):
    st = skyline.SkylineStream(eng, W)
    lat = []
    for t in range(triggers):
        for b0 in range(t * per, (t + 1) * per, batch):
            st.append(ids[b0:b0 + batch], vals[b0:b0 + batch])
        t0 = time.perf_counter()
        st.query_host_view()
        lat.append(round((time.perf_counter() - t0) * 1e3, 2))
    print(f"pass {rnd}: {lat}", flush=True)
    st.close()
