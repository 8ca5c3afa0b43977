#!/usr/bin/env python3
"""Route bits of consecutive queries on one engine (plan learned / replayed / missed), with the
measurement build's SKY_DEBUG=1 miss reasons.  Usage: python tools/plan_miss_probe.py algo dist D n P seeds..."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "flink-skyline-qos_amd"))
sys.path.insert(0, os.path.join(R, "tests"))
import skyline  # noqa: E402
from conftest import Oracle  # noqa: E402

algo, dist, D, n, P = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
orc = Oracle()
eng = skyline.SkylineEngine(D, P, algo, 1000.0, 0)
for seed in sys.argv[6:]:
    ids, _ = eng.query(orc.synth(dist, D, n, seed=int(seed)))
    _, counters = eng.phases()
    print(f"seed {seed}: out {len(ids)} route_bits {int(counters[7]) & 0xff}", flush=True)
eng.close()
