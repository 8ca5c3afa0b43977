"""GPU probe: stream append NaN admission (prints the flag path step by step)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "flink-skyline-qos_amd"))
import torch  # noqa
import skyline
from skyline._abi import SkylineError
eng = skyline.SkylineEngine(4, 8, "mr-angle", 1000.0, 0)
for W in (0, 5000):
    st = skyline.SkylineStream(eng, W)
    v = np.random.default_rng(1).integers(0, 1000, size=(10000, 4)).astype(np.float64)
    ids = np.arange(10000, dtype=np.int64)
    bad = v.copy(); bad[1234, 2] = np.nan
    try:
        st.append(ids, bad); print("W", W, "fresh: no raise", st.size())
    except SkylineError as e:
        print("W", W, "fresh: raised", e.code, st.size())
    st.append(ids, v); st.query()
    try:
        st.append(ids + 10000, bad); print("W", W, "after query: no raise", st.size())
    except SkylineError as e:
        print("W", W, "after query: raised", e.code, st.size())
    st.close()
