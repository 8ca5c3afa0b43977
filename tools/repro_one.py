"""Debug helper: one failing configuration, repeated, with SKY_DEBUG=3 summaries."""
import os
import sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "flink-skyline-qos_amd"))
import torch  # noqa: E402,F401
import skyline  # noqa: E402
from conftest import Oracle  # noqa: E402
orc = Oracle()
vals = orc.synth(3, 4, 100000, seed=3)
exp, keys, els, esv = orc.query_sfs("angle", vals, 8)
print("oracle", len(exp), "local sizes", els.tolist(), flush=True)
for path in ("1", "0"):
    os.environ["SKY_SFS16"] = path
    for rep in range(3):
        eng = skyline.SkylineEngine(4, 8, "mr-angle", 1000.0, 0)
        ids, _ = eng.query(vals)
        ls, sv = eng.stats()
        print(f"path {path} rep {rep}: got {len(ids)} ls {ls.tolist()} sv {sv.tolist()}", flush=True)
        eng.close()
