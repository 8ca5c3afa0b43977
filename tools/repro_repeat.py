"""Debug helper: the repeated-query sequence of tests/test_gpu_engine.py, several
times per SFS path, reporting mismatches against the oracle."""
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
for path in ("1", "0"):
    os.environ["SKY_SFS16"] = path
    for rep in range(2):
        eng = skyline.SkylineEngine(4, 8, "mr-angle", 1000.0, 0)
        for seed in range(4):
            for n in (100000, 3000, 0, 50000):
                vals = orc.synth(seed % 4, 4, n, seed=seed)
                ids, _ = eng.query(vals)
                exp, _, els, esv = orc.query_sfs("angle", vals, 8)
                ls, sv = eng.stats()
                ok = np.array_equal(ids, exp) and np.array_equal(ls, els) and np.array_equal(sv, esv)
                extra = np.setdiff1d(ids, exp)
                missing = np.setdiff1d(exp, ids)
                print(f"sfs16={path} rep={rep} seed={seed} n={n}: {'ok' if ok else 'MISMATCH'} "
                      f"got={len(ids)} exp={len(exp)} extra={len(extra)} missing={len(missing)}", flush=True)
        eng.close()
