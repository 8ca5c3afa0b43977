"""HIP path vs the oracle on the golden streams (reference generator) — the parity gate.

Bar: the skyline ID SET is identical, and |L_k| / survivors_k (the integers behind
optimality, FlinkSkyline.java:593-608) are identical, for every stream x
partitioner x P in the committed fixtures.  Keys are bit-exact."""
import os

import numpy as np
import pytest

from conftest import golden_streams, load_golden

pytestmark = pytest.mark.gpu

ALGO_NAME = {"dim": "mr-dim", "grid": "mr-grid", "angle": "mr-angle"}


@pytest.mark.parametrize("path", golden_streams(), ids=lambda p: os.path.basename(p)[7:-4])
def test_keys_bit_exact(path, gpu_engine_factory):
    g = load_golden(path)
    D = g["values"].shape[1]
    for algo in ("dim", "grid", "angle"):
        for P in (4, 8, 16):
            eng = gpu_engine_factory(D, P, ALGO_NAME[algo])
            keys = eng.partition_keys(g["values"])
            np.testing.assert_array_equal(keys, g[f"keys_{algo}_{P}"].astype(np.int32), err_msg=f"{algo} P={P}")
            eng.close()


@pytest.mark.parametrize("path", golden_streams(), ids=lambda p: os.path.basename(p)[7:-4])
def test_query_matches_golden(path, gpu_engine_factory):
    g = load_golden(path)
    D = g["values"].shape[1]
    for algo in ("dim", "grid", "angle"):
        for P in (4, 8, 16):
            eng = gpu_engine_factory(D, P, ALGO_NAME[algo])
            ids, org = eng.query(g["values"], g["ids"])
            assert np.all(np.diff(ids) > 0), "output must be in stream order, unique"
            np.testing.assert_array_equal(ids, g[f"gsky_{algo}_{P}"].astype(np.int64), err_msg=f"{algo} P={P}")
            keys = g[f"keys_{algo}_{P}"].astype(np.int32)
            np.testing.assert_array_equal(org, keys[ids])
            ls, sv = eng.stats()
            np.testing.assert_array_equal(ls, g[f"lsz_{algo}_{P}"], err_msg=f"local sizes {algo} P={P}")
            np.testing.assert_array_equal(sv, g[f"surv_{algo}_{P}"], err_msg=f"survivors {algo} P={P}")
            eng.close()
