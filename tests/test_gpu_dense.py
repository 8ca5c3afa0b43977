"""The small-set route's dense all-pairs kernels run alone (sky_profile_pairs_dev): every row
against every row, ServiceTuple.dominates (ServiceTuple.java:67-77) over all pairs as the BNL
loops of FlinkSkyline.java:424-441 / :548-566 would evaluate them.  k_brute16_pairs (integer
rows, packed u16, the x chunk ordered by partition in LDS), k_brute_pairs<float> and <double>
must give every row exactly the fates of a numpy brute force: bit 0 = a row of its partition
dominates it, bit 1 = some row does.  The same kernels serve every query whose slots take the
brute route (C1-C4), which the configuration tests check end to end against the oracle."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def numpy_fates(vals, keys, block=512):
    n = len(vals)
    out = np.zeros(n, np.uint32)
    for i0 in range(0, n, block):
        y = vals[i0:i0 + block]                                   # [b, D]
        le = (vals[None, :, :] <= y[:, None, :]).all(-1)         # x_j <= y_i everywhere
        lt = (vals[None, :, :] < y[:, None, :]).any(-1)
        dom = le & lt                                             # [b, n]
        same = keys[None, :] == keys[i0:i0 + block, None]
        out[i0:i0 + block] = (dom & same).any(1).astype(np.uint32) | (dom.any(1).astype(np.uint32) << 1)
    return out


def run(eng, vals, keys):
    dv = torch.from_numpy(np.ascontiguousarray(vals)).cuda()
    dk = torch.from_numpy(np.ascontiguousarray(keys, np.int32)).cuda()
    df = torch.empty(len(vals), dtype=torch.int32, device="cuda")
    kind, ms = eng.profile_pairs_dev(dv, dk, df)
    eng.sync()
    return kind, df.cpu().numpy().astype(np.uint32)


@pytest.mark.parametrize("case", ["u16_std_anti", "u16_dups_many_parts", "u16_one_part", "f32_negative",
                                  "f64_inexact", "u16_16d"])
def test_dense_pairs_equal_numpy(case, gpu_engine_factory, oracle):
    rng = np.random.default_rng(sum(map(ord, case)))
    D, n, P = 8, 9000, 16
    if case == "u16_std_anti":
        vals = oracle.synth(3, D, n, seed=5)
        keys = rng.integers(0, P, n)
        want = 0
    elif case == "u16_dups_many_parts":
        vals = rng.integers(0, 6, size=(n, D)).astype(np.float64)   # many duplicates and ties
        keys = rng.integers(0, 200, n)
        want = 0
    elif case == "u16_one_part":
        vals = oracle.synth(2, D, n, seed=6)
        keys = np.zeros(n, np.int64)
        want = 0
    elif case == "f32_negative":
        vals = (rng.integers(-50, 50, size=(n, 4)) * 0.25).astype(np.float64)
        D = 4
        keys = rng.integers(0, P, n)
        want = 1
    elif case == "f64_inexact":
        vals = rng.integers(0, 40, size=(n, 5)).astype(np.float64) + 0.1
        D = 5
        keys = rng.integers(0, P, n)
        want = 2
    else:
        D = 16
        vals = oracle.synth(3, D, 4000, seed=7)
        keys = rng.integers(0, P, len(vals))
        want = 0
    eng = gpu_engine_factory(D, P)
    kind, got = run(eng, vals, keys)
    eng.close()
    assert kind == want
    np.testing.assert_array_equal(got, numpy_fates(vals, keys))
