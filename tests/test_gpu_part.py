"""The per-key operator state (sky_part_*, k_part.hip): SkylineLocalProcessor.processBuffer
(FlinkSkyline.java:417-444) sets S <- SKY(S u B) per buffer B; the state is held as distinct
vectors + the tuples on them and updated incrementally.  After every insert the snapshot
(ids in insertion order, their values) must equal the oracle's skyline of everything inserted
so far: duplicate-heavy keys (the reference anti-correlated formula: the all-zero tuples),
large skylines (std-anti), random flush sizes, +-0 / +-inf / non-f32 values, states where later
tuples kill most reps (lazy compaction), and a NaN batch that is rejected without a trace."""
import numpy as np
import pytest

from skyline._abi import SKY_E_NAN, SkylineError

pytestmark = pytest.mark.gpu


def replay(eng_factory, oracle, vals, flushes, D, check_every=1):
    from skyline.operators import _LocalPart
    eng = eng_factory(D, 8)
    ids = np.arange(len(vals), dtype=np.int64) * 3 + 11
    part = _LocalPart(eng, 0)
    s = 0
    for i, f in enumerate(flushes):
        part.insert(ids[s:s + f], vals[s:s + f])
        s += f
        if i % check_every == 0 or s == len(vals):
            got_ids, got_vals = part.snapshot()
            exp, _, _, _ = oracle.query_sfs("dim", vals[:s], 1)
            np.testing.assert_array_equal(got_ids, ids[exp])          # insertion order
            np.testing.assert_array_equal(got_vals, vals[exp])
    part.close()
    eng.close()


@pytest.mark.parametrize("dist,D,n", [(2, 8, 60000), (2, 4, 60000), (1, 4, 40000), (0, 6, 40000), (3, 4, 40000),
                                      (3, 8, 15000)])
def test_part_state_vs_oracle(dist, D, n, gpu_engine_factory, oracle):
    vals = oracle.synth(dist, D, n, seed=60 + D + dist)
    flushes = [5000] * (n // 5000) + ([n % 5000] if n % 5000 else [])
    replay(gpu_engine_factory, oracle, vals, flushes, D)


def test_part_state_random_flushes(gpu_engine_factory, oracle):
    rng = np.random.default_rng(9)
    vals = oracle.synth(3, 5, 50000, seed=3)
    flushes = []
    left = len(vals)
    while left:
        f = int(min(left, rng.integers(1, 9000)))
        flushes.append(f)
        left -= f
    replay(gpu_engine_factory, oracle, vals, flushes, 5, check_every=3)


def test_part_state_special_values(gpu_engine_factory, oracle):
    rng = np.random.default_rng(4)
    v = rng.integers(-2, 3, size=(20000, 3)).astype(np.float64) * 0.5
    v[v == 0] = np.where(rng.random((v == 0).sum()) < 0.5, -0.0, 0.0)
    v[::53, 0] = np.inf
    v[7::61, 2] = -np.inf
    v[3::17] += 0.1                      # not exact in f32
    replay(gpu_engine_factory, oracle, v, [777] * 25 + [20000 - 777 * 25], 3)


def test_part_state_kills_and_compaction(gpu_engine_factory, oracle):
    """Every batch dominates most of the state before it: reps die, their tuples are dropped
    by the lazy compaction, and the survivors keep their insertion order."""
    rng = np.random.default_rng(12)
    n, D = 30000, 3
    base = np.repeat(np.arange(n // 1000)[::-1], 1000)[:, None] * 40.0
    vals = base + rng.integers(0, 60, size=(n, D)).astype(np.float64)
    vals[::9] = vals[::9].round(-1)       # duplicates inside and across batches
    replay(gpu_engine_factory, oracle, vals, [1000] * (n // 1000), D)


def test_part_state_nan_batch_rejected(gpu_engine_factory, oracle):
    from skyline.operators import _LocalPart
    D = 4
    vals = oracle.synth(2, D, 15000, seed=8)
    ids = np.arange(len(vals), dtype=np.int64)
    eng = gpu_engine_factory(D, 8)
    part = _LocalPart(eng, 1)
    part.insert(ids[:5000], vals[:5000])
    before = part.snapshot()
    bad = vals[5000:10000].copy()
    bad[123, 2] = np.nan
    with pytest.raises(SkylineError) as e:
        part.insert(ids[5000:10000], bad)
    assert e.value.code == SKY_E_NAN
    after = part.snapshot()
    np.testing.assert_array_equal(before[0], after[0])
    np.testing.assert_array_equal(before[1], after[1])
    part.insert(ids[10000:], vals[10000:])
    got_ids, _ = part.snapshot()
    keep = np.r_[0:5000, 10000:15000]
    exp, _, _, _ = oracle.query_sfs("dim", vals[keep], 1)
    np.testing.assert_array_equal(got_ids, ids[keep][exp])
    part.close()
    eng.close()
