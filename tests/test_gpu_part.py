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


def test_part_state_pruner_classes(gpu_engine_factory, oracle):
    """k_parts_prune's corner cases: many tuples equal to a pruner (classes sharing its fate, the
    first of them the equal-earlier tuple), criterion ties where the chosen pruner (the smaller
    index) is dominated by a later tuple with the same rounded criterion, pruners equal to each
    other, -0.0 / +0.0 twins, and rows whose criterion is NaN (+inf and -inf in one row)."""
    rng = np.random.default_rng(21)
    n, D = 24000, 3
    v = rng.integers(0, 4, size=(n, D)).astype(np.float64)
    v[::3] = [1.0, 1.0, 1.0]                        # a big class of one vector
    v[5::97] = [1.0, 1e-17, 0.0]                     # same f64 sum as (1, 0, 0) ...
    v[6::97] = [1.0, 0.0, 0.0]                       # ... which dominates it
    v[40::211] = [-0.0, 2.0, 2.0]
    v[41::211] = [0.0, 2.0, 2.0]
    v[77::509] = [np.inf, -np.inf, 1.0]              # criterion NaN
    v[78::509] = [-np.inf, 5.0, 5.0]
    replay(gpu_engine_factory, oracle, v, [5000, 1, 2, 4000, 997, 3000] + [2000] * 4 + [n - 17000], D)


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


def test_part_async_inserts_without_sync(gpu_engine_factory, oracle):
    """Hundreds of inserts issued back to back with no synchronisation in between (bounds from
    the host mirror, capacities grown on the stream, in-insert compaction of a kill-heavy
    stream): the one snapshot at the end equals the oracle."""
    from skyline.operators import _LocalPart
    rng = np.random.default_rng(31)
    n, D = 60000, 3
    base = np.repeat(np.arange(n // 500)[::-1], 500)[:, None] * 25.0
    vals = base + rng.integers(0, 40, size=(n, D)).astype(np.float64)
    vals[::7] = vals[::7].round(-1)
    ids = np.arange(n, dtype=np.int64) * 5 + 1
    eng = gpu_engine_factory(D, 8)
    part = _LocalPart(eng, 3)
    s = 0
    while s < n:
        f = int(min(n - s, rng.integers(1, 700)))
        part.insert(ids[s:s + f], vals[s:s + f])
        s += f
    got_ids, got_vals = part.snapshot()
    exp, _, _, _ = oracle.query_sfs("dim", vals, 1)
    np.testing.assert_array_equal(got_ids, ids[exp])
    np.testing.assert_array_equal(got_vals, vals[exp])
    part.close()
    eng.close()


@pytest.mark.parametrize("dist,D", [(2, 8), (3, 4), (4, 6)])
def test_parts_insert_batched_keys_vs_oracle(dist, D, gpu_engine_factory, oracle):
    """sky_parts_insert: the full buffers of several keys per call (each key at most once per
    call), no synchronisation until the trigger; every key's snapshot equals the oracle's local
    skyline of its tuples, and equals one sky_part_insert per buffer."""
    from skyline.operators import _LocalPart
    n, P, buf = 120000, 8, 5000
    vals = oracle.synth(dist, D, n, seed=90 + D)
    ids = np.arange(n, dtype=np.int64)
    eng = gpu_engine_factory(D, P)
    keys = eng.partition_keys(vals)
    rng = np.random.default_rng(D)
    per = {k: np.flatnonzero(keys == k) for k in range(P)}
    a = {k: _LocalPart(eng, k) for k in range(P)}
    b = {k: _LocalPart(eng, k) for k in range(P)}
    pos = {k: 0 for k in range(P)}
    while any(pos[k] < len(per[k]) for k in range(P)):
        call = [k for k in range(P) if pos[k] < len(per[k]) and rng.random() < 0.6]
        batches = []
        for k in call:
            f = int(min(len(per[k]) - pos[k], rng.integers(1, 2 * buf)))
            sel = per[k][pos[k]:pos[k] + f]
            batches.append((ids[sel], vals[sel]))
            pos[k] += f
            b[k].insert(ids[sel], vals[sel])
        _LocalPart.insert_many([a[k] for k in call], batches)
    for k in range(P):
        got_ids, got_vals = a[k].snapshot()
        ref_ids, _ = b[k].snapshot()
        exp, _, _, _ = oracle.query_sfs("dim", vals[per[k]], 1)
        np.testing.assert_array_equal(got_ids, ids[per[k]][exp])
        np.testing.assert_array_equal(got_vals, vals[per[k]][exp])
        np.testing.assert_array_equal(ref_ids, got_ids)
    for x in list(a.values()) + list(b.values()):
        x.close()
    eng.close()


def test_parts_insert_nan_rejects_the_whole_call(gpu_engine_factory, oracle):
    from skyline.operators import _LocalPart
    D = 4
    vals = oracle.synth(3, D, 20000, seed=2)
    ids = np.arange(len(vals), dtype=np.int64)
    eng = gpu_engine_factory(D, 8)
    p0, p1 = _LocalPart(eng, 0), _LocalPart(eng, 1)
    _LocalPart.insert_many([p0, p1], [(ids[:5000], vals[:5000]), (ids[5000:10000], vals[5000:10000])])
    before = [p0.snapshot(), p1.snapshot()]
    bad = vals[15000:20000].copy()
    bad[4999, 0] = np.nan
    with pytest.raises(SkylineError) as e:
        _LocalPart.insert_many([p0, p1], [(ids[10000:15000], vals[10000:15000]), (ids[15000:], bad)])
    assert e.value.code == SKY_E_NAN
    after = [p0.snapshot(), p1.snapshot()]
    for x, y in zip(before, after):
        np.testing.assert_array_equal(x[0], y[0])
        np.testing.assert_array_equal(x[1], y[1])
    with pytest.raises(SkylineError):                     # one part twice in one call
        _LocalPart.insert_many([p0, p0], [(ids[:10], vals[:10]), (ids[10:20], vals[10:20])])
    p0.close()
    p1.close()
    eng.close()


@pytest.mark.parametrize("dist,D,n", [(2, 8, 80000), (3, 4, 40000), (0, 3, 30000)])
def test_parts_global_merge_equals_snapshot_merge(dist, D, n, gpu_engine_factory, oracle):
    """sky_parts_global_merge over device-resident states == sky_global_merge over their
    snapshots (ids, origins, order, |L_k|, survivors_k), and == the oracle's two-level skyline."""
    from skyline.operators import _LocalPart
    P = 8
    eng = gpu_engine_factory(D, P)
    vals = oracle.synth(dist, D, n, seed=90 + D)
    vals[5::101] = vals[7]                          # the same vector in several keys
    ids = np.arange(n, dtype=np.int64) * 5 + 3
    keys = eng.partition_keys(vals)
    parts = {k: _LocalPart(eng, k) for k in range(P)}
    for k in range(P):
        sel = np.nonzero(keys == k)[0]
        for s0 in range(0, len(sel), 5000):
            parts[k].insert(ids[sel[s0:s0 + 5000]], vals[sel[s0:s0 + 5000]])
    order = [3, 0, 7, 1, 5, 2, 6, 4]                # any list order: the output follows it
    plist = [parts[k] for k in order]
    g_ids, g_org = _LocalPart.global_merge_many(eng, plist, order)
    ls_dev, sv_dev = eng.stats()
    snaps = [p.snapshot() for p in plist]
    e_ids, e_org = eng.global_merge(order, [s[0] for s in snaps], [s[1] for s in snaps])
    ls_ref, sv_ref = eng.stats()
    np.testing.assert_array_equal(g_ids, e_ids)
    np.testing.assert_array_equal(g_org, e_org)
    np.testing.assert_array_equal(ls_dev, ls_ref)
    np.testing.assert_array_equal(sv_dev, sv_ref)
    # the distinct-vector messages (what the Java LocalProcessor ships): same expansion, same merge
    reps = [p.snapshot_reps() for p in plist]
    for r, sn in zip(reps, snaps):
        np.testing.assert_array_equal(r.ids, sn[0])
        np.testing.assert_array_equal(r.values(), sn[1])
        np.testing.assert_array_equal(r.rep_counts, np.bincount(r.rep_idx, minlength=len(r.reps)))
        assert len(np.unique(r.reps, axis=0)) == len(r.reps)
    r_ids, r_org = eng.global_merge_reps(order, [(r.ids, r.rep_idx, r.reps, r.rep_counts) for r in reps])
    ls_r, sv_r = eng.stats()
    np.testing.assert_array_equal(r_ids, e_ids)
    np.testing.assert_array_equal(r_org, e_org)
    np.testing.assert_array_equal(ls_r, ls_ref)
    np.testing.assert_array_equal(sv_r, sv_ref)
    exp, _, _, _ = oracle.query_bnl("angle", vals, ids, P)
    assert sorted(g_ids.tolist()) == sorted(exp.tolist())
    for p in parts.values():
        p.close()
    eng.close()


def test_parts_global_merge_edge_cases(gpu_engine_factory, oracle):
    """Empty parts (never inserted into), a single part, a state with dead vectors (compacted by the
    merge), and no parts at all: sky_parts_global_merge equals the snapshot-based merge."""
    from skyline.operators import _LocalPart
    D = 4
    eng = gpu_engine_factory(D, 8)
    rng = np.random.default_rng(33)
    a = _LocalPart(eng, 0)
    b = _LocalPart(eng, 1)                          # stays empty
    c = _LocalPart(eng, 2)
    base = rng.integers(20, 60, size=(3000, D)).astype(np.float64)
    a.insert(np.arange(3000, dtype=np.int64), base)
    a.insert(np.arange(3000, 4000, dtype=np.int64), base[:1000] - 15.0)   # kills most of a's vectors
    c.insert(np.arange(5000, 5500, dtype=np.int64), rng.integers(0, 80, size=(500, D)).astype(np.float64))
    for plist, pids in (([a, b, c], [0, 1, 2]), ([b], [1]), ([c], [7]), ([], [])):
        g_ids, g_org = _LocalPart.global_merge_many(eng, plist, pids)
        ls_dev, sv_dev = eng.stats()
        snaps = [p.snapshot() for p in plist]
        e_ids, e_org = eng.global_merge(pids, [s[0] for s in snaps], [s[1] for s in snaps])
        ls_ref, sv_ref = eng.stats()
        np.testing.assert_array_equal(g_ids, e_ids)
        np.testing.assert_array_equal(g_org, e_org)
        np.testing.assert_array_equal(ls_dev, ls_ref)
        np.testing.assert_array_equal(sv_dev, sv_ref)
        reps = [p.snapshot_reps() for p in plist]
        r_ids, r_org = eng.global_merge_reps(pids, [(r.ids, r.rep_idx, r.reps, r.rep_counts) for r in reps])
        np.testing.assert_array_equal(r_ids, e_ids)
        np.testing.assert_array_equal(r_org, e_org)
        for x, y in zip(eng.stats(), (ls_ref, sv_ref)):
            np.testing.assert_array_equal(x, y)
    # a rep index outside its list's reps is an argument error, not an out-of-range read
    r = a.snapshot_reps()
    bad = r.rep_idx.copy()
    bad[len(bad) // 2] = len(r.reps)
    with pytest.raises(SkylineError) as e:
        eng.global_merge_reps([0], [(r.ids, bad, r.reps, r.rep_counts)])
    assert e.value.code == -1
    # malformed tuple counts per rep (the merge's weights): a zero / negative count, or counts
    # that do not sum to the list's tuples, are argument errors (else survivors_k > |L_k|)
    assert len(r.reps) >= 2
    for mutate in ("zero", "negative", "sum"):
        rc = r.rep_counts.copy()
        if mutate == "zero":
            rc[0] = 0
        elif mutate == "negative":
            rc[0], rc[1] = -rc[1], rc[0] + 2 * rc[1]        # the sum stays right
        else:
            rc[0] += 1
        with pytest.raises(SkylineError) as e:
            eng.global_merge_reps([0], [(r.ids, r.rep_idx, r.reps, rc)])
        assert e.value.code == -1 and "rep_counts" in str(e.value), (mutate, str(e.value))
    ok_ids, _ = eng.global_merge_reps([0], [(r.ids, r.rep_idx, r.reps, r.rep_counts)])   # still usable
    assert len(ok_ids) > 0
    for p in (a, b, c):
        p.close()
    eng.close()
