"""HIP path vs oracle beyond the golden fixtures: seeded synthetic streams at
larger N (device generator), all partitioners, edge cases the reference's
semantics reach (empty, single tuple, all duplicates, P=1, D=1, NaN, infinities,
non-f32 values -> f64 path, score ties, ±0), repeated queries on one context."""
import numpy as np
import pytest
import torch

from conftest import Oracle

pytestmark = pytest.mark.gpu

DISTS = {"uniform": 0, "correlated": 1, "anti_correlated": 2, "std_anti": 3, "mixed": 4}


def run_query(make, vals, P, algo, ids=None, sem="reference"):
    eng = make(vals.shape[1], P, algo, semantics=sem)
    out = eng.query(vals, ids)
    st = eng.stats()
    eng.close()
    return out, st


def check_vs_oracle(make, orc, vals, P, algo, sem=0):
    (ids, org), (ls, sv) = run_query(make, vals, P, algo, sem="complete" if sem else "reference")
    exp, keys, els, esv = orc.query_sfs(algo, vals, P, 1000.0, sem)
    np.testing.assert_array_equal(ids, exp)
    np.testing.assert_array_equal(org, keys[exp])
    np.testing.assert_array_equal(ls, els)
    np.testing.assert_array_equal(sv, esv)
    return len(ids)


@pytest.mark.parametrize("dist", list(DISTS))
@pytest.mark.parametrize("D", [2, 3, 5, 8])
def test_synth_streams_vs_oracle(dist, D, gpu_engine_factory, oracle):
    n = 60000 if dist != "std_anti" else 20000
    vals = oracle.synth(DISTS[dist], D, n, seed=100 + D)
    for algo, P in (("mr-angle", 16), ("mr-dim", 8), ("mr-grid", 8)):
        check_vs_oracle(gpu_engine_factory, oracle, vals, P, algo)


def test_device_generator_matches_host(gpu_engine_factory, oracle):
    import skyline
    for dist in DISTS.values():
        for D in (1, 2, 4, 7, 8, 16):
            n = 5000
            eng = gpu_engine_factory(D, 4)
            dv = torch.empty((n, D), dtype=torch.float64, device="cuda")
            di = torch.empty(n, dtype=torch.int64, device="cuda")
            eng.synth_dev(dist, n, dv, di, seed=99, id0=12345)
            eng.sync()
            hv, hi = skyline.synth_host(dist, D, n, seed=99, id0=12345)
            ov = oracle.synth(dist, D, n, seed=99, id0=12345)
            np.testing.assert_array_equal(dv.cpu().numpy(), hv)
            np.testing.assert_array_equal(hv, ov)
            np.testing.assert_array_equal(di.cpu().numpy(), hi)
            eng.close()


def test_repeated_queries_one_context(gpu_engine_factory, oracle):
    eng = gpu_engine_factory(4, 8, "mr-angle")
    for seed in range(4):
        for n in (100000, 3000, 0, 50000):
            vals = oracle.synth(seed % 4, 4, n, seed=seed)
            ids, _ = eng.query(vals)
            exp, _, els, esv = oracle.query_sfs("angle", vals, 8)
            np.testing.assert_array_equal(ids, exp)
            ls, sv = eng.stats()
            np.testing.assert_array_equal(ls, els)
            np.testing.assert_array_equal(sv, esv)
    eng.close()


def test_edge_empty_and_single(gpu_engine_factory):
    eng = gpu_engine_factory(3, 4)
    ids, org = eng.query(np.zeros((0, 3)))
    assert len(ids) == 0
    ids, org = eng.query(np.array([[5.0, 1.0, 2.0]]), np.array([42]))
    assert ids.tolist() == [42]
    ls, sv = eng.stats()
    assert ls.sum() == 1 and sv.sum() == 1
    eng.close()


def test_all_duplicates_survive(gpu_engine_factory):
    vals = np.tile(np.array([[3.0, 4.0, 5.0, 6.0]]), (70000, 1))
    (ids, _), (ls, sv) = run_query(gpu_engine_factory, vals, 8, "mr-angle")
    assert len(ids) == 70000          # equal vectors never dominate each other
    assert ls.sum() == 70000 and sv.sum() == 70000


def test_one_partition_and_one_dim(gpu_engine_factory, oracle):
    rng = np.random.default_rng(5)
    vals = rng.integers(0, 50, size=(30000, 1)).astype(np.float64)
    check_vs_oracle(gpu_engine_factory, oracle, vals, 1, "mr-angle")
    check_vs_oracle(gpu_engine_factory, oracle, vals, 8, "mr-dim")
    vals = rng.integers(0, 1000, size=(30000, 6)).astype(np.float64)
    check_vs_oracle(gpu_engine_factory, oracle, vals, 1, "mr-grid")


def test_nan_is_rejected(gpu_engine_factory):
    from skyline._abi import SkylineError
    vals = np.ones((100, 2))
    vals[37, 1] = np.nan
    eng = gpu_engine_factory(2, 4)
    with pytest.raises(SkylineError) as e:
        eng.query(vals)
    assert e.value.code == -4
    eng.close()


def test_f64_path_and_score_ties(gpu_engine_factory, oracle):
    rng = np.random.default_rng(11)
    # not representable in f32 -> f64 rows; sums inexact -> tie-safe SFS
    vals = rng.random((40000, 4)) * 1000.0
    check_vs_oracle(gpu_engine_factory, oracle, vals, 8, "mr-angle")
    # equal-sum, mutually dominating-by-rounding data: huge and tiny magnitudes mixed
    base = rng.integers(0, 4, size=(20000, 3)).astype(np.float64)
    base[:, 0] *= 1e17
    base[:, 1] += rng.integers(0, 3, size=20000)
    check_vs_oracle(gpu_engine_factory, oracle, base, 4, "mr-dim")
    check_vs_oracle(gpu_engine_factory, oracle, base, 4, "mr-angle")


def test_infinities_and_signed_zero(gpu_engine_factory, oracle):
    rng = np.random.default_rng(3)
    vals = rng.integers(0, 20, size=(20000, 3)).astype(np.float64)
    vals[rng.random(20000) < 0.05, 1] = np.inf
    vals[rng.random(20000) < 0.05, 2] = -np.inf
    vals[rng.random(20000) < 0.2, 0] = -0.0
    for algo in ("mr-angle", "mr-dim", "mr-grid"):
        n = check_vs_oracle(gpu_engine_factory, oracle, vals, 8, algo)
        bnl, _, _, _ = oracle.query_bnl(algo[3:], vals, np.arange(len(vals)), 8)
        assert n == len(bnl)


def test_negative_values(gpu_engine_factory, oracle):
    rng = np.random.default_rng(8)
    vals = rng.integers(-500, 500, size=(50000, 4)).astype(np.float64)
    for algo in ("mr-angle", "mr-dim", "mr-grid"):
        check_vs_oracle(gpu_engine_factory, oracle, vals, 8, algo)


def test_grid_complete_semantics(gpu_engine_factory, oracle):
    vals = oracle.synth(0, 4, 50000, seed=3)
    n_ref = check_vs_oracle(gpu_engine_factory, oracle, vals, 8, "mr-grid", sem=0)
    n_all = check_vs_oracle(gpu_engine_factory, oracle, vals, 8, "mr-grid", sem=1)
    assert n_all >= n_ref
    assert len(oracle.brute(vals[:3000])) >= 0


def test_keys_random_f64_bit_exact(gpu_engine_factory, oracle):
    rng = np.random.default_rng(21)
    for D in (2, 3, 4, 8, 13, 16):
        v = rng.random((20000, D)) * rng.choice([1e-3, 1.0, 1e3, 1e6], size=(20000, 1))
        v[::7] = np.floor(v[::7])
        v[::11, 0] = 0.0
        for algo, name in ((0, "dim"), (1, "grid"), (2, "angle")):
            for P in (1, 7, 16, 256):
                eng = gpu_engine_factory(D, P, ["mr-dim", "mr-grid", "mr-angle"][algo], 1000.0)
                np.testing.assert_array_equal(eng.partition_keys(v), oracle.keys(name, v, P), err_msg=f"{name} D={D} P={P}")
                eng.close()


def test_angle_keys_near_partition_boundaries(gpu_engine_factory, oracle):
    """Tuples whose exact avg*P sits on / next to an integer force the exact fdlibm
    fallback of the filtered MR-Angle key; all must match the oracle bit for bit."""
    rng = np.random.default_rng(4)
    for D, P in ((2, 8), (2, 16), (3, 16), (4, 8), (8, 16), (8, 256)):
        rows = []
        for k in range(P + 1):
            for eps in (0.0, 1e-12, -1e-12, 1e-7, -1e-7, 1e-4, -1e-4):
                th = (k / P + eps) * (np.pi / 2)
                r = rng.random() * 1000 + 1
                v = np.zeros(D)
                v[0] = r * np.cos(th)
                v[1:] = r * np.sin(th) / np.sqrt(D - 1)
                rows.append(v)
                rows.append(np.round(v))
        v = np.asarray(rows)
        v = np.concatenate([v, -v[:20], np.abs(v) * 1e-16, np.abs(v) * 1e17])
        eng = gpu_engine_factory(D, P, "mr-angle")
        np.testing.assert_array_equal(eng.partition_keys(v), oracle.keys("angle", v, P), err_msg=f"D={D} P={P}")
        eng.close()


def test_angle_keys_many_random(gpu_engine_factory, oracle):
    rng = np.random.default_rng(12)
    for D in (2, 4, 8):
        v = rng.integers(0, 1001, size=(400000, D)).astype(np.float64)
        v[rng.random(len(v)) < 0.3] = 0.0
        v[rng.random(len(v)) < 0.1, 0] = 0.0
        eng = gpu_engine_factory(D, 16, "mr-angle")
        np.testing.assert_array_equal(eng.partition_keys(v), oracle.keys("angle", v, 16))
        eng.close()


def test_device_query_matches_host_query(gpu_engine_factory, oracle):
    n, D = 200000, 8
    vals = oracle.synth(2, D, n, seed=77)
    eng = gpu_engine_factory(D, 16)
    hid, horg = eng.query(vals, np.arange(n) + 10)
    dv = torch.from_numpy(vals).cuda()
    di = torch.arange(n, dtype=torch.int64, device="cuda") + 10
    oi = torch.empty(n, dtype=torch.int64, device="cuda")
    oo = torch.empty(n, dtype=torch.int32, device="cuda")
    g = eng.query_dev(di, dv, oi, oo, n)
    eng.sync()
    np.testing.assert_array_equal(oi[:g].cpu().numpy(), hid)
    np.testing.assert_array_equal(oo[:g].cpu().numpy(), horg)
    eng.close()


@pytest.mark.parametrize("dist,D,n", [("std_anti", 8, 300000), ("uniform", 6, 400000), ("anti_correlated", 4, 400000)])
def test_u16_path_equals_generic_path_at_scale(dist, D, n, gpu_engine_factory, oracle, monkeypatch):
    """The integer-packed dominance path (k_dom16: multi-round SFS, growing blocks,
    tiled tri/rest items) against the generic f32 SFS on streams too large for the
    oracle's SFS; both are checked against the oracle on the smaller cases above."""
    vals = oracle.synth(DISTS[dist], D, n, seed=500 + D)
    res = []
    for flag in ("1", "0"):
        monkeypatch.setenv("SKY_SFS16", flag)
        eng = gpu_engine_factory(D, 16, "mr-angle")
        ids, org = eng.query(vals)
        ls, sv = eng.stats()
        res.append((ids, org, ls, sv))
        eng.close()
    for a, b in zip(res[0], res[1]):
        np.testing.assert_array_equal(a, b)


def test_u16_path_tiny_segments_and_ties(gpu_engine_factory, oracle):
    """Integer rows with many equal scores, one-element partitions and P=256."""
    rng = np.random.default_rng(17)
    vals = rng.integers(0, 6, size=(30000, 5)).astype(np.float64)
    for algo, P in (("mr-angle", 256), ("mr-dim", 3), ("mr-grid", 32)):
        check_vs_oracle(gpu_engine_factory, oracle, vals, P, algo)


@pytest.mark.parametrize("D,P_,dist", [(2, 8, 0), (3, 8, 2), (3, 4, 1), (4, 16, 0)])
def test_grid_dominance_filter(gpu_engine_factory, oracle, D, P_, dist):
    """MR-Grid dominance filter (FlinkSkyline.java:716-733, disabled in the reference):
    tuples with every value >= maxVal/2 are removed before keyBy (key -1); the query
    equals the oracle's job with the same filter.  Also: with a tuple in the all-better
    quadrant present, the filtered skyline equals the unfiltered one."""
    import skyline
    vals = oracle.synth(dist, D, 30000, seed=21 + D)
    ids = np.arange(len(vals), dtype=np.int64)
    eng = skyline.SkylineEngine(D, P_, "mr-grid", 1000.0, 0, grid_filter=True)
    try:
        oracle.L.orc_set_grid_filter(1)
        keys = eng.partition_keys(vals)
        np.testing.assert_array_equal(keys, oracle.keys("grid", vals, P_))
        assert (keys == -1).sum() == int((vals >= 500.0).all(axis=1).sum())
        got, org = eng.query(vals, ids)
        exp, _, els, esv = oracle.query_bnl("grid", vals, ids, P_)
        assert sorted(got.tolist()) == sorted(exp.tolist())
        ls, sv = eng.stats()
        assert (ls == els).all() and (sv == esv).all()
    finally:
        oracle.L.orc_set_grid_filter(0)
    if ((vals < 500.0).all(axis=1)).any():
        plain = skyline.SkylineEngine(D, P_, "mr-grid", 1000.0, 0)
        g2, _ = plain.query(vals, ids)
        if 2 ** D <= P_:   # every key is queried: the filter cannot change the skyline
            assert sorted(g2.tolist()) == sorted(got.tolist())
        plain.close()
    eng.close()


@pytest.mark.parametrize("algo,P_,dist", [("mr-angle", 16, 2), ("mr-grid", 8, 1), ("mr-dim", 8, 3)])
def test_batched_readback_equals_per_range_copies(gpu_engine_factory, oracle, monkeypatch, algo, P_, dist):
    """Counter read-backs by one k_gather_words launch into the host-mapped staging
    buffer (default) and by one hipMemcpyAsync per range (SKY_GATHER=0): the same ids,
    origins and |L_k| / survivors_k, both equal to the oracle."""
    vals = oracle.synth(dist, 6, 40000, seed=77 + P_)
    res = []
    for flag in ("1", "0"):
        monkeypatch.setenv("SKY_GATHER", flag)
        res.append(run_query(gpu_engine_factory, vals, P_, algo))
    (a_ids, a_org), a_st = res[0]
    (b_ids, b_org), b_st = res[1]
    np.testing.assert_array_equal(a_ids, b_ids)
    np.testing.assert_array_equal(a_org, b_org)
    for x, y in zip(a_st, b_st):
        np.testing.assert_array_equal(x, y)
    monkeypatch.setenv("SKY_GATHER", "1")
    check_vs_oracle(gpu_engine_factory, oracle, vals, P_, algo)


@pytest.mark.parametrize("dist,D,P_,algo", [("anti_correlated", 8, 16, "mr-angle"), ("uniform", 6, 256, "mr-angle"),
                                            ("correlated", 4, 8, "mr-grid"), ("std_anti", 3, 8, "mr-dim"),
                                            ("uniform", 1, 4, "mr-dim")])
def test_candidate_prefilter_is_exact(dist, D, P_, algo, gpu_engine_factory, oracle, monkeypatch):
    """The candidate prefilter (second-level pruners drawn from the candidates, dropping the
    candidates they dominate before the sort) and the one-launch brute-force fates of small rep
    sets and the single-pass output never change a result: on/off combinations (SKY_PREFILTER,
    SKY_BRUTE, SKY_FUSED_OUT) give the
    same ids, origins and |L_k| / survivors_k, equal to the oracle."""
    n = 150_000
    vals = oracle.synth(DISTS[dist], D, n, seed=900 + D + P_)
    res = []
    for pre, brute, fused in (("1", "1", "1"), ("0", "0", "0"), ("1", "0", "2"), ("0", "1", "2")):
        monkeypatch.setenv("SKY_PREFILTER", pre)
        monkeypatch.setenv("SKY_BRUTE", brute)
        monkeypatch.setenv("SKY_FUSED_OUT", fused)
        res.append(run_query(gpu_engine_factory, vals, P_, algo))
    for r in res[1:]:
        for a, b in zip(res[0][0] + res[0][1], r[0] + r[1]):
            np.testing.assert_array_equal(a, b)
    for k in ("SKY_PREFILTER", "SKY_BRUTE", "SKY_FUSED_OUT"):
        monkeypatch.setenv(k, "1")
    check_vs_oracle(gpu_engine_factory, oracle, vals, P_, algo)


def test_device_query_capacity_and_buffer_reuse(gpu_engine_factory, oracle):
    """sky_query_dev with too small an output (SKY_E_CAPACITY, the required count reported),
    then with other output buffers on the same context: the single-pass output and the
    count + write path agree, and a later run never reuses a stale output decision."""
    from skyline._abi import SkylineError
    n, D = 120_000, 4
    vals = oracle.synth(2, D, n, seed=41)
    exp, keys, _, _ = oracle.query_sfs("angle", vals, 8)
    eng = gpu_engine_factory(D, 8)
    dv = torch.from_numpy(vals).cuda()
    di = torch.arange(n, dtype=torch.int64, device="cuda") * 3
    small_i = torch.empty(5, dtype=torch.int64, device="cuda")
    small_o = torch.empty(5, dtype=torch.int32, device="cuda")
    with pytest.raises(SkylineError) as e:
        eng.query_dev(di, dv, small_i, small_o, 5)
    assert e.value.code == -3
    for _ in range(2):
        oi = torch.full((n,), -1, dtype=torch.int64, device="cuda")
        oo = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        g = eng.query_dev(di, dv, oi, oo, n)
        eng.sync()
        np.testing.assert_array_equal(oi[:g].cpu().numpy(), exp * 3)
        np.testing.assert_array_equal(oo[:g].cpu().numpy(), keys[exp])
        assert (oi[g:].cpu().numpy() == -1).all()
    eng.close()


def test_duplicated_pruner_with_non_f32_values(gpu_engine_factory, oracle):
    """A pruner (sample minimum) whose values are not exact f32 and that other tuples duplicate
    becomes a slot: the row type must be f64 then, even if every candidate is f32-exact."""
    rng = np.random.default_rng(5)
    n, D = 200_000, 3
    vals = rng.integers(1, 1000, size=(n, D)).astype(np.float64)
    p = np.array([0.1, 0.2, 0.30000000000000004])          # not representable in f32
    vals[::7] = p                                          # duplicated, and dominating most tuples
    vals[3::11] = p + np.array([1e-9, 0.0, 0.0])           # dominated by p only in f64 arithmetic
    for algo in ("mr-angle", "mr-dim"):
        check_vs_oracle(gpu_engine_factory, oracle, vals, 8, algo)


@pytest.mark.parametrize("dist,D,algo", [("uniform", 6, "mr-angle"), ("std_anti", 4, "mr-dim"),
                                         ("anti_correlated", 8, "mr-angle")])
def test_candidate_slot_overflow_reruns(dist, D, algo, gpu_engine_factory, oracle, monkeypatch):
    """Candidate slots are sized by the last runs' need, not by n: a run whose candidates
    overflow them (SKY_SLOT_MIN forces a tiny first allocation) is re-run with room for all of
    them, with the same result as the oracle; later queries on the context reuse the grown slots."""
    monkeypatch.setenv("SKY_SLOT_MIN", "64")
    vals = oracle.synth(DISTS[dist], D, 80000, seed=44 + D)
    eng = gpu_engine_factory(D, 8, algo)
    exp, keys, els, esv = oracle.query_sfs(algo[3:], vals, 8)
    for _ in range(2):
        ids, org = eng.query(vals)
        np.testing.assert_array_equal(ids, exp)
        np.testing.assert_array_equal(org, keys[exp])
        ls, sv = eng.stats()
        np.testing.assert_array_equal(ls, els)
        np.testing.assert_array_equal(sv, esv)
    eng.close()


def test_warmup_then_queries(gpu_engine_factory, oracle):
    """sky_ctx_warmup runs every pipeline branch once on device-generated data; the context's
    later queries (small and large rep sets) are unaffected."""
    eng = gpu_engine_factory(6, 8, "mr-angle")
    eng.warmup()
    for dist, n in (("std_anti", 30000), ("anti_correlated", 60000), ("uniform", 50000)):
        vals = oracle.synth(DISTS[dist], 6, n, seed=5)
        ids, org = eng.query(vals)
        exp, keys, els, esv = oracle.query_sfs("angle", vals, 8)
        np.testing.assert_array_equal(ids, exp)
        ls, sv = eng.stats()
        np.testing.assert_array_equal(ls, els)
        np.testing.assert_array_equal(sv, esv)
    eng.close()


@pytest.mark.parametrize("D", [1, 2, 3, 5, 8, 9, 12, 16])
def test_packed_u16_brute_pass(D, gpu_engine_factory, oracle, monkeypatch):
    """Small candidate sets of integer rows go through k_brute16_pairs (packed u16 words,
    sum tie-break); it must agree with the oracle and with the f32 brute pass, at the ends
    of the u16 range, with heavy duplication and padding words (odd D, D > 8)."""
    rng = np.random.default_rng(700 + D)
    n = 12000
    a = rng.integers(0, 65536, size=(n, D))
    a[: n // 4] = rng.choice(np.array([0, 1, 65534, 65535]), size=(n // 4, D))
    a[n // 4: n // 2] = a[rng.integers(0, n // 4, size=n // 4)]          # duplicates
    vals = rng.permutation(a).astype(np.float64)
    for algo, P in (("mr-angle", 8), ("mr-dim", 4)):
        for flag in ("0", "1"):
            monkeypatch.setenv("SKY_BRUTE16", flag)
            check_vs_oracle(gpu_engine_factory, oracle, vals, P, algo)
    monkeypatch.setenv("SKY_BRUTE16", "1")


def test_use_torch_stream_equals_own_stream(gpu_engine_factory, oracle):
    """SkylineEngine.use_torch_stream(): the library runs on the caller's torch stream (a side
    stream here), so the *_dev calls skip the cross-stream events.  The tensors are produced and
    consumed on that stream with no extra synchronisation; every query -- the synchronised route
    and the planned replays, whose one-workgroup tail writes the final read into host-mapped
    memory -- equals the oracle, as on the library's own stream."""
    D, P, n = 2, 8, 200000
    vals = oracle.synth(0, D, n, seed=55)
    exp, keys, els, esv = oracle.query_sfs("dim", vals, P)
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        eng = gpu_engine_factory(D, P, "mr-dim")
        eng.use_torch_stream()
        for rep in range(4):
            dv = torch.from_numpy(vals).cuda()
            di = torch.arange(n, dtype=torch.int64, device="cuda")
            oi = torch.full((n,), -1, dtype=torch.int64, device="cuda")
            oo = torch.full((n,), -1, dtype=torch.int32, device="cuda")
            g = eng.query_dev(di, dv, oi, oo, n)
            got = oi[:g].cpu().numpy()                      # ordered after the query on `side`
            np.testing.assert_array_equal(got, exp)
            np.testing.assert_array_equal(oo[:g].cpu().numpy(), keys[exp])
            ls, sv = eng.stats()
            np.testing.assert_array_equal(ls, els)
            np.testing.assert_array_equal(sv, esv)
        eng.set_stream(None)                                 # back on the library's own stream
        g = eng.query_dev(di, dv, oi, oo, n)
        np.testing.assert_array_equal(oi[:g].cpu().numpy(), exp)
        eng.close()
