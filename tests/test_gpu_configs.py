"""BASELINE.json configurations at their full sizes, checked against the oracle.

  C2  MR-Grid  4D correlated       10M tuples, P=8, one GPU
  C3  MR-Angle 4D anti-correlated  50M tuples, P=8, one GPU and sharded 2/4/8 ways
  C4  MR-Angle 8D anti-correlated 100M tuples, P=16 (one GPU's share of the headline)
  C5  6D mixed stream, MR-Angle P=8, landmark and count-based sliding windows

The checker at these sizes is the chunked oracle (oracle/skyline_oracle_big.c): the same
restatement of FlinkSkyline.java:417-444 / :548-566 / :593-608 as the golden-size oracle,
computed as SKY(U SKY(chunk)) per key and globally over distinct vectors (pinned against
every golden stream in test_cpu_oracle.py).  Streams come from the device generator,
which equals the oracle's generator bit for bit (test_gpu_engine.py).
"""
import numpy as np
import pytest
import torch
from conftest import dist_emulate

pytestmark = pytest.mark.gpu

DISTS = {"uniform": 0, "correlated": 1, "anti_correlated": 2, "std_anti": 3, "mixed": 4}


def device_stream(eng, dist, n, seed, id0=0):
    vals = torch.empty((n, eng.dims), dtype=torch.float64, device="cuda")
    ids = torch.empty(n, dtype=torch.int64, device="cuda")
    eng.synth_dev(dist, n, vals, ids, seed=seed, id0=id0)
    eng.sync()
    return vals, ids


def query_dev(eng, vals, ids):
    n = vals.shape[0]
    oi = torch.empty(max(n, 1), dtype=torch.int64, device="cuda")
    oo = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")
    g = eng.query_dev(ids, vals, oi, oo, n)
    eng.sync()
    ls, sv = eng.stats()
    return oi[:g].cpu().numpy(), oo[:g].cpu().numpy(), ls, sv


def check_full(oracle, algo, vals_np, P, got):
    gi, go, ls, sv = got
    exp, keys, els, esv, _ = oracle.query_sfs_chunked(algo, vals_np, P)
    np.testing.assert_array_equal(gi, exp)            # ids = row index, stream order
    np.testing.assert_array_equal(go, keys[exp])
    np.testing.assert_array_equal(ls, els)
    np.testing.assert_array_equal(sv, esv)
    return exp


# ---- mixed streams spanning every generator block ------------------------------------
@pytest.mark.parametrize("D", [2, 4, 6, 8])
def test_mixed_streams_span_three_blocks(D, gpu_engine_factory, oracle):
    """'mixed' switches distribution every 65,536 ids (uniform, correlated, anti-correlated):
    streams of 4 x 65,536 + 1,234 tuples cover all three and a partial fourth block."""
    n = 4 * 65536 + 1234
    vals = oracle.synth(DISTS["mixed"], D, n, seed=300 + D)
    blocks = (np.arange(n) >> 16) % 3
    assert set(blocks.tolist()) == {0, 1, 2}
    for algo, P in (("mr-angle", 8), ("mr-dim", 8), ("mr-grid", 8)):
        eng = gpu_engine_factory(D, P, algo)
        ids, org = eng.query(vals)
        ls, sv = eng.stats()
        eng.close()
        exp, keys, els, esv = oracle.query_sfs(algo[3:], vals, P)
        np.testing.assert_array_equal(ids, exp)
        np.testing.assert_array_equal(org, keys[exp])
        np.testing.assert_array_equal(ls, els)
        np.testing.assert_array_equal(sv, esv)


# ---- C5: 6D mixed continuous queries ---------------------------------------------------
@pytest.mark.parametrize("W", [0, 100_000, 262_144])
def test_c5_stream_6d_mixed_vs_oracle(W, gpu_engine_factory, oracle):
    """Config C5 as configured: 6D mixed stream, MR-Angle, P=8, micro-batches appended from
    the device at irregular sizes, triggers at irregular points; every answer (id set in
    arrival order, |L_k|, survivors_k) equals the oracle over the landmark prefix (W=0) or
    the last W tuples (sliding window, extension)."""
    import skyline
    D, P_, n = 6, 8, 700_000
    eng = gpu_engine_factory(D, P_, "mr-angle")
    dv, di = device_stream(eng, "mixed", n, seed=55 + W)
    vals = dv.cpu().numpy()
    st = skyline.SkylineStream(eng, W)
    rng = np.random.default_rng(W + 1)
    oi = torch.empty(n, dtype=torch.int64, device="cuda")
    oo = torch.empty(n, dtype=torch.int32, device="cuda")
    pos, checks = 0, 0
    while pos < n:
        b = int(min(n - pos, rng.integers(1, 90_000)))
        st.append_dev(di[pos:pos + b], dv[pos:pos + b], b)
        pos += b
        if rng.random() < 0.3 or pos == n:
            g = st.query_dev(oi, oo, n)
            eng.sync()
            got = oi[:g].cpu().numpy()
            org = oo[:g].cpu().numpy()
            ls, sv = eng.stats()
            lo = max(0, pos - W) if W else 0
            exp, keys, els, esv, _ = oracle.query_sfs_chunked("angle", vals[lo:pos], P_, chunk=65536)
            np.testing.assert_array_equal(got, exp + lo)          # ids = stream index, arrival order
            np.testing.assert_array_equal(org, keys[exp])
            np.testing.assert_array_equal(ls, els)
            np.testing.assert_array_equal(sv, esv)
            checks += 1
    assert checks >= 3
    st.close()
    eng.close()


def test_stream_nan_append_is_rejected_and_stream_stays_queryable(gpu_engine_factory, oracle):
    """A micro-batch holding a NaN is rejected whole (SKY_E_NAN) before it becomes resident;
    the landmark state stays queryable and equal to the oracle over the accepted batches."""
    import skyline
    from skyline._abi import SkylineError
    D, P_ = 4, 8
    vals = oracle.synth(2, D, 30000, seed=9)
    ids = np.arange(len(vals), dtype=np.int64)
    for W in (0, 5000):
        eng = gpu_engine_factory(D, P_, "mr-angle")
        st = skyline.SkylineStream(eng, W)
        st.append(ids[:10000], vals[:10000])
        st.query()
        bad = vals[10000:20000].copy()
        bad[8000, 2] = np.nan       # inside the newest 5000 of the batch (the window keeps those)
        before = st.size()
        with pytest.raises(SkylineError) as e:
            st.append(ids[10000:20000], bad)
        assert e.value.code == -4
        assert st.size() == before
        st.append(ids[20000:], vals[20000:])
        got, _ = st.query()
        keep = np.r_[0:10000, 20000:30000]
        lo = 0 if W == 0 else len(keep) - W
        sel = keep[lo:]
        exp, _, els, esv = oracle.query_sfs("angle", vals[sel], P_)
        np.testing.assert_array_equal(got, sel[exp])
        ls, sv = eng.stats()
        np.testing.assert_array_equal(ls, els)
        np.testing.assert_array_equal(sv, esv)
        st.close()
        eng.close()


# ---- C2 / C3 / C4 at full size -----------------------------------------------------------
def test_c1_dim_2d_uniform_1m(gpu_engine_factory, oracle):
    """C1 at its stated size: MR-Dim, 2D independent (uniform), 1M tuples, P = 8 (Flink
    parallelism 4).  Checked against the chunked oracle AND the literal per-key BNL restatement
    with 5000-tuple buffers (FlinkSkyline.java:417-444, :548-566), ids and integers."""
    D, P_, n = 2, 8, 1_000_000
    eng = gpu_engine_factory(D, P_, "mr-dim")
    dv, di = device_stream(eng, "uniform", n, seed=1234 + D)
    got = query_dev(eng, dv, di)
    eng.close()
    vals = dv.cpu().numpy()
    exp = check_full(oracle, "dim", vals, P_, got)
    g, keys, ls, sv = oracle.query_bnl("dim", vals, np.arange(n, dtype=np.int64), P_)
    np.testing.assert_array_equal(np.sort(g), exp)
    np.testing.assert_array_equal(ls, got[2])
    np.testing.assert_array_equal(sv, got[3])


def test_c2_grid_4d_correlated_10m(gpu_engine_factory, oracle, monkeypatch):
    D, P_, n = 4, 8, 10_000_000
    eng = gpu_engine_factory(D, P_, "mr-grid")
    dv, di = device_stream(eng, "correlated", n, seed=1204)
    got = query_dev(eng, dv, di)
    vals = dv.cpu().numpy()
    exp = check_full(oracle, "grid", vals, P_, got)
    assert (vals[exp] == 0).all()                       # PDF p.15: the correlated skyline is [0,...,0]
    monkeypatch.setenv("SKY_SFS16", "0")                 # the generic f32 SFS agrees at full size
    got2 = query_dev(eng, dv, di)
    for a, b in zip(got, got2):
        np.testing.assert_array_equal(a, b)
    eng.close()


def test_c3_angle_4d_anti_50m_one_gpu_and_sharded(gpu_engine_factory, oracle):
    """C3 on one GPU, and the same stream split into 2, 4 and 8 rank shards run through the
    multi-GPU step (sky_dist_export -> all-gather -> sky_dist_merge -> all-reduce ->
    sky_dist_finish, one context per emulated rank):
    every decomposition returns the one-GPU ids, origins, |L_k| and survivors_k."""
    D, P_, n = 4, 8, 50_000_000
    eng = gpu_engine_factory(D, P_, "mr-angle")
    dv, di = device_stream(eng, "anti_correlated", n, seed=1234 + D)
    got = query_dev(eng, dv, di)
    eng.close()
    vals = dv.cpu().numpy()
    exp = check_full(oracle, "angle", vals, P_, got)
    zeros = np.nonzero((vals == 0).all(axis=1))[0]
    np.testing.assert_array_equal(exp, zeros)           # the skyline is the zero tuples
    del vals
    for W in (2, 4, 8):
        bounds = np.linspace(0, n, W + 1).astype(np.int64)
        engs = [gpu_engine_factory(D, P_, "mr-angle") for _ in range(W)]
        sl = [slice(int(bounds[r]), int(bounds[r + 1])) for r in range(W)]
        out = dist_emulate(engs, [di[x] for x in sl], [dv[x] for x in sl])[0]
        for e in engs:
            e.close()
        np.testing.assert_array_equal(out["ls"], got[2])
        np.testing.assert_array_equal(out["sv"], got[3])
        np.testing.assert_array_equal(out["ids"], got[0])
        np.testing.assert_array_equal(out["org"], got[1])
    del dv, di
    torch.cuda.empty_cache()


def test_c4_angle_8d_anti_100m(gpu_engine_factory, oracle):
    """C4's per-GPU share at full size: 100M 8D tuples of the reference formula, P=16.
    Property: the global skyline is exactly the all-zero tuples, all in key 0
    (|L_0| = survivors_0 = their count, survivors_k = 0 otherwise); and the chunked oracle
    agrees on every id, origin, |L_k| and survivors_k."""
    D, P_, n = 8, 16, 100_000_000
    eng = gpu_engine_factory(D, P_, "mr-angle")
    dv, di = device_stream(eng, "anti_correlated", n, seed=1242)
    gi, go, ls, sv = query_dev(eng, dv, di)
    eng.close()
    zeros = torch.nonzero((dv == 0).all(dim=1)).flatten().cpu().numpy()
    np.testing.assert_array_equal(gi, zeros)
    assert (go == 0).all()
    assert ls[0] == len(zeros) and sv[0] == len(zeros) and (sv[1:] == 0).all()
    vals = dv.cpu().numpy()
    del dv, di
    torch.cuda.empty_cache()
    check_full(oracle, "angle", vals, P_, (gi, go, ls, sv))


def test_c4_8way_decomposition(gpu_engine_factory):
    """C4 as configured (100M 8D tuples over 8 GPUs): the whole stream split into 8 rank shards
    run through the multi-GPU step (one context per emulated rank, the collectives as device
    concatenation / sum) equals the one-GPU query: ids, origins, |L_k|, survivors_k.  Steps
    after the first replay the planned route: exactly ONE host read per rank per step."""
    D, P_, n, W = 8, 16, 100_000_000, 8
    eng = gpu_engine_factory(D, P_, "mr-angle")
    dv, di = device_stream(eng, "anti_correlated", n, seed=1242)
    gi, go, ls, sv = query_dev(eng, dv, di)
    eng.close()
    bounds = np.linspace(0, n, W + 1).astype(np.int64)
    sl = [slice(int(bounds[r]), int(bounds[r + 1])) for r in range(W)]
    engs = [gpu_engine_factory(D, P_, "mr-angle") for _ in range(W)]
    outs = dist_emulate(engs, [di[x] for x in sl], [dv[x] for x in sl], steps=3)
    for e in engs:
        e.close()
    for out in outs:
        np.testing.assert_array_equal(out["ids"], gi)
        np.testing.assert_array_equal(out["org"], go)
        np.testing.assert_array_equal(out["ls"], ls)
        np.testing.assert_array_equal(out["sv"], sv)
    for out in outs[1:]:
        assert out["attempts"] == 1
        assert out["syncs"] == [1] * W, out["syncs"]
    del dv, di
    torch.cuda.empty_cache()


# ---- MR-Grid with no queried tuple (advisor round 1) -------------------------------------
@pytest.mark.parametrize("mode", ["unqueried_cells", "grid_filter"])
def test_grid_no_candidates_large(mode, gpu_engine_factory):
    """More than 9M tuples and none of them reaches a queried partition: every MR-Grid key is
    >= P (reference semantics drop them, FlinkSkyline.java:152-154), or every tuple is
    removed by the dominance filter (:716-733).  The query must return an empty skyline on a
    fresh context (the fate pass's scan scratch is sized even with no candidate)."""
    import skyline
    D, P_, n = 8, 16, 9_500_000
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    vals = torch.randint(0, 1000, (n, D), device="cuda", generator=g).to(torch.float64)
    if mode == "unqueried_cells":
        vals[:, 4:] = 500.0 + vals[:, 4:] / 2           # dims 4..7 >= maxVal/2: key mask >= 16
        eng = skyline.SkylineEngine(D, P_, "mr-grid", 1000.0, 0)
    else:
        vals = 500.0 + vals / 2                          # every value >= maxVal/2: filtered out
        eng = skyline.SkylineEngine(D, P_, "mr-grid", 1000.0, 0, grid_filter=True)
    ids = torch.arange(n, dtype=torch.int64, device="cuda")
    gi, go, ls, sv = query_dev(eng, vals, ids)
    assert len(gi) == 0 and ls.sum() == 0 and sv.sum() == 0
    eng.close()


# ---- radix sort at scale ---------------------------------------------------------------
@pytest.mark.parametrize("n", [16_000_000, 3_000_000])
@pytest.mark.parametrize("pattern", ["compressed_runs", "partition_score_hash", "full_bytes"])
def test_radix_sort_at_scale(pattern, n, gpu_engine_factory):
    """The pipeline's onesweep radix sort (k_radix.hip) on 16M (u64, u32) pairs equals a
    stable torch sort: keys sorted, values follow their keys, ties keep index order.
    'compressed_runs' spreads 28 varying bits over 7 bytes in 4 runs, so the order-preserving
    bit compression (k_rs_compress / k_rs_expand) is active: the regression case of commit
    e3568d8 (corruption past ~65k keys).  16M keys use 4096-key tiles, 3M the 1024-key tiles
    of the query's candidate sorts."""
    eng = gpu_engine_factory(2, 4)
    g = torch.Generator(device="cuda")
    g.manual_seed(11)

    def bits(lo, width):
        return torch.randint(0, 1 << width, (n,), device="cuda", dtype=torch.int64, generator=g) << lo

    if pattern == "compressed_runs":
        keys = bits(0, 4) | bits(12, 8) | bits(28, 8) | bits(44, 8) | (1 << 62)
        exp_passes = 4
    elif pattern == "partition_score_hash":
        keys = bits(56, 4) | bits(24, 20) | bits(0, 16)   # few distinct scores: long equal runs
        exp_passes = None
    else:
        keys = bits(0, 62)
        exp_passes = 8
    vals = torch.arange(n, dtype=torch.int32, device="cuda")
    skeys, order = torch.sort(keys, stable=True)
    k = keys.clone()
    passes, _ = eng.profile_sort_dev(k, vals)
    eng.sync()
    if exp_passes is not None:
        assert passes == exp_passes
    assert torch.equal(k, skeys)
    assert torch.equal(vals.to(torch.int64), order)
    eng.close()


# ---- operator mirror: bad id after a trigger ------------------------------------------------
def test_run_job_bad_id_raises_in_stream_order(oracle):
    """A record whose id is not a Java long fails the job at processElement1 (Long.parseLong,
    FlinkSkyline.java:276), in stream order: the trigger before it is still answered."""
    from skyline.operators import run_job
    vals = oracle.synth(0, 2, 3000, seed=4)
    lines = [f"{i}," + ",".join(str(int(x)) for x in row) for i, row in enumerate(vals)]
    lines.insert(2000, "x7,1,2")
    results = []
    with pytest.raises(ValueError, match="NumberFormatException"):
        run_job(lines, [(1500, "1,1000")], algo="mr-dim", parallelism=2, dims=2, barrier="global", out=results)
    assert len(results) == 1
    import json
    assert json.loads(results[0])["query_id"] == "1"
