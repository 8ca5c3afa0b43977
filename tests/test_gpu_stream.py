"""Continuous queries (sky_stream_*) against the oracle.

Landmark window (the reference's semantics, FlinkSkyline.java:265-316 + :417-444): after
any sequence of micro-batch appends, a query equals the oracle's BNL job over every tuple
appended so far (skyline id set, |L_k|, survivors_k).  Sliding window (labelled
extension): a query equals the oracle over the last W appended tuples."""
import numpy as np
import pytest
import torch

from conftest import golden_streams, load_golden

pytestmark = pytest.mark.gpu


def _check(orc, algo, vals, ids, P_, got_ids, eng):
    exp, _, els, esv = orc.query_bnl(algo, vals, ids, P_)
    assert sorted(got_ids.tolist()) == sorted(exp.tolist())
    ls, sv = eng.stats()
    assert (ls == els).all() and (sv == esv).all()


@pytest.mark.parametrize("path", [p for p in golden_streams() if "4d" in p or "2d" in p or "6d" in p],
                         ids=lambda p: p.split("stream_")[-1][:-4])
def test_landmark_stream_matches_prefix_queries(gpu_engine_factory, oracle, path):
    import skyline
    g = load_golden(path)
    vals, ids = g["values"], g["ids"].astype(np.int64)
    n, D = vals.shape
    P_ = 8
    eng = gpu_engine_factory(D, P_, "mr-angle")
    st = skyline.SkylineStream(eng, 0)
    rng = np.random.default_rng(n + D)
    pos = 0
    checks = 0
    while pos < n:
        b = int(min(n - pos, rng.integers(1, max(2, n // 8))))
        st.append(ids[pos:pos + b], vals[pos:pos + b])
        pos += b
        if rng.random() < 0.25 or pos == n:
            got, org = st.query()
            assert (np.diff(got) > 0).all()          # arrival order (ids increase along the stream)
            _check(oracle, "angle", vals[:pos], ids[:pos], P_, got, eng)
            checks += 1
            resident, appended = st.size()
            assert appended == pos and resident <= pos
    assert checks >= 2
    st.close()
    eng.close()


@pytest.mark.parametrize("W", [1000, 7777])
def test_sliding_window_matches_window_queries(gpu_engine_factory, oracle, W):
    import skyline
    g = load_golden([p for p in golden_streams() if "anti_correlated_3d" in p][0])
    vals, ids = g["values"], g["ids"].astype(np.int64)
    n, D = vals.shape
    eng = gpu_engine_factory(D, 8, "mr-dim")
    st = skyline.SkylineStream(eng, W)
    rng = np.random.default_rng(W)
    pos = 0
    while pos < n:
        b = int(min(n - pos, rng.integers(1, 3 * W // 2)))
        st.append(ids[pos:pos + b], vals[pos:pos + b])
        pos += b
        if rng.random() < 0.4 or pos == n:
            got, _ = st.query()
            lo = max(0, pos - W)
            _check(oracle, "dim", vals[lo:pos], ids[lo:pos], 8, got, eng)
            assert st.size()[0] == pos - lo
    st.close()
    eng.close()


def test_stream_device_appends_match_whole_query(gpu_engine_factory):
    """Device-resident micro-batches (C5 shape: 6D mixed blocks, P=8): the landmark stream's
    answer at each trigger equals a whole-prefix sky_query_dev on the same device rows."""
    import skyline
    n, D, P_ = 2_000_000, 6, 8
    eng = gpu_engine_factory(D, P_, "mr-angle")
    dv = torch.empty((n, D), dtype=torch.float64, device="cuda")
    di = torch.empty(n, dtype=torch.int64, device="cuda")
    eng.synth_dev("mixed", n, dv, di, seed=5)
    st = skyline.SkylineStream(eng, 0)
    oi = torch.empty(n, dtype=torch.int64, device="cuda")
    oo = torch.empty(n, dtype=torch.int32, device="cuda")
    qi = torch.empty(n, dtype=torch.int64, device="cuda")
    qo = torch.empty(n, dtype=torch.int32, device="cuda")
    step = 50_000
    for pos in range(0, n, step):
        st.append_dev(di[pos:pos + step], dv[pos:pos + step])
        if (pos + step) % 500_000 == 0:
            g = st.query_dev(oi, oo, n)
            ls, sv = eng.stats()
            m = pos + step
            h = eng.query_dev(di[:m], dv[:m], qi, qo, m)
            ls2, sv2 = eng.stats()
            assert g == h and torch.equal(oi[:g], qi[:h]) and torch.equal(oo[:g], qo[:h])
            assert (ls == ls2).all() and (sv == sv2).all()
    st.close()
    eng.close()


@pytest.mark.parametrize("W", [0, 5000])
def test_stream_reserve_then_queries(gpu_engine_factory, oracle, W):
    """sky_stream_reserve (SkylineStream.reserve) before the stream, again mid-stream with tuples
    resident, and a stream that outgrows its reservation: every host-view query still equals the
    oracle over the window (landmark: every tuple so far)."""
    import skyline
    g = load_golden([p for p in golden_streams() if "anti_correlated_4d" in p][0])
    vals, ids = g["values"], g["ids"].astype(np.int64)
    n, D = vals.shape
    eng = gpu_engine_factory(D, 8, "mr-angle")
    st = skyline.SkylineStream(eng, W)
    st.reserve(max(64, n // 4))                     # smaller than the stream: it has to grow
    pos, step = 0, max(1, n // 10)
    while pos < n:
        b = min(step, n - pos)
        st.append(ids[pos:pos + b], vals[pos:pos + b])
        pos += b
        if pos >= n // 2 and pos - b < n // 2:
            st.reserve(n)                           # again, with tuples resident
        k = st.query_host_view()
        got_ids, _ = st.view()
        lo = max(0, pos - W) if W else 0
        _check(oracle, "angle", vals[lo:pos], ids[lo:pos], 8, got_ids[:k].copy(), eng)
    st.close()
    eng.close()


@pytest.mark.parametrize("path", [p for p in golden_streams() if "anti_correlated_4d" in p or "uniform_6d" in p
                                  or "uniform_2d" in p], ids=lambda p: p.split("stream_")[-1][:-4])
def test_landmark_vectors_count_distinct_local_skyline_vectors(gpu_engine_factory, oracle, path):
    """sky_stream_vectors after a query = the distinct (key, row) vectors of the local skylines L_k
    over every tuple so far (the state the next query starts from), and + the rows appended since
    before the next query.  The inert holes of k_ls_new_reps' publishing races are not counted."""
    import skyline
    g = load_golden(path)
    vals, ids = g["values"], g["ids"].astype(np.int64)
    n, D = vals.shape
    P_ = 8
    eng = gpu_engine_factory(D, P_, "mr-angle")
    st = skyline.SkylineStream(eng, 0)
    cuts = sorted({n // 5, n // 2, (4 * n) // 5, n})
    pos = 0
    for cut in cuts:
        st.append(ids[pos:cut], vals[pos:cut])
        assert st.vectors() >= cut - pos
        pos = cut
        st.query()
        _, keys, _, _, inl = oracle.query_sfs_chunked("angle", vals[:pos], P_)
        loc = np.nonzero(inl)[0]
        distinct = len({(int(keys[i]),) + tuple(vals[i].view(np.int64).tolist()) for i in loc})
        assert st.vectors() == distinct, (pos, st.vectors(), distinct)
    st.append(ids[:7], vals[:7])                   # appended rows count until the next query
    assert st.vectors() == distinct + 7
    st.close()
    eng.close()


@pytest.mark.parametrize("W", [0, 5000])
def test_stream_query_async_then_wait(gpu_engine_factory, oracle, W):
    """sky_stream_query_async returns the integers (skyline size, sky_global_stats) and leaves the
    id copy in flight; appends go on meanwhile; after sky_stream_wait the host view holds the same
    ids as the oracle's answer for that trigger (the copy did not see the later appends)."""
    import skyline
    g = load_golden([p for p in golden_streams() if "anti_correlated_6d" in p][0])
    vals, ids = g["values"], g["ids"].astype(np.int64)
    n, D = vals.shape
    eng = gpu_engine_factory(D, 8, "mr-angle")
    st = skyline.SkylineStream(eng, W)
    st.reserve(n)
    pos, step = 0, max(1, n // 6)
    while pos < n:
        b = min(step, n - pos)
        st.append(ids[pos:pos + b], vals[pos:pos + b])
        pos += b
        k = st.query_async_host_view()
        ls, sv = eng.stats()
        lo = max(0, pos - W) if W else 0
        exp, _, els, esv = oracle.query_bnl("angle", vals[lo:pos], ids[lo:pos], 8)
        assert k == len(exp) and (ls == els).all() and (sv == esv).all()
        if pos < n:                                 # the next micro-batch while the copy runs
            b2 = min(step, n - pos)
            st.append(ids[pos:pos + b2], vals[pos:pos + b2])
        ms = st.wait()
        assert ms >= 0.0
        got, _ = st.view()
        assert sorted(got[:k].tolist()) == sorted(exp.tolist())
        if pos < n:
            pos += b2
    assert st.wait() == 0.0                         # nothing pending
    st.close()
    eng.close()
