"""The multi-GPU step with one host read (sky_dist_export_dev -> all-gather -> sky_dist_merge_dev
-> all-reduce -> sky_dist_finish), several ranks emulated on one GPU (one context per rank; the
collectives as device concatenation / sum, which is what RCCL moves between processes).  Every
decomposition must return the one-GPU query's ids, origins, |L_k| and survivors_k
(FlinkSkyline.java:548-566 merge rule, :593-608 integers), on both union routes (one pair kernel
over the blocks; the bounding-box pass of own tiles against union tiles for packed-u16, f32 and
f64 rows), through capacity regrowth, a planned-route miss (SKY_E_RETRY), NaN and empty shards."""
import numpy as np
import pytest
import torch
from conftest import dist_emulate

pytestmark = pytest.mark.gpu


def _split(vals, ids, W):
    b = np.linspace(0, len(vals), W + 1).astype(np.int64)
    dv = [torch.from_numpy(np.ascontiguousarray(vals[b[r]:b[r + 1]])).cuda() for r in range(W)]
    di = [torch.from_numpy(np.ascontiguousarray(ids[b[r]:b[r + 1]])).cuda() for r in range(W)]
    return dv, di


def _expect(factory, vals, ids, D, P, algo="mr-angle"):
    e = factory(D, P, algo)
    gi, go = e.query(vals, ids)
    ls, sv = e.stats()
    e.close()
    return gi, go, ls, sv


def _check(out, exp):
    np.testing.assert_array_equal(out["ids"], exp[0])
    np.testing.assert_array_equal(out["org"], exp[1])
    np.testing.assert_array_equal(out["ls"], exp[2])
    np.testing.assert_array_equal(out["sv"], exp[3])


@pytest.mark.parametrize("dist_id,D,W,algo", [(2, 8, 1, "mr-angle"), (2, 8, 4, "mr-angle"), (0, 2, 3, "mr-dim"),
                                              (1, 4, 2, "mr-grid"), (3, 4, 5, "mr-angle"), (4, 6, 2, "mr-angle")])
def test_dist_step_equals_one_query(dist_id, D, W, algo, gpu_engine_factory, oracle):
    n, P = 120000, 8
    vals = oracle.synth(dist_id, D, n, seed=70 + D + W)
    ids = np.arange(n, dtype=np.int64) * 3 + 11
    exp = _expect(gpu_engine_factory, vals, ids, D, P, algo)
    e_or, _, e_ls, e_sv = oracle.query_sfs(algo[3:], vals, P)
    np.testing.assert_array_equal(exp[2], e_ls)
    engs = [gpu_engine_factory(D, P, algo) for _ in range(W)]
    dv, di = _split(vals, ids, W)
    for out in dist_emulate(engs, di, dv, steps=3):
        _check(out, exp)
        np.testing.assert_array_equal(out["ids"], ids[e_or])
    for e in engs:
        e.close()


@pytest.mark.parametrize("scale,W", [(1.0, 4), (0.5, 2), (0.1, 3)])
def test_dist_union_bounding_box_route(scale, W, gpu_engine_factory, oracle, monkeypatch):
    """Own tiles vs union tiles (k_mbr_pairs with a separate y set, FULL test): packed u16
    (integers), f32 (halves) and f64 (tenths) rows; duplicates across ranks stay twins."""
    monkeypatch.setenv("SKY_DIST_BRUTE_PAIRS", "0")
    n, D, P = 160000, 6, 8
    vals = oracle.synth(3, D, n, seed=5 + W) * scale
    vals[n // 2:n // 2 + 500] = vals[:500]                 # the same vectors on two ranks
    ids = np.arange(n, dtype=np.int64)
    exp = _expect(gpu_engine_factory, vals, ids, D, P)
    e_or, _, _, _ = oracle.query_sfs("angle", vals, P)
    engs = [gpu_engine_factory(D, P) for _ in range(W)]
    dv, di = _split(vals, ids, W)
    for out in dist_emulate(engs, di, dv, steps=2):
        _check(out, exp)
        np.testing.assert_array_equal(out["ids"], e_or)
    assert [int(e.phases()[1][6]) for e in engs] == [1] * W      # the bounding-box route ran
    for e in engs:
        e.close()


def test_dist_std_anti_large_union(gpu_engine_factory):
    """std-anti 8D, 4 ranks x 300k: ~1M-vector union on the bounding-box route == one GPU."""
    D, P, W, per = 8, 16, 4, 300_000
    eng = gpu_engine_factory(D, P)
    vals = torch.empty((W * per, D), dtype=torch.float64, device="cuda")
    ids = torch.empty(W * per, dtype=torch.int64, device="cuda")
    eng.synth_dev("std_anti", W * per, vals, ids, seed=77)
    oi = torch.empty(W * per, dtype=torch.int64, device="cuda")
    oo = torch.empty(W * per, dtype=torch.int32, device="cuda")
    g = eng.query_dev(ids, vals, oi, oo, W * per)
    eng.sync()
    exp = (oi[:g].cpu().numpy(), oo[:g].cpu().numpy()) + eng.stats()
    eng.close()
    engs = [gpu_engine_factory(D, P) for _ in range(W)]
    outs = dist_emulate(engs, [ids[r * per:(r + 1) * per] for r in range(W)],
                        [vals[r * per:(r + 1) * per] for r in range(W)], steps=2)
    for out in outs:
        _check(out, exp)
    assert int(engs[0].phases()[1][6]) == 1
    for e in engs:
        e.close()


def test_dist_capacity_regrow(gpu_engine_factory, oracle):
    """cap 16 << exported vectors: every rank gets SKY_E_CAPACITY with the same need, the
    blocks are rewritten larger (no local re-run) and the step completes."""
    n, D, P, W = 60000, 4, 8, 3
    vals = oracle.synth(3, D, n, seed=9)
    ids = np.arange(n, dtype=np.int64)
    exp = _expect(gpu_engine_factory, vals, ids, D, P)
    engs = [gpu_engine_factory(D, P) for _ in range(W)]
    dv, di = _split(vals, ids, W)
    out = dist_emulate(engs, di, dv, cap=16)[0]
    assert out["attempts"] == 2 and out["cap"] > 16
    _check(out, exp)
    for e in engs:
        e.close()


def test_dist_retry_after_planned_miss(gpu_engine_factory, oracle):
    """Steps on a few-candidate stream learn the planned route; a step on a stream with far more
    candidates misses its bounds on the device: every rank gets SKY_E_RETRY, the missing rank
    re-runs synchronised, and the answer is exact."""
    D, P, W, n = 8, 16, 2, 200000
    a = oracle.synth(2, D, n, seed=21)
    b = oracle.synth(3, D, n, seed=22)
    b[: n // 2] = a[: n // 2]
    ids = np.arange(n, dtype=np.int64)
    engs = [gpu_engine_factory(D, P) for _ in range(W)]
    dv, di = _split(a, ids, W)
    outs = dist_emulate(engs, di, dv, steps=2)
    _check(outs[1], _expect(gpu_engine_factory, a, ids, D, P))
    assert outs[1]["syncs"] == [1] * W
    dv, di = _split(b, ids, W)
    out = dist_emulate(engs, di, dv)[0]
    assert out["attempts"] >= 2
    _check(out, _expect(gpu_engine_factory, b, ids, D, P))
    for e in engs:
        e.close()


def test_dist_nan_every_rank_reports_it(gpu_engine_factory, oracle):
    from skyline._abi import SkylineError
    from skyline.dist import block_words, stats_words
    n, D, P, W = 30000, 4, 8, 3
    vals = oracle.synth(0, D, n, seed=4)
    vals[n - 7, 2] = np.nan                               # only the last rank's shard
    ids = np.arange(n, dtype=np.int64)
    engs = [gpu_engine_factory(D, P) for _ in range(W)]
    dv, di = _split(vals, ids, W)
    cap = 4096
    send = [torch.empty(block_words(cap, D), dtype=torch.int64, device="cuda") for _ in range(W)]
    for r, e in enumerate(engs):
        e.dist_export_dev(di[r], dv[r], send[r], cap)
    recv = torch.cat(send)
    st = [torch.zeros(stats_words(P), dtype=torch.int64, device="cuda") for _ in range(W)]
    oi = torch.empty(n, dtype=torch.int64, device="cuda")
    oo = torch.empty(n, dtype=torch.int32, device="cuda")
    for r, e in enumerate(engs):
        e.dist_merge_dev(recv, W, r, cap, oi, oo, n, st[r])
    tot = torch.stack(st).sum(0)
    for e in engs:
        with pytest.raises(SkylineError) as ei:
            e.dist_finish(tot, n)
        assert ei.value.code == -4
    # the contexts stay usable: a clean step afterwards is exact
    vals[n - 7, 2] = 5.0
    dv, di = _split(vals, ids, W)
    _check(dist_emulate(engs, di, dv)[0], _expect(gpu_engine_factory, vals, ids, D, P))
    for e in engs:
        e.close()


def test_dist_empty_shard(gpu_engine_factory, oracle):
    n, D, P = 50000, 4, 8
    vals = oracle.synth(2, D, n, seed=8)
    ids = np.arange(n, dtype=np.int64)
    exp = _expect(gpu_engine_factory, vals, ids, D, P)
    engs = [gpu_engine_factory(D, P) for _ in range(3)]
    dv = [torch.from_numpy(vals[:20000]).cuda(), torch.empty((0, D), dtype=torch.float64, device="cuda"),
          torch.from_numpy(vals[20000:]).cuda()]
    di = [torch.from_numpy(ids[:20000]).cuda(), torch.empty(0, dtype=torch.int64, device="cuda"),
          torch.from_numpy(ids[20000:]).cuda()]
    for out in dist_emulate(engs, di, dv, steps=2):
        _check(out, exp)
    for e in engs:
        e.close()


def test_dist_route_large_small_large(gpu_engine_factory, oracle, monkeypatch):
    """A merge picks its union route from the previous step's |own| x |union|.  After a small step
    a large one on the same engines must not run the pair kernel over the large union: the kernel
    checks this step's sizes on the device, every rank gets SKY_E_RETRY through the all-reduced
    route-miss word, and the retry takes the bounding-box route (counters[6] = 1), exact."""
    monkeypatch.setenv("SKY_DIST_BRUTE_PAIRS", str(1 << 20))
    monkeypatch.setenv("SKY_PLAN", "0")                # no planned-route misses: a retry is the route's
    D, P, W = 6, 8, 3
    big = oracle.synth(3, D, 150000, seed=31)          # std-anti: large local skylines
    small = oracle.synth(1, D, 30000, seed=32)         # correlated: a handful of vectors
    engs = [gpu_engine_factory(D, P) for _ in range(W)]
    routes, cap = [], 4096
    for step, vals in enumerate((big, small, big)):
        ids = np.arange(len(vals), dtype=np.int64) + 1000 * step
        dv, di = _split(vals, ids, W)
        out = dist_emulate(engs, di, dv, cap=cap)[0]
        cap = out["cap"]
        _check(out, _expect(gpu_engine_factory, vals, ids, D, P))
        routes.append(int(engs[0].phases()[1][6]))
        if step == 2:
            assert out["attempts"] == 2                 # the route miss, then the sized route
        own, union = int(engs[0].phases()[1][3]), int(engs[0].phases()[1][5])
        assert (own * union > (1 << 20)) == (step != 1)
    assert routes == [1, 0, 1]
    for e in engs:
        e.close()
