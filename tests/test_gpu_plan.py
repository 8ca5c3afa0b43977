"""The planned route (engine.hip pipe_run_planned): a query that repeats the last query's
small-set route (prefilter rounds, then the brute pair pass) with device-sized launches and
no host read before the final one, which verifies the route's assumptions and re-runs the
query synchronised on a miss.  Every answer is checked against the oracle
(FlinkSkyline.java:417-444 local BNL, :548-566 global BNL, :593-608 stats), whichever route
served it; counters[7] bit 3 = planned, bit 4 = a planned attempt missed."""
import os

import numpy as np
import pytest

from conftest import Oracle  # noqa: F401  (the checker)

pytestmark = pytest.mark.gpu

PLANNED, MISSED = 8, 16


def route(eng):
    _, cnt = eng.phases()
    return int(cnt[7]), int(cnt[1])


def check(eng, orc, vals, P, algo="angle"):
    ids, org = eng.query(vals)
    exp, keys, els, esv = orc.query_sfs(algo, vals, P)
    np.testing.assert_array_equal(ids, exp)
    np.testing.assert_array_equal(org, keys[exp])
    ls, sv = eng.stats()
    np.testing.assert_array_equal(ls, els)
    np.testing.assert_array_equal(sv, esv)
    return route(eng)


@pytest.mark.parametrize("dist,D,n,P", [(2, 8, 200000, 16), (0, 5, 200000, 16), (0, 4, 400000, 8), (1, 3, 100000, 8)])
def test_planned_equals_oracle(gpu_engine_factory, oracle, dist, D, n, P):
    """The first query learns the route, the next ones (other seeds, same shape) replay it."""
    eng = gpu_engine_factory(D, P, "mr-angle")
    r0, _ = check(eng, oracle, oracle.synth(dist, D, n, seed=11), P)
    assert not r0 & PLANNED
    planned = 0
    for seed in (12, 13, 14):
        r, m = check(eng, oracle, oracle.synth(dist, D, n, seed=seed), P)
        planned += bool(r & PLANNED)
    assert planned >= 2, "the small-set route was not replayed"
    eng.close()


def test_planned_prefilter_rounds(gpu_engine_factory, oracle):
    """A stream whose candidates pass the prefilter threshold (>= 4096 slots): the replay
    runs its prefilter rounds on device-sized launches."""
    eng = gpu_engine_factory(8, 16, "mr-angle")
    check(eng, oracle, oracle.synth(2, 8, 2500000, seed=21), 16)
    r, m = check(eng, oracle, oracle.synth(2, 8, 2500000, seed=22), 16)
    assert m >= 4096
    assert r & PLANNED
    eng.close()


def test_plan_miss_on_larger_stream(gpu_engine_factory, oracle):
    """Learned on a stream with few candidates, replayed on one with far more: the counts
    exceed the bounds, the query re-runs synchronised (and learns the new route)."""
    eng = gpu_engine_factory(5, 8, "mr-angle")
    check(eng, oracle, oracle.synth(1, 5, 20000, seed=31), 8)
    check(eng, oracle, oracle.synth(1, 5, 20000, seed=32), 8)
    r, _ = check(eng, oracle, oracle.synth(0, 5, 300000, seed=33), 8)
    assert r & MISSED and not r & PLANNED
    r, _ = check(eng, oracle, oracle.synth(0, 5, 300000, seed=34), 8)
    assert r & PLANNED
    eng.close()


def test_plan_miss_on_row_type(gpu_engine_factory, oracle):
    """Learned on integer rows (packed-u16 pair pass), replayed on f32-exact non-integer rows
    and on f64 rows: the compare type no longer holds, so the query re-runs."""
    eng = gpu_engine_factory(4, 8, "mr-angle")
    base = oracle.synth(0, 4, 100000, seed=41)
    check(eng, oracle, base, 8)
    r, _ = check(eng, oracle, base, 8)
    assert r & PLANNED                                    # planned replay of the integer route
    r, _ = check(eng, oracle, base + 0.5, 8)
    assert r & MISSED
    r, _ = check(eng, oracle, base + 0.1, 8)              # not exact in f32: the f64 pass
    assert r & MISSED and r & 1
    r, _ = check(eng, oracle, base + 0.3, 8)              # f64 route replayed
    assert r & PLANNED and r & 1
    eng.close()


def test_plan_nan_and_recovery(gpu_engine_factory, oracle):
    """A NaN tuple on the planned route is rejected as on the synchronised one; the context
    stays usable."""
    from skyline._abi import SkylineError
    eng = gpu_engine_factory(4, 8, "mr-angle")
    vals = oracle.synth(2, 4, 50000, seed=51)
    check(eng, oracle, vals, 8)
    check(eng, oracle, vals, 8)
    bad = vals.copy()
    bad[4321, 2] = np.nan
    with pytest.raises(SkylineError) as e:
        eng.query(bad)
    assert e.value.code == -4
    r, _ = check(eng, oracle, oracle.synth(2, 4, 50000, seed=52), 8)
    eng.close()


def test_plan_slot_overflow(gpu_engine_factory, oracle):
    """Candidate slots sized by a small stream (SKY_SLOT_MIN forces small slots); the planned
    replay on a stream with more candidates than slots counts the overflow on the device and
    re-runs with room for all."""
    os.environ["SKY_SLOT_MIN"] = "64"
    try:
        eng = gpu_engine_factory(5, 8, "mr-angle")
        check(eng, oracle, oracle.synth(1, 5, 20000, seed=61), 8)
        check(eng, oracle, oracle.synth(1, 5, 20000, seed=62), 8)
        r, m = check(eng, oracle, oracle.synth(0, 5, 200000, seed=63), 8)
        assert r & MISSED and m > 64
        eng.close()
    finally:
        del os.environ["SKY_SLOT_MIN"]


def test_plan_disabled_equals(gpu_engine_factory, oracle):
    """SKY_PLAN=0 (read per query) keeps every query on the synchronised route."""
    os.environ["SKY_PLAN"] = "0"
    try:
        eng = gpu_engine_factory(6, 16, "mr-angle")
        for seed in (71, 72):
            r, _ = check(eng, oracle, oracle.synth(4, 6, 200000, seed=seed), 16)
            assert not r & PLANNED
        eng.close()
    finally:
        del os.environ["SKY_PLAN"]


TINY = 32


@pytest.mark.parametrize("algo,dist,D,n,P", [("mr-dim", 0, 2, 1000000, 8), ("mr-angle", 1, 2, 100000, 8),
                                             ("mr-grid", 0, 2, 200000, 16), ("mr-grid", 1, 3, 100000, 8)])
def test_tiny_tail_equals_oracle(gpu_engine_factory, oracle, algo, dist, D, n, P):
    """Few final slots: the planned replay runs its whole tail (pruner slots, prefilter rounds,
    brute pass, fate tables, output counts, stats) as ONE workgroup (k_tiny_tail, counters[7]
    bit 5); every answer equals the oracle's, and equals SKY_TINY=0's launch-per-stage tail."""
    short = algo.split("-")[1]
    eng = gpu_engine_factory(D, P, algo)
    check(eng, oracle, oracle.synth(dist, D, n, seed=81), P, short)
    tiny = 0
    for seed in (82, 83, 84):
        r, _ = check(eng, oracle, oracle.synth(dist, D, n, seed=seed), P, short)
        tiny += bool(r & TINY)
        assert not (r & TINY) or r & PLANNED
    assert tiny >= 2, "the one-workgroup tail did not run"
    os.environ["SKY_TINY"] = "0"
    try:
        r, _ = check(eng, oracle, oracle.synth(dist, D, n, seed=85), P, short)
        assert not r & TINY
    finally:
        del os.environ["SKY_TINY"]
    eng.close()


def test_tiny_tail_prefilter_round(gpu_engine_factory, oracle):
    """C1's shape: >= 4096 candidate slots (kPrefilterMin), so the learned route has a prefilter
    round that the one-workgroup tail replays (in-LDS criterion minima, pick, compaction)."""
    eng = gpu_engine_factory(2, 8, "mr-dim")
    check(eng, oracle, oracle.synth(0, 2, 1000000, seed=91), 8, "dim")
    for seed in (92, 93):
        r, m = check(eng, oracle, oracle.synth(0, 2, 1000000, seed=seed), 8, "dim")
        assert m >= 4096 and r & TINY, (r, m)
    eng.close()


def test_tiny_tail_miss(gpu_engine_factory, oracle):
    """A stream whose final slots outgrow the tail's LDS even after the prefilter round it runs
    itself (3D independent, 20k tuples, ~600 slots): the tail raises its miss flag, nothing it
    wrote is used, the query re-runs synchronised with the oracle's answer, and the next queries
    (kTinyBlock) do not try the tail."""
    eng = gpu_engine_factory(3, 8, "mr-angle")
    check(eng, oracle, oracle.synth(0, 3, 20000, seed=81), 8)
    r, m = check(eng, oracle, oracle.synth(0, 3, 20000, seed=82), 8)
    assert r & MISSED and not r & TINY, (r, m)
    for seed in (83, 84):
        r, _ = check(eng, oracle, oracle.synth(0, 3, 20000, seed=seed), 8)
        assert r & PLANNED and not r & TINY, r
    eng.close()


def test_cand_fused_pass_equals_launch_chain(gpu_engine_factory, oracle):
    """The prefilter's pick / live test / scan / compaction as one launch with a decoupled look-back
    (k_cand_fused) after one k_cand_pick with one slot per thread (default, SKY_CAND_FUSED=2), with the
    pick redone in every workgroup (SKY_CAND_FUSED=1) and as the launch chain (SKY_CAND_FUSED=0, read per
    query): both routes
    (synchronised, planned) give the oracle's answer on a stream with prefilter rounds."""
    for knob in ("1", "2", "0"):
        os.environ["SKY_CAND_FUSED"] = knob
        try:
            eng = gpu_engine_factory(8, 16, "mr-angle")
            r0, m0 = check(eng, oracle, oracle.synth(2, 8, 2500000, seed=111), 16)
            r1, m1 = check(eng, oracle, oracle.synth(2, 8, 2500000, seed=112), 16)
            assert m0 >= 4096                       # learned with a prefilter round, replayed with it
            assert r1 & PLANNED
            eng.close()
        finally:
            del os.environ["SKY_CAND_FUSED"]


@pytest.mark.parametrize("algo,dist,D,n,P", [("mr-angle", 0, 5, 200000, 16), ("mr-grid", 1, 4, 1000000, 8)])
def test_tail_counts_equals_launch_chain(gpu_engine_factory, oracle, algo, dist, D, n, P):
    """The brute route's output counts, scan, stats and final read in one workgroup (k_tail_counts,
    default) and as four launches (SKY_TAIL_COUNTS=0, read per query): the oracle's answer on the
    synchronised and the planned brute route either way."""
    short = algo.split("-")[1]
    for knob in ("1", "0"):
        os.environ["SKY_TAIL_COUNTS"] = knob
        try:
            eng = gpu_engine_factory(D, P, algo)
            check(eng, oracle, oracle.synth(dist, D, n, seed=121), P, short)
            r, _ = check(eng, oracle, oracle.synth(dist, D, n, seed=122), P, short)
            assert r & PLANNED
            eng.close()
        finally:
            del os.environ["SKY_TAIL_COUNTS"]


@pytest.mark.parametrize("algo,dist,D,n,P,planned", [("mr-grid", 1, 4, 2500000, 8, True),
                                                      ("mr-angle", 1, 5, 2200000, 16, False)])
def test_out_epilogue_equals_launches(gpu_engine_factory, oracle, algo, dist, D, n, P, planned):
    """Past k_tail_counts' 1024 tiles, the brute route's stat reduce and final read run as the write
    pass's epilogue workgroups (default) or as k_stat_reduce + k_gather_words (SKY_OUT_EPILOGUE=0):
    the oracle's ids, origins and stats on the synchronised and the planned route either way."""
    short = algo.split("-")[1]
    for knob in ("1", "0"):
        os.environ["SKY_OUT_EPILOGUE"] = knob
        try:
            eng = gpu_engine_factory(D, P, algo)
            check(eng, oracle, oracle.synth(dist, D, n, seed=131), P, short)
            r, _ = check(eng, oracle, oracle.synth(dist, D, n, seed=132), P, short)
            assert bool(r & PLANNED) or not planned
            eng.close()
        finally:
            del os.environ["SKY_OUT_EPILOGUE"]


@pytest.mark.parametrize("algo,dist,D,n,P", [("mr-angle", 0, 5, 200000, 16), ("mr-grid", 1, 4, 2500000, 8)])
def test_finish_fold_equals_launch(gpu_engine_factory, oracle, algo, dist, D, n, P):
    """The planned brute route's finish (alive flags, per-partition counts) inside k_fate_tables
    (default) and as its own k_brute_finish launch (SKY_FINISH_FOLD=0): the oracle's ids, origins and
    stats either way, on the planned route."""
    short = algo.split("-")[1]
    for knob in ("1", "0"):
        os.environ["SKY_FINISH_FOLD"] = knob
        try:
            eng = gpu_engine_factory(D, P, algo)
            # (seed 141 -> 142 is a genuine plan miss at this shape: 34 % more slots than learned)
            check(eng, oracle, oracle.synth(dist, D, n, seed=131), P, short)
            r, _ = check(eng, oracle, oracle.synth(dist, D, n, seed=132), P, short)
            assert r & PLANNED
            check(eng, oracle, oracle.synth(dist, D, n, seed=142), P, short)   # (planned or a miss)
            eng.close()
        finally:
            del os.environ["SKY_FINISH_FOLD"]


MEASURE_LIB = os.path.join(__import__("conftest").PKG, "build_measure", "libskyline_hip.so")
_TINY_CAP_CHILD = r"""
import os, sys, numpy as np
sys.path.insert(0, sys.argv[1])
import skyline
from skyline._abi import SkylineError
vals, ids = skyline.synth_host("uniform", 2, 200000, seed=5)
eng = skyline.SkylineEngine(2, 8, "mr-dim", 1000.0, 0)
ref = eng.query(vals, ids)[0]                  # synchronised: learns the small-set plan
os.environ["SKY_TINY_CAP"] = sys.argv[2]       # the replay's tail gets a capacity far too small
try:
    eng.query(vals, ids)
    print("NO-ERROR", flush=True)
except SkylineError as e:
    print("CODE", e.code, str(e), flush=True)
del os.environ["SKY_TINY_CAP"]
os.environ["SKY_TINY"] = "0"                   # the same context still answers afterwards
got = eng.query(vals, ids)[0]
print("AFTER", int(np.array_equal(got, ref)), flush=True)
"""


@pytest.mark.parametrize("algo,dist,D,n,P", [("mr-grid", 1, 4, 2500000, 8), ("mr-dim", 0, 2, 1000000, 8)])
def test_sparse_write_pass_equals_dense(gpu_engine_factory, oracle, algo, dist, D, n, P):
    """After a run that selected < 1/32 of its tuples, the next run of the shape loads ids only in the
    selected lanes of the write pass (default) or every id first (SKY_SPARSE_OUT=0): the oracle's ids,
    origins and stats either way (the caller's ids here are not the tuple indices)."""
    short = algo.split("-")[1]
    for knob in ("1", "0"):
        os.environ["SKY_SPARSE_OUT"] = knob
        try:
            eng = gpu_engine_factory(D, P, algo)
            for seed in (131, 132, 133):
                vals = oracle.synth(dist, D, n, seed=seed)
                ids = np.arange(n, dtype=np.int64) * 7 + 1000
                got, org = eng.query(vals, ids)
                exp, keys, els, esv = oracle.query_sfs(short, vals, P)
                np.testing.assert_array_equal(got, ids[exp])
                np.testing.assert_array_equal(org, keys[exp])
                ls, sv = eng.stats()
                np.testing.assert_array_equal(ls, els)
                np.testing.assert_array_equal(sv, esv)
                assert len(exp) * 32 < n
            eng.close()
        finally:
            del os.environ["SKY_SPARSE_OUT"]


_EPOCH_CHILD = r"""
import hashlib, os, sys
sys.path.insert(0, sys.argv[1])
import skyline
eng = skyline.SkylineEngine(2, 8, "mr-dim", 1000.0, 0)
for dist, n, seed in [("uniform", 200000, 1), ("anti_correlated", 200000, 2), ("uniform", 17000000, 3),
                      ("correlated", 200000, 4), ("uniform", 200000, 5), ("uniform", 17000000, 6), ("uniform", 300000, 7)]:
    vals, ids = skyline.synth_host(dist, 2, n, seed=seed)
    got = eng.query(vals, ids)[0]
    print(hashlib.sha1(got.tobytes()).hexdigest(), flush=True)
"""


def test_sample_minima_tags_across_the_wrap():
    """The sample minima are tagged per query instead of filled (launch_select_pruners): a word of an
    earlier query must read as empty.  The measurement build starts the 16-bit query count at 65533
    (SKY_PMIN_EPOCH0), so the tags run 1, 0, then wrap (a fill) every two queries, over streams that pick
    their pruners in the filter (200k) and in k_pick_pruners (17M); every answer must equal the product
    build's with no wrap in sight."""
    import subprocess
    import sys
    from conftest import PKG
    if not os.path.exists(MEASURE_LIB):
        pytest.fail("build_measure/libskyline_hip.so missing: __graft_entry__.build() builds it")
    outs = []
    for lib, extra in ((MEASURE_LIB, {"SKY_PMIN_EPOCH0": "65533"}), (None, {})):
        env = dict(os.environ, **extra)
        if lib:
            env["SKYLINE_HIP_LIB"] = lib
        r = subprocess.run([sys.executable, "-c", _EPOCH_CHILD, PKG], env=env, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(r.stdout.split())
    assert len(outs[0]) == 7 and outs[0] == outs[1]


@pytest.mark.parametrize("algo,dist,D,n,P", [("mr-dim", 0, 2, 1000000, 8), ("mr-angle", 2, 8, 2500000, 16)])
def test_fill_embed_equals_fill_launch(gpu_engine_factory, oracle, algo, dist, D, n, P):
    """The query's zero / all-ones fills done by the sample pass's threads (default) or as their own
    k_fill_multi launch (SKY_FILL_EMBED=0): the oracle's ids, origins and stats on the synchronised and
    the planned route either way."""
    short = algo.split("-")[1]
    for knob in ("1", "0"):
        os.environ["SKY_FILL_EMBED"] = knob
        try:
            eng = gpu_engine_factory(D, P, algo)
            for seed in (151, 152, 153):
                check(eng, oracle, oracle.synth(dist, D, n, seed=seed), P, short)
            eng.close()
        finally:
            del os.environ["SKY_FILL_EMBED"]


@pytest.mark.parametrize("capspec", ["0:4", "6:16"])
def test_tiny_tail_guard_is_an_error_not_a_fault(capspec):
    """k_tiny_tail checks every global index it computes against the capacity the host passed
    for that array (the product build too): with the slot capacity (0:4) or the status words'
    capacity (6:16) forced tiny through the measurement build's SKY_TINY_CAP, the planned query
    must come back as SKY_E_HIP with a message -- no access past the capacity, no fault, nothing
    written into the caller's buffers -- and the context answers the next query correctly."""
    import subprocess
    import sys
    from conftest import PKG
    if not os.path.exists(MEASURE_LIB):
        pytest.fail("build_measure/libskyline_hip.so missing: __graft_entry__.build() builds it")
    env = dict(os.environ, SKYLINE_HIP_LIB=MEASURE_LIB)
    r = subprocess.run([sys.executable, "-c", _TINY_CAP_CHILD, PKG, capspec], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.strip().splitlines()
    assert lines[-2].startswith("CODE -2") and "device guard" in lines[-2], lines
    assert lines[-1] == "AFTER 1", lines
