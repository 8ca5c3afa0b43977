"""The bounding-box pruned all-pairs pass over large representative sets (k_mbr.hip):
both skyline levels (L_k, G) in one launch instead of the SFS rounds.  Forced onto small
sets (SKY_MBR_MIN=1, brute path off) it must equal the oracle for every row type (packed
u16, f32, f64 with +-0 twins / ties / infinities / negatives), every partitioner, the
single-partition callers (global merge of lists, the per-key operator state), and at scale
it must equal the round-based SFS (SKY_MBR=0) that the round-1 suite pinned."""
import numpy as np
import pytest

from test_gpu_engine import DISTS, check_vs_oracle, run_query

pytestmark = pytest.mark.gpu


@pytest.fixture
def force_mbr(monkeypatch):
    monkeypatch.setenv("SKY_MBR", "1")
    monkeypatch.setenv("SKY_MBR_MIN", "1")
    monkeypatch.setenv("SKY_BRUTE", "0")
    yield monkeypatch


@pytest.mark.parametrize("dist,D,P_,algo,n", [("std_anti", 8, 16, "mr-angle", 20000),
                                              ("std_anti", 3, 8, "mr-dim", 40000),
                                              ("anti_correlated", 4, 8, "mr-angle", 60000),
                                              ("anti_correlated", 8, 16, "mr-angle", 60000),
                                              ("uniform", 6, 256, "mr-angle", 60000),
                                              ("correlated", 4, 8, "mr-grid", 60000),
                                              ("mixed", 6, 8, "mr-angle", 200000),
                                              ("uniform", 1, 4, "mr-dim", 30000),
                                              ("std_anti", 16, 8, "mr-angle", 8000),
                                              ("std_anti", 12, 4, "mr-grid", 8000)])
@pytest.mark.parametrize("prefilter", ["1", "0"])
def test_mbr_vs_oracle(dist, D, P_, algo, n, prefilter, force_mbr, gpu_engine_factory, oracle):
    force_mbr.setenv("SKY_PREFILTER", prefilter)
    vals = oracle.synth(DISTS[dist], D, n, seed=300 + D + P_)
    check_vs_oracle(gpu_engine_factory, oracle, vals, P_, algo)
    force_mbr.setenv("SKY_SFS16", "0")                    # the same reps as f32 rows
    check_vs_oracle(gpu_engine_factory, oracle, vals, P_, algo)


def test_mbr_generic_rows(force_mbr, gpu_engine_factory, oracle):
    """f64 rows (values not exact in f32), score ties, +-0 twins, infinities, negatives."""
    rng = np.random.default_rng(11)
    cases = []
    v = rng.integers(0, 50, size=(30000, 4)).astype(np.float64) + 0.1   # not f32-exact -> f64 rows
    cases.append(v)
    v = rng.integers(0, 8, size=(30000, 5)).astype(np.float64)          # many equal scores
    cases.append(v)
    v = rng.integers(-3, 3, size=(20000, 3)).astype(np.float64) * 0.5   # negatives, +-0
    v[v == 0] = np.where(rng.random((v == 0).sum()) < 0.5, -0.0, 0.0)
    cases.append(v)
    # integer data (the packed-u16 candidate) with -0.0 / +0.0 twins: MR-Angle keys read the sign
    # bit, so the twins land in different partitions; -0.0 must keep the rows off the u16 path,
    # whose distinct-vector test would make the twins dominate each other
    v = rng.integers(0, 6, size=(30000, 4)).astype(np.float64)
    v[v == 0] = np.where(rng.random((v == 0).sum()) < 0.5, -0.0, 0.0)
    cases.append(v)
    v = rng.integers(0, 100, size=(20000, 3)).astype(np.float64)
    v[::97, 1] = np.inf
    v[5::89, 2] = -np.inf
    cases.append(v)
    for vals in cases:
        for algo, P_ in (("mr-angle", 8), ("mr-dim", 4)):
            check_vs_oracle(gpu_engine_factory, oracle, vals, P_, algo)


def test_mbr_single_partition_callers(force_mbr, gpu_engine_factory, oracle):
    """sky_global_merge (one partition, given origins) and the per-key operator state
    (sky_part_insert: local level only) through the pruned pass."""
    from skyline.operators import _LocalPart
    rng = np.random.default_rng(3)
    eng = gpu_engine_factory(4, 8)
    lists_v, lists_i, pids = [], [], []
    off = 0
    for k in range(5):
        nk = int(rng.integers(1000, 6000))
        v = oracle.synth(3, 4, nk, seed=40 + k)
        lists_v.append(v)
        lists_i.append(np.arange(off, off + nk, dtype=np.int64))
        pids.append(k)
        off += nk
    gids, gorg = eng.global_merge(pids, lists_i, lists_v)
    allv = np.concatenate(lists_v)
    alli = np.concatenate(lists_i)
    exp, _, _, _ = oracle.query_sfs("dim", allv, 1)
    assert sorted(gids.tolist()) == sorted(alli[exp].tolist())
    vals = oracle.synth(3, 4, 23000, seed=6)
    ids = np.arange(len(vals), dtype=np.int64) + 7
    part = _LocalPart(eng, 3)
    for s in range(0, len(vals), 5000):
        part.insert(ids[s:s + 5000], vals[s:s + 5000])
        got_ids, got_vals = part.snapshot()
        exp, _, _, _ = oracle.query_sfs("dim", vals[:s + 5000], 1)
        np.testing.assert_array_equal(got_ids, ids[exp])
        np.testing.assert_array_equal(got_vals, vals[exp])
    part.close()
    eng.close()


@pytest.mark.parametrize("dist,D,n", [("std_anti", 8, 300000), ("std_anti", 5, 400000),
                                      ("uniform", 6, 400000), ("anti_correlated", 4, 400000)])
def test_mbr_equals_sfs_at_scale(dist, D, n, gpu_engine_factory, oracle, monkeypatch):
    """Beyond the oracle's reach: the pruned all-pairs pass (default for >= 16384 reps) and
    the round-based SFS give the same ids, origins and |L_k| / survivors_k."""
    vals = oracle.synth(DISTS[dist], D, n, seed=700 + D)
    res = []
    for mbr in ("1", "0"):
        monkeypatch.setenv("SKY_MBR", mbr)
        (ids, org), (ls, sv) = run_query(gpu_engine_factory, vals, 16, "mr-angle")
        res.append((ids, org, ls, sv))
    for a, b in zip(res[0], res[1]):
        np.testing.assert_array_equal(a, b)


MEASURE_LIB = __import__("os").path.join(__import__("conftest").PKG, "build_measure", "libskyline_hip.so")
_QCAP_CHILD = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import skyline
from skyline._abi import SkylineError
n, D = 60000, 8
vals, ids = skyline.synth_host("std_anti", D, n, seed=3)
eng = skyline.SkylineEngine(D, 16, "mr-angle", 1000.0, 0)
try:
    eng.query(vals, ids)
    print("NO-ERROR")
except SkylineError as e:
    print("CODE", e.code, str(e))
"""


def test_mbr_queue_overflow_is_an_error_not_a_fault():
    """k_mbr_order guards its work queue on the device: with the queue's capacity forced tiny
    (SKY_MBR_QCAP, a knob of the measurement build only) the query must come back as SKY_E_HIP
    with a message -- no item written past the queue, no pair pass over a partial queue."""
    import os
    import subprocess
    import sys
    from conftest import PKG
    if not os.path.exists(MEASURE_LIB):
        pytest.fail("build_measure/libskyline_hip.so missing: __graft_entry__.build() builds it")
    env = dict(os.environ, SKYLINE_HIP_LIB=MEASURE_LIB, SKY_MBR_QCAP="8", SKY_MBR="1", SKY_MBR_MIN="1",
               SKY_BRUTE="0", SKY_PLAN="0")
    r = subprocess.run([sys.executable, "-c", _QCAP_CHILD, PKG], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    out = r.stdout.strip().splitlines()[-1]
    assert out.startswith("CODE -2") and "work items outgrew their queue" in out, out


_YT_CHILD = r"""
import os, sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
sys.path.insert(0, sys.argv[2])
import skyline
from conftest import dist_emulate
out = {}
def one(tag, dist, D, n, seed, P):
    vals, ids = skyline.synth_host(dist, D, n, seed=seed)
    for yt in ("1", "2"):
        os.environ["SKY_MBR_YT"] = yt
        eng = skyline.SkylineEngine(D, P, "mr-angle", 1000.0, 0)
        gi, go = eng.query(vals, ids)
        ls, sv = eng.stats()
        reps = int(eng.phases()[1][2])
        eng.close()
        out[f"{tag}_{yt}_ids"], out[f"{tag}_{yt}_org"] = gi, go
        out[f"{tag}_{yt}_ls"], out[f"{tag}_{yt}_sv"] = ls, sv
        out[f"{tag}_{yt}_reps"] = np.array([reps])
one("small", "std_anti", 8, 60000, 360, 16)
one("big", "std_anti", 8, 300000, 708, 16)
one("uni", "uniform", 6, 400000, 706, 16)
one("odd", "std_anti", 5, 150001, 505, 8)
# the multi-GPU union route (own tiles vs union tiles, the full test): 2 emulated ranks
os.environ["SKY_DIST_BRUTE_PAIRS"] = "0"
D, n = 8, 80000
vals, ids = skyline.synth_host("std_anti", D, n, seed=77)
dv, di = torch.from_numpy(vals).cuda(), torch.from_numpy(ids).cuda()
for yt in ("1", "2"):
    os.environ["SKY_MBR_YT"] = yt
    engs = [skyline.SkylineEngine(D, 16, "mr-angle", 1000.0, 0) for _ in range(2)]
    r = dist_emulate(engs, [di[:n // 2], di[n // 2:]], [dv[:n // 2], dv[n // 2:]], steps=2)[-1]
    route = int(engs[0].phases()[1][6])
    for e in engs:
        e.close()
    out[f"dist_{yt}_ids"], out[f"dist_{yt}_org"], out[f"dist_{yt}_ls"], out[f"dist_{yt}_sv"] = r["ids"], r["org"], r["ls"], r["sv"]
    out[f"dist_{yt}_route"] = np.array([route])
np.savez(sys.argv[3], **out)
print("DONE", flush=True)
"""


def test_mbr_two_tile_items_equal_one_tile_items(tmp_path, oracle):
    """The pair pass's two-y-tile work items (YT = 2, the default above 65536 y tiles, i.e. ~4.2M
    reps) forced at test sizes through the measurement build's SKY_MBR_YT: the ids, origins,
    |L_k| and survivors_k equal the one-tile items on std-anti 8D 60k / 300k, uniform 6D 400k,
    a stream with an odd y-tile count (the last unit holds one tile), and the multi-GPU union
    route (own tiles vs union tiles, the full test, gmerge); the 60k case also equals the oracle."""
    import os
    import subprocess
    import sys
    from conftest import PKG, REPO
    if not os.path.exists(MEASURE_LIB):
        pytest.fail("build_measure/libskyline_hip.so missing: __graft_entry__.build() builds it")
    npz = str(tmp_path / "yt.npz")
    env = dict(os.environ, SKYLINE_HIP_LIB=MEASURE_LIB, SKY_MBR="1", SKY_MBR_MIN="1", SKY_BRUTE="0")
    r = subprocess.run([sys.executable, "-c", _YT_CHILD, PKG, os.path.join(REPO, "tests"), npz], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "DONE" in r.stdout, r.stderr[-3000:]
    z = np.load(npz)
    for tag in ("small", "big", "uni", "odd", "dist"):
        for f in ("ids", "org", "ls", "sv"):
            np.testing.assert_array_equal(z[f"{tag}_1_{f}"], z[f"{tag}_2_{f}"], err_msg=f"{tag} {f}")
    tiles = [(int(z[f"{t}_1_reps"][0]) + 63) // 64 for t in ("small", "big", "uni", "odd")]
    assert any(t % 2 == 1 for t in tiles), tiles              # a unit with one tile in it
    assert int(z["dist_1_route"][0]) == 1                      # the bounding-box union route ran
    import skyline
    vals, _ = skyline.synth_host("std_anti", 8, 60000, seed=360)
    exp, keys, els, esv = oracle.query_sfs("angle", vals, 16)
    np.testing.assert_array_equal(z["small_2_ids"], exp)
    np.testing.assert_array_equal(z["small_2_org"], keys[exp])
    np.testing.assert_array_equal(z["small_2_ls"], els)
    np.testing.assert_array_equal(z["small_2_sv"], esv)
