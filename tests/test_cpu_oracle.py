"""CPU-only checks: the oracle against every golden vector (pinning it), its
internal cross-checks (BNL == SFS == brute-force definition, order/partition
invariance), and the host pieces of the product that need no GPU."""
import math
import os
import struct

import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from conftest import GOLDEN, golden_streams, load_golden


# ---- fdlibm atan2 (MR-Angle) ------------------------------------------------------
FDLIBM_HEX = {
    0: ["3FDDAC670561BB4F", "3FE921FB54442D18", "3FEF730BD281F69B", "3FF921FB54442D18"],
    1: ["3C7A2B7F222F65E2", "3C81A62633145C07", "3C7007887AF0CBBD", "3C91A62633145C07"],
    2: ["3FD555555555550D", "BFC999999998EBC4", "3FC24924920083FF", "BFBC71C6FE231671", "3FB745CDC54C206E",
        "BFB3B0F2AF749A6D", "3FB10D66A0D03D51", "BFADDE2D52DEFD9A", "3FA97B4B24760DEB", "BFA2B4442C6A6C2F",
        "3F90AD3AE322DA11"],
}


def test_fdlibm_constants_match_published_hex(oracle):
    for table, hexes in FDLIBM_HEX.items():
        t = oracle.L.orc_fdlibm_table(table)
        for i, h in enumerate(hexes):
            assert struct.pack(">d", t[i]).hex().upper() == h


def test_fdlibm_atan2_vs_v8_golden(oracle):
    """Bit-exact against V8's independent fdlibm port, except the documented
    FreeBSD fix (|y/x| > 2^60 with x < 0: `m &= 1`) that the JDK's original
    fdlibm 5.3 does not carry."""
    z = np.load(os.path.join(GOLDEN, "atan2_v8_fdlibm.npz"))
    bad = []
    for (y, x), ref in zip(z["yx"], z["atan2"]):
        got = oracle.L.orc_fdlibm_atan2(float(y), float(x))
        if struct.pack("<d", got) != struct.pack("<d", float(ref)):
            bad.append((y, x))
    for y, x in bad:
        hy = struct.unpack("<q", struct.pack("<d", abs(y)))[0] >> 52
        hx = struct.unpack("<q", struct.pack("<d", abs(x)))[0] >> 52
        assert x < 0 and hy - hx > 60, (y, x)
    assert len(bad) <= 3


# ---- golden streams ----------------------------------------------------------------
@pytest.mark.parametrize("path", golden_streams(), ids=lambda p: os.path.basename(p)[7:-4])
def test_oracle_keys_and_query_match_golden(path, oracle):
    g = load_golden(path)
    vals, ids = g["values"], g["ids"]
    for algo in ("dim", "grid", "angle"):
        for P in (4, 8, 16):
            np.testing.assert_array_equal(oracle.keys(algo, vals, P), g[f"keys_{algo}_{P}"].astype(np.int32))
            gids, _, ls, sv = oracle.query_bnl(algo, vals, ids, P)
            np.testing.assert_array_equal(np.sort(gids), g[f"gsky_{algo}_{P}"])
            np.testing.assert_array_equal(ls, g[f"lsz_{algo}_{P}"])
            np.testing.assert_array_equal(sv, g[f"surv_{algo}_{P}"])
            sfs, _, ls2, sv2 = oracle.query_sfs(algo, vals, P)
            np.testing.assert_array_equal(sfs, g[f"gsky_{algo}_{P}"])
            np.testing.assert_array_equal(ls2, ls)
            np.testing.assert_array_equal(sv2, sv)


def test_pdf_p15_kat_correlated_2d_is_all_zero(oracle):
    """project_documentation.pdf p.15: the correlated 2D skyline is [0,0] duplicates."""
    vals = np.load(os.path.join(GOLDEN, "kat_pdf15_correlated_2d.npz"))["values"].astype(np.float64)
    sky = oracle.brute(vals)
    assert len(sky) > 1 and np.all(vals[sky] == 0)
    gids, _, _, _ = oracle.query_bnl("angle", vals, np.arange(len(vals)), 8, 10000.0)
    assert sorted(gids.tolist()) == sky.tolist()


def test_reference_8d_anti_skyline_is_the_zero_vectors(oracle):
    """at D>=4 the reference formula's skyline is exactly the all-zero tuples."""
    g = load_golden(os.path.join(GOLDEN, "stream_anti_correlated_8d.npz"))
    zeros = np.nonzero(np.all(g["values"] == 0, axis=1))[0]
    np.testing.assert_array_equal(g["gsky_angle_16"], zeros)


# ---- oracle self-consistency ---------------------------------------------------------
vectors = st.lists(st.lists(st.integers(0, 6), min_size=3, max_size=3), min_size=0, max_size=60)


@settings(max_examples=60, deadline=None)
@given(rows=vectors, algo=st.sampled_from(["dim", "grid", "angle"]), P=st.sampled_from([1, 2, 4, 8]), rnd=st.randoms())
def test_bnl_equals_definition_and_is_order_invariant(rows, algo, P, rnd, oracle):
    vals = np.asarray(rows, np.float64).reshape(-1, 3)
    n = len(vals)
    ids = np.arange(n, dtype=np.int64)
    g1, _, ls1, sv1 = oracle.query_bnl(algo, vals, ids, P, 6.0, sem=1, buffer_size=3)
    perm = list(range(n))
    rnd.shuffle(perm)
    perm = np.asarray(perm, np.int64)
    g2, _, ls2, sv2 = oracle.query_bnl(algo, vals[perm] if n else vals, ids[perm] if n else ids, P, 6.0, sem=1,
                                       buffer_size=7)
    assert sorted(g1.tolist()) == sorted(g2.tolist())
    np.testing.assert_array_equal(ls1, ls2)
    np.testing.assert_array_equal(sv1, sv2)
    if n:
        assert sorted(g1.tolist()) == oracle.brute(vals).tolist()   # complete semantics == definition


def test_duplicates_never_dominate_each_other(oracle):
    vals = np.array([[1, 1], [1, 1], [0, 2], [0, 2], [2, 0], [1, 2]], np.float64)
    g, _, _, _ = oracle.query_bnl("dim", vals, np.arange(6), 2, 3.0)
    assert sorted(g.tolist()) == [0, 1, 2, 3, 4]


def test_grid_reference_semantics_drops_unqueried_keys(oracle):
    """MR-Grid keys >= P are never queried (FlinkSkyline.java:152-154, 775-788)."""
    vals = oracle.synth(0, 4, 20000, seed=1)
    keys = oracle.keys("grid", vals, 8)
    assert keys.max() >= 8
    g_ref, _, _, _ = oracle.query_bnl("grid", vals, np.arange(len(vals)), 8, 1000.0, sem=0)
    assert np.all(keys[g_ref] < 8)
    g_all, _, _, _ = oracle.query_bnl("grid", vals, np.arange(len(vals)), 8, 1000.0, sem=1)
    assert len(g_all) >= len(g_ref)


def test_java_int_narrowing_and_clamps(oracle):
    vals = np.array([[-5.0, 1.0], [1e300, 1.0], [999.999, 0.0], [1000.0, 0.0], [np.inf, 0.0]], np.float64)
    assert oracle.keys("dim", vals, 8).tolist() == [0, 7, 7, 7, 7]


# ---- host pieces of the product (no GPU needed) ----------------------------------------
def test_library_exports_every_header_symbol():
    import skyline
    from skyline import _abi
    L = skyline.lib()
    names = _abi.exported_symbols_in_header()
    assert len(names) >= 30
    for name in names:
        assert hasattr(L, name), name
    assert set(names) == set(_abi.SIGNATURES), set(names) ^ set(_abi.SIGNATURES)
    assert b"gfx950" in L.sky_version()


def test_ctx_create_without_gpu_fails_loudly():
    import skyline
    from skyline._abi import SkylineError
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(SkylineError) as e:
        skyline.SkylineEngine(2, 4)
    assert e.value.code == -6


def test_subtask_device_map():
    """HipSkylineOperators puts subtask i's context on sky_device_for_subtask(i, sky_device_count()):
    round-robin over the node's GPUs (the reference runs `parallelism` subtasks over 2p keys,
    FlinkSkyline.java:66,76,138).  No GPU here: zero devices, not an error."""
    import ctypes
    import torch
    import skyline
    from skyline._abi import SKY_E_ARG, SKY_OK
    L = skyline.lib()
    n = ctypes.c_int32(-1)
    assert L.sky_device_count(ctypes.byref(n)) == SKY_OK
    if not torch.cuda.is_available():
        assert n.value == 0
    dev = ctypes.c_int32(-1)
    got = []
    for sub in range(12):
        assert L.sky_device_for_subtask(sub, 8, ctypes.byref(dev)) == SKY_OK
        got.append(dev.value)
    assert got == [0, 1, 2, 3, 4, 5, 6, 7, 0, 1, 2, 3]
    for sub in range(5):                                 # one GPU: every subtask on device 0
        assert L.sky_device_for_subtask(sub, 1, ctypes.byref(dev)) == SKY_OK and dev.value == 0
    assert L.sky_device_for_subtask(3, 0, ctypes.byref(dev)) == SKY_E_ARG    # no device: the caller must not create
    assert L.sky_device_for_subtask(-1, 8, ctypes.byref(dev)) == SKY_E_ARG
    from skyline.operators import device_for_subtask
    assert [device_for_subtask(s, 3) for s in range(7)] == [0, 1, 2, 0, 1, 2, 0]


def test_host_generator_matches_oracle(oracle):
    import skyline
    for dist in range(5):
        for D in (1, 2, 3, 4, 5, 8, 16):
            hv, hi = skyline.synth_host(dist, D, 3000, seed=17, id0=99)
            np.testing.assert_array_equal(hv, oracle.synth(dist, D, 3000, seed=17, id0=99))
            np.testing.assert_array_equal(hi, np.arange(99, 3099))


def test_generator_restates_reference_formula_shape(oracle):
    """Reference anti-correlated formula: target<0 w.p. ~22/42/44% at 4/6/8D."""
    for D, frac in ((4, 0.22), (6, 0.42), (8, 0.44)):
        v = oracle.synth(2, D, 40000, seed=D)
        z = np.mean(np.all(v == 0, axis=1))
        assert abs(z - frac) < 0.03, (D, z)


def test_java_format_4f():
    from skyline.operators import java_format_4f
    assert java_format_4f(0.25) == "0.2500"
    assert java_format_4f(0.12345) == "0.1235"          # HALF_UP on the shortest repr
    assert java_format_4f(0.7378999999999999) == "0.7379"
    assert java_format_4f(2 / 3) == "0.6667"
    assert java_format_4f(0.0) == "0.0000"


def test_multithreaded_bnl_equals_single(oracle):
    """The multi-core CPU baseline (one thread per subtask) gives the same answer."""
    for dist, D in ((2, 4), (0, 3), (1, 6)):
        vals = oracle.synth(dist, D, 20000, seed=3)
        ids = np.arange(20000, dtype=np.int64)
        a = oracle.query_bnl("angle", vals, ids, 8)
        for T in (1, 3, 8):
            b = oracle.query_bnl_mt("angle", vals, ids, 8, T)
            assert sorted(a[0].tolist()) == sorted(b[0].tolist())
            assert (a[2] == b[2]).all() and (a[3] == b[3]).all()


def test_grid_filter_oracle_is_exact_when_best_quadrant_nonempty(oracle):
    """The filter only removes tuples dominated by any all-better tuple."""
    for dist in (0, 1, 2):
        vals = oracle.synth(dist, 3, 5000, seed=9)
        ids = np.arange(5000, dtype=np.int64)
        if not (vals < 500).all(axis=1).any():
            continue
        a = oracle.query_bnl("grid", vals, ids, 8)[0]
        oracle.L.orc_set_grid_filter(1)
        try:
            b = oracle.query_bnl("grid", vals, ids, 8)[0]
        finally:
            oracle.L.orc_set_grid_filter(0)
        assert sorted(a.tolist()) == sorted(b.tolist())


# ---- chunked oracle (oracle/skyline_oracle_big.c): the checker of the full-size configs ----
@pytest.mark.parametrize("path", golden_streams(), ids=lambda p: os.path.basename(p)[7:-4])
def test_chunked_oracle_matches_golden(path, oracle):
    """SKY(U SKY(chunk)) per key and globally, over distinct vectors, equals the golden BNL
    results for every chunk size (including chunks smaller than a partition's share)."""
    g = load_golden(path)
    vals = g["values"]
    for algo in ("dim", "grid", "angle"):
        for P in (4, 16):
            for chunk in (97, 1000, 1 << 20):
                gi, keys, ls, sv, _ = oracle.query_sfs_chunked(algo, vals, P, chunk=chunk, threads=4)
                np.testing.assert_array_equal(gi, g[f"gsky_{algo}_{P}"])
                np.testing.assert_array_equal(ls, g[f"lsz_{algo}_{P}"])
                np.testing.assert_array_equal(sv, g[f"surv_{algo}_{P}"])


def test_chunked_oracle_edge_values(oracle):
    """Duplicates, -0.0 == +0.0, infinities, negatives, complete MR-Grid semantics: the
    chunked oracle equals the single-threaded SFS restatement and the BNL restatement."""
    rng = np.random.default_rng(12)
    vals = rng.integers(-5, 6, size=(20000, 4)).astype(np.float64)
    vals[rng.random(20000) < 0.1, 0] = -0.0
    vals[rng.random(20000) < 0.03, 1] = np.inf
    vals[rng.random(20000) < 0.03, 2] = -np.inf
    ids = np.arange(len(vals), dtype=np.int64)
    for algo in ("dim", "grid", "angle"):
        for sem in (0, 1):
            if sem and algo != "grid":
                continue
            exp, ekeys, els, esv = oracle.query_sfs(algo, vals, 8, sem=sem)
            for chunk in (333, 5000):
                gi, keys, ls, sv, _ = oracle.query_sfs_chunked(algo, vals, 8, sem=sem, chunk=chunk, threads=3)
                np.testing.assert_array_equal(gi, exp)
                np.testing.assert_array_equal(keys, ekeys)
                np.testing.assert_array_equal(ls, els)
                np.testing.assert_array_equal(sv, esv)
        bnl, _, bls, bsv = oracle.query_bnl(algo, vals, ids, 8)
        np.testing.assert_array_equal(np.sort(bnl), oracle.query_sfs_chunked(algo, vals, 8, chunk=777)[0])


def test_c_replay_formats_optimality_like_java():
    """tests/operator_replay.c formats optimality as String.format(Locale.US, "%.4f", x):
    HALF_UP on the shortest repr (not C's round-half-even on the binary value)."""
    import subprocess
    from skyline.operators import java_format_4f
    binp = os.path.join(os.path.dirname(GOLDEN), "..", "flink-skyline-qos_amd", "build", "operator_replay")
    if not os.path.exists(binp):
        pytest.skip("operator_replay not built")
    xs = [0.0, 1.0, 0.25, 1 / 3, 2 / 3, 0.00005, 0.00015, 0.12345, 0.99995, 0.999949999, 0.7379, 0.5415,
          0.000049999999, 1e-9, 0.0625 + 1e-12, 0.1 + 0.2]
    rng = np.random.default_rng(1)
    xs += [float(x) for x in rng.random(300)]
    xs += [k / 10000 + 0.00005 for k in range(0, 10000, 97)]
    out = subprocess.run([binp, "--fmt"] + [repr(x) for x in xs], capture_output=True, text=True, check=True)
    got = out.stdout.split()
    assert got == [java_format_4f(x) for x in xs]
