"""Shared fixtures.  The oracle (oracle/) is TEST INFRASTRUCTURE: it is only the
checker here, never the thing under test."""
import ctypes
import glob
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "flink-skyline-qos_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
if PKG not in sys.path:
    sys.path.insert(0, PKG)
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libskyline_hip.so)")


_ORACLE = None


def load_oracle():
    global _ORACLE
    if _ORACLE is None:
        so = os.path.join(REPO, "oracle", "_build", "liboracle.so")
        if not os.path.exists(so):
            subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
        L = ctypes.CDLL(so)
        dp = ctypes.c_void_p
        L.orc_fdlibm_atan2.restype = ctypes.c_double
        L.orc_fdlibm_atan2.argtypes = [ctypes.c_double, ctypes.c_double]
        L.orc_fdlibm_table.restype = ctypes.POINTER(ctypes.c_double)
        L.orc_fdlibm_table.argtypes = [ctypes.c_int]
        L.orc_dominates.argtypes = [dp, dp, ctypes.c_int]
        L.orc_keys.argtypes = [ctypes.c_int, dp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_double, dp]
        L.orc_query_bnl.restype = ctypes.c_int64
        L.orc_query_bnl.argtypes = [ctypes.c_int, dp, dp, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_double, ctypes.c_int, ctypes.c_int, dp, dp, ctypes.c_int64, dp, dp]
        L.orc_query_bnl_mt.restype = ctypes.c_int64
        L.orc_query_bnl_mt.argtypes = [ctypes.c_int, dp, dp, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_double, ctypes.c_int, ctypes.c_int, dp, dp, ctypes.c_int64, dp, dp]
        L.orc_query_sfs.restype = ctypes.c_int64
        L.orc_query_sfs.argtypes = [ctypes.c_int, dp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                    ctypes.c_int, dp, dp, dp, dp, dp]
        L.orc_query_sfs_chunked.restype = ctypes.c_int64
        L.orc_query_sfs_chunked.argtypes = [ctypes.c_int, dp, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_double, ctypes.c_int, ctypes.c_int64, ctypes.c_int, dp, dp, dp,
                                            dp, dp]
        L.orc_skyline_brute.argtypes = [dp, ctypes.c_int64, ctypes.c_int, dp]
        L.orc_synth.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                ctypes.c_int64, ctypes.c_int64, dp]
        L.orc_set_grid_filter.argtypes = [ctypes.c_int]
        L.orc_java_parse_double.restype = ctypes.c_int
        L.orc_java_parse_double.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double)]
        L.orc_parse_csv.restype = ctypes.c_int64
        L.orc_parse_csv.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_int, dp, dp, dp, ctypes.c_int64]
        _ORACLE = L
    return _ORACLE


def P(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class Oracle:
    """numpy-friendly wrapper over oracle/_build/liboracle.so."""
    ALGO = {"dim": 0, "grid": 1, "angle": 2, "mr-dim": 0, "mr-grid": 1, "mr-angle": 2}

    def __init__(self):
        self.L = load_oracle()

    def keys(self, algo, vals, P_, domain=1000.0):
        v = np.ascontiguousarray(vals, np.float64)
        out = np.zeros(len(v), np.int32)
        self.L.orc_keys(self.ALGO[algo], P(v), len(v), v.shape[1], P_, domain, P(out))
        return out

    def query_bnl(self, algo, vals, ids, P_, domain=1000.0, sem=0, buffer_size=5000):
        v = np.ascontiguousarray(vals, np.float64)
        ids = np.ascontiguousarray(ids, np.int64)
        n, D = v.shape
        K = P_ if not (self.ALGO[algo] == 1 and sem == 1) else max(P_, 1 << D)
        oi = np.zeros(max(n, 1), np.int64)
        oo = np.zeros(max(n, 1), np.int32)
        ls = np.zeros(K, np.int64)
        sv = np.zeros(K, np.int64)
        g = self.L.orc_query_bnl(self.ALGO[algo], P(v), P(ids), n, D, P_, domain, buffer_size, sem, P(oi), P(oo),
                                 n, P(ls), P(sv))
        assert g >= 0
        return oi[:g], oo[:g], ls, sv

    def query_bnl_mt(self, algo, vals, ids, P_, threads, domain=1000.0, buffer_size=5000):
        v = np.ascontiguousarray(vals, np.float64)
        ids = np.ascontiguousarray(ids, np.int64)
        n, D = v.shape
        oi = np.zeros(max(n, 1), np.int64)
        oo = np.zeros(max(n, 1), np.int32)
        ls = np.zeros(P_, np.int64)
        sv = np.zeros(P_, np.int64)
        g = self.L.orc_query_bnl_mt(self.ALGO[algo], P(v), P(ids), n, D, P_, domain, buffer_size, threads, P(oi),
                                    P(oo), n, P(ls), P(sv))
        assert g >= 0
        return oi[:g], oo[:g], ls, sv

    def query_sfs(self, algo, vals, P_, domain=1000.0, sem=0):
        v = np.ascontiguousarray(vals, np.float64)
        n, D = v.shape
        K = P_ if not (self.ALGO[algo] == 1 and sem == 1) else max(P_, 1 << D)
        keys = np.zeros(max(n, 1), np.int32)
        inl = np.zeros(max(n, 1), np.uint8)
        ing = np.zeros(max(n, 1), np.uint8)
        ls = np.zeros(K, np.int64)
        sv = np.zeros(K, np.int64)
        g = self.L.orc_query_sfs(self.ALGO[algo], P(v), n, D, P_, domain, sem, P(keys), P(inl), P(ing), P(ls), P(sv))
        assert g >= 0
        return np.nonzero(ing[:n])[0], keys[:n], ls, sv

    def query_sfs_chunked(self, algo, vals, P_, domain=1000.0, sem=0, chunk=1 << 20, threads=None):
        """orc_query_sfs_chunked (oracle/skyline_oracle_big.c): the same outputs as query_sfs, computed
        as SKY(U SKY(chunk)) per key then globally, over distinct vectors, on `threads` threads.
        Returns (global ids = row indices, keys, |L_k|, survivors_k, in_local flags)."""
        v = np.ascontiguousarray(vals, np.float64)
        n, D = v.shape
        K = P_ if not (self.ALGO[algo] == 1 and sem == 1) else max(P_, 1 << D)
        if threads is None:
            threads = max(1, min(16, len(os.sched_getaffinity(0))))
        keys = np.zeros(max(n, 1), np.int32)
        inl = np.zeros(max(n, 1), np.uint8)
        ing = np.zeros(max(n, 1), np.uint8)
        ls = np.zeros(K, np.int64)
        sv = np.zeros(K, np.int64)
        g = self.L.orc_query_sfs_chunked(self.ALGO[algo], P(v), n, D, P_, domain, sem, int(chunk), int(threads),
                                         P(keys), P(inl), P(ing), P(ls), P(sv))
        assert g >= 0
        return np.nonzero(ing[:n])[0], keys[:n], ls, sv, inl[:n]

    def java_parse_double(self, s):
        """Double.parseDouble restatement: float, or None for a NumberFormatException."""
        b = s.encode() if isinstance(s, str) else bytes(s)
        buf = ctypes.create_string_buffer(b, len(b))
        out = ctypes.c_double(0)
        ok = self.L.orc_java_parse_double(buf, ctypes.cast(ctypes.addressof(buf) + len(b), ctypes.c_char_p),
                                          ctypes.byref(out))
        return out.value if ok else None

    def parse_csv(self, text, D):
        """-> (status u8[records], ids i64[records], values f64[records, D]); rows valid where status == 0."""
        b = bytes(text)
        cap = len(b) // 2 + 2
        st = np.zeros(cap, np.uint8)
        ids = np.zeros(cap, np.int64)
        vals = np.zeros((cap, D), np.float64)
        n = self.L.orc_parse_csv(b, len(b), D, P(ids), P(vals), P(st), cap)
        return st[:n], ids[:n], vals[:n]

    def brute(self, vals):
        v = np.ascontiguousarray(vals, np.float64)
        out = np.zeros(max(len(v), 1), np.uint8)
        self.L.orc_skyline_brute(P(v), len(v), v.shape[1], P(out))
        return np.nonzero(out[:len(v)])[0]

    def synth(self, dist, D, n, seed=1234, id0=0, dmin=0, dmax=1000):
        out = np.zeros((n, D), np.float64)
        self.L.orc_synth(dist, D, dmin, dmax, seed, id0, n, P(out))
        return out


@pytest.fixture(scope="session")
def oracle():
    return Oracle()


def golden_streams():
    return sorted(glob.glob(os.path.join(GOLDEN, "stream_*.npz")))


def load_golden(path):
    z = np.load(path)   # allow_pickle stays False
    d = {k: z[k] for k in z.files}
    d["values"] = d["values"].astype(np.float64)
    return d


@pytest.fixture(scope="session")
def gpu_engine_factory():
    """Builds SkylineEngine objects; skips cleanly when no GPU is visible (CPU runs)."""
    import skyline
    from skyline._abi import SkylineError

    def make(dims, P_, algo="mr-angle", domain=1000.0, semantics="reference"):
        try:
            return skyline.SkylineEngine(dims, P_, algo, domain, 0, semantics)
        except SkylineError as e:
            if e.code == -6:
                pytest.fail("no HIP device visible for a gpu-marked test: " + str(e))
            raise
    return make


def dist_emulate(engs, d_ids, d_vals, cap=4096, steps=1, max_attempts=8):
    """W ranks of the multi-GPU step emulated on one GPU: one engine (context) per rank, the
    all-gather = concatenation of the ranks' device blocks, the all-reduce = a device sum
    (the collectives RCCL performs between processes).  Returns, per step, the per-rank
    (ids, origins) and the job-wide (|L_k|, survivors_k), plus per-step per-rank host
    synchronisations and the attempts each step took."""
    import torch
    from skyline import _abi
    from skyline.dist import block_words, stats_words
    W = len(engs)
    D, K = engs[0].dims, engs[0].K
    dev = d_vals[0].device
    outs = []
    for _ in range(steps):
        h0 = [e.host_syncs() for e in engs]
        oi = [torch.empty(max(v.shape[0], 1), dtype=torch.int64, device=dev) for v in d_vals]
        oo = [torch.empty(max(v.shape[0], 1), dtype=torch.int32, device=dev) for v in d_vals]
        export, attempts = True, 0
        while True:
            attempts += 1
            assert attempts <= max_attempts
            send = [torch.empty(block_words(cap, D), dtype=torch.int64, device=dev) for _ in range(W)]
            for r, e in enumerate(engs):
                if export:
                    e.dist_export_dev(d_ids[r], d_vals[r], send[r], cap)
                else:
                    e.dist_reblock_dev(send[r], cap)
            recv = torch.cat(send)
            stats = [torch.empty(stats_words(K), dtype=torch.int64, device=dev) for _ in range(W)]
            for r, e in enumerate(engs):
                e.dist_merge_dev(recv, W, r, cap, oi[r], oo[r], d_vals[r].shape[0], stats[r])
            tot = torch.stack(stats).sum(0)
            res = [e.dist_finish(tot, d_vals[r].shape[0]) for r, e in enumerate(engs)]
            rcs = {x[0] for x in res}
            assert len(rcs) == 1, f"ranks disagree: {res}"
            rc = rcs.pop()
            if rc == _abi.SKY_OK:
                break
            if rc == _abi.SKY_E_RETRY:
                export = True
            else:
                need = {x[2] for x in res}
                assert len(need) == 1
                cap = need.pop() + 64
                export = False
        got = [(oi[r][:res[r][1]].cpu().numpy(), oo[r][:res[r][1]].cpu().numpy()) for r in range(W)]
        ls, sv = engs[0].stats()
        for e in engs[1:]:
            l2, s2 = e.stats()
            np.testing.assert_array_equal(l2, ls)
            np.testing.assert_array_equal(s2, sv)
        outs.append({"ids": np.concatenate([g[0] for g in got]), "org": np.concatenate([g[1] for g in got]),
                     "ls": ls, "sv": sv, "syncs": [e.host_syncs() - h for e, h in zip(engs, h0)],
                     "attempts": attempts, "cap": cap})
    return outs
