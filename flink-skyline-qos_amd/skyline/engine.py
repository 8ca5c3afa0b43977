"""Python handle over one sky_ctx (one MI355X).

Host-buffer methods take numpy arrays; `*_dev` methods take torch CUDA tensors
(HBM-resident) and pass their data pointers through the C ABI.
"""
import ctypes

import numpy as np

from . import _abi
from ._abi import check, lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def _tptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class _Ordered:
    """Brackets a *_dev call: the library's stream first waits for the caller's current
    torch stream (which produced the inputs), and the torch stream then waits for the
    library (which wrote the outputs).  GPU-side events only.  An engine bound to a torch
    stream (SkylineEngine.use_torch_stream) runs ON that stream: no events, no stream lookup."""

    def __init__(self, h, device, bound=None):
        self.h = h
        self.s = None
        if bound is not None:
            return
        t = _abi.torch
        if t is not None and t.cuda.is_available():
            self.s = ctypes.c_void_p(t.cuda.current_stream(device).cuda_stream)

    def __enter__(self):
        if self.s is not None:
            check(lib().sky_ctx_wait_stream(self.h, self.s))
        return self

    def __exit__(self, *exc):
        if self.s is not None and exc[0] is None:
            check(lib().sky_ctx_signal_stream(self.h, self.s))
        return False


class SkylineEngine:
    """One context = one device, D dims, P partitions, one partitioner.

    Mirrors the job-level knobs of FlinkSkyline.main (FlinkSkyline.java:66-76):
    algo (--algo), domain (--domain), dims (--dims), num_partitions = 2 x parallelism.
    """

    def __init__(self, dims, num_partitions, algo="mr-angle", domain=1000.0, device=0,
                 semantics="reference", grid_filter=False):
        if isinstance(algo, str):
            algo = _abi.ALGOS.get(algo.lower(), _abi.ALGO_ANGLE)  # reference default branch (:129-133)
        self.dims = int(dims)
        self.P = int(num_partitions)
        self.algo = int(algo)
        self.domain = float(domain)
        self.device = int(device)
        h = ctypes.c_void_p()
        dev = (ctypes.c_int32 * 1)(device)
        check(lib().sky_ctx_create(dev, 1, self.dims, self.P, self.algo, self.domain, ctypes.byref(h)))
        self.h = h
        if semantics != "reference":
            check(lib().sky_ctx_set_semantics(self.h, _abi.SEM_COMPLETE))
        if grid_filter:   # GridDominanceFilter (FlinkSkyline.java:716-733)
            check(lib().sky_ctx_set_grid_filter(self.h, 1))
        self._bound = None               # use_torch_stream: the torch stream the library runs on
        self.last_dist_stats = None      # set by skyline.dist.distributed_query
        self.K = self.P if not (self.algo == _abi.ALGO_GRID and semantics == "complete") else max(self.P, 1 << self.dims)

    def warmup(self):
        """sky_ctx_warmup: first launches and allocations of every pipeline branch, once."""
        check(lib().sky_ctx_warmup(self.h))

    def close(self):
        if self.h:
            lib().sky_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- partitioners ----------------------------------------------------------
    def partition_keys(self, values):
        v = np.ascontiguousarray(values, dtype=np.float64).reshape(-1, self.dims)
        out = np.empty(len(v), np.int32)
        check(lib().sky_partition_keys(self.h, _ptr(v), len(v), _ptr(out)))
        return out

    def partition_keys_dev(self, d_values, d_keys_out):
        n = d_values.numel() // self.dims
        with _Ordered(self.h, self.device, self._bound):
            check(lib().sky_partition_keys_dev(self.h, _tptr(d_values), n, _tptr(d_keys_out)))

    # ---- fused query ---------------------------------------------------------------
    def query(self, values, ids=None):
        """Global skyline of the whole stream (trigger after the last tuple).
        Returns (ids, origin) in stream order."""
        v = np.ascontiguousarray(values, dtype=np.float64).reshape(-1, self.dims)
        n = len(v)
        idv = None if ids is None else np.ascontiguousarray(ids, dtype=np.int64)
        cnt = ctypes.c_int64(0)
        out_ids = np.empty(max(n, 1), np.int64)
        out_org = np.empty(max(n, 1), np.int32)
        check(lib().sky_query(self.h, _ptr(idv), _ptr(v), n, _ptr(out_ids), _ptr(out_org), n, ctypes.byref(cnt)))
        g = cnt.value
        return out_ids[:g].copy(), out_org[:g].copy()

    def query_dev(self, d_ids, d_values, d_ids_out, d_origin_out, cap):
        n = d_values.numel() // self.dims
        cnt = ctypes.c_int64(0)
        with _Ordered(self.h, self.device, self._bound):
            check(lib().sky_query_dev(self.h, _tptr(d_ids), _tptr(d_values), n, _tptr(d_ids_out),
                                      _tptr(d_origin_out), cap, ctypes.byref(cnt)))
        return cnt.value

    def stats(self):
        """(local_sizes[K], survivors[K]) of the last query/merge (FlinkSkyline.java:593-608)."""
        k = ctypes.c_int32(0)
        check(lib().sky_global_stats(self.h, None, None, ctypes.byref(k)))
        ls = np.zeros(max(k.value, 1), np.int64)
        sv = np.zeros(max(k.value, 1), np.int64)
        check(lib().sky_global_stats(self.h, _ptr(ls), _ptr(sv), ctypes.byref(k)))
        return ls[:k.value], sv[:k.value]

    def set_stats(self, local_sizes, survivors):
        """Record job-wide |L_k| / survivors_k (the all-reduced per-rank shares of a
        multi-GPU query) so that stats() returns them."""
        ls = np.ascontiguousarray(local_sizes, np.int64)
        sv = np.ascontiguousarray(survivors, np.int64)
        check(lib().sky_global_stats_set(self.h, len(ls), _ptr(ls), _ptr(sv)))

    # ---- global merge of local lists ------------------------------------------------
    def global_merge(self, part_ids, ids_lists, values_lists):
        n = len(part_ids)
        vals = [np.ascontiguousarray(v, dtype=np.float64).reshape(-1, self.dims) for v in values_lists]
        idl = [np.ascontiguousarray(i, dtype=np.int64) for i in ids_lists]
        counts = np.array([len(v) for v in vals], np.int64)
        pids = np.ascontiguousarray(part_ids, dtype=np.int32)
        vp = (ctypes.c_void_p * max(n, 1))(*[v.ctypes.data for v in vals])
        ip = (ctypes.c_void_p * max(n, 1))(*[i.ctypes.data for i in idl])
        tot = int(counts.sum())
        out_ids = np.empty(max(tot, 1), np.int64)
        out_org = np.empty(max(tot, 1), np.int32)
        cnt = ctypes.c_int64(0)
        check(lib().sky_global_merge(self.h, n, _ptr(pids), ip, vp, _ptr(counts), _ptr(out_ids), _ptr(out_org),
                                     tot, ctypes.byref(cnt)))
        g = cnt.value
        return out_ids[:g].copy(), out_org[:g].copy()

    def global_merge_reps(self, part_ids, lists):
        """sky_global_merge_reps: the merge over local skylines shipped as distinct vectors;
        lists[g] = (ids int64 [T], rep_idx int32 [T], reps f64 [R, dims], rep_counts int32 [R]).
        Same (ids, origins) and stats as global_merge over the expanded lists."""
        n = len(part_ids)
        idl = [np.ascontiguousarray(l[0], np.int64) for l in lists]
        rpi = [np.ascontiguousarray(l[1], np.int32) for l in lists]
        rps = [np.ascontiguousarray(l[2], np.float64).reshape(-1, self.dims) for l in lists]
        rpc = [np.ascontiguousarray(l[3], np.int32) for l in lists]
        counts = np.array([len(a) for a in idl], np.int64)
        nreps = np.array([len(a) for a in rps], np.int64)
        pids = np.ascontiguousarray(part_ids, dtype=np.int32)

        def arr(xs):
            return (ctypes.c_void_p * max(n, 1))(*[a.ctypes.data for a in xs])
        tot = int(counts.sum())
        out_ids = np.empty(max(tot, 1), np.int64)
        out_org = np.empty(max(tot, 1), np.int32)
        cnt = ctypes.c_int64(0)
        check(lib().sky_global_merge_reps(self.h, n, _ptr(pids), arr(idl), arr(rpi), _ptr(counts), arr(rps), arr(rpc),
                                          _ptr(nreps), _ptr(out_ids), _ptr(out_org), tot, ctypes.byref(cnt)))
        g = cnt.value
        return out_ids[:g].copy(), out_org[:g].copy()

    # ---- multi-GPU step with one host read (sky_dist_*) ------------------------------------
    def dist_export_dev(self, d_ids, d_values, d_block, cap):
        """Local skylines of this rank's shard -> its fixed-size exchange block (no host read)."""
        n = d_values.numel() // self.dims
        with _Ordered(self.h, self.device, self._bound):
            check(lib().sky_dist_export_dev(self.h, _tptr(d_ids), _tptr(d_values), n, _tptr(d_block), cap))

    def dist_reblock_dev(self, d_block, cap):
        """Rewrite this rank's block with a larger capacity (after SKY_E_CAPACITY with need_cap)."""
        with _Ordered(self.h, self.device, self._bound):
            check(lib().sky_dist_reblock_dev(self.h, _tptr(d_block), cap))

    def dist_merge_dev(self, d_blocks, world, rank, cap, d_ids_out, d_origin_out, out_cap, d_stats):
        """Own vectors vs the gathered union; output ids and this rank's stat shares (no host read)."""
        with _Ordered(self.h, self.device, self._bound):
            check(lib().sky_dist_merge_dev(self.h, _tptr(d_blocks), world, rank, cap, _tptr(d_ids_out),
                                           _tptr(d_origin_out), out_cap, _tptr(d_stats)))

    def dist_finish(self, d_stats_sum, out_cap):
        """The step's one host read -> (status, this rank's output count, needed exchange capacity);
        status is SKY_OK or SKY_E_RETRY / SKY_E_CAPACITY (the caller re-runs), other codes raise."""
        n = ctypes.c_int64(0)
        need = ctypes.c_int64(0)
        with _Ordered(self.h, self.device, self._bound):
            rc = lib().sky_dist_finish(self.h, _tptr(d_stats_sum), out_cap, ctypes.byref(n), ctypes.byref(need))
        if rc not in (_abi.SKY_OK, _abi.SKY_E_RETRY, _abi.SKY_E_CAPACITY) or \
                (rc == _abi.SKY_E_CAPACITY and need.value == 0):
            check(rc)
        return rc, n.value, need.value

    def host_syncs(self):
        """Host synchronisations (device read-backs) this context has made."""
        n = ctypes.c_int64(0)
        check(lib().sky_profile_host_syncs(self.h, ctypes.byref(n)))
        return n.value

    # ---- utilities -----------------------------------------------------------------------
    def synth_dev(self, dist, n, d_values, d_ids=None, seed=1234, id0=0, dmin=0, dmax=1000):
        if isinstance(dist, str):
            dist = _abi.DISTS[dist]
        with _Ordered(self.h, self.device, self._bound):
            check(lib().sky_synth_dev(self.h, dist, dmin, dmax, seed, id0, n, _tptr(d_values), _tptr(d_ids)))

    # ---- bulk CSV ingest (ServiceTuple.fromString over raw records, ServiceTuple.java:89-104)
    def parse_csv(self, text):
        """Host bytes -> (ids int64[n], values f64[n, D], counts int64[4]); counts =
        [records, malformed, bad id, wrong arity].  Decoded on the device."""
        b = bytes(text)
        rmax = len(b) // 2 + 1
        ids = np.empty(rmax, np.int64)
        vals = np.empty((rmax, self.dims), np.float64)
        n = ctypes.c_int64(0)
        cnt = np.zeros(4, np.int64)
        check(lib().sky_parse_csv(self.h, b, len(b), _ptr(ids), _ptr(vals), rmax, ctypes.byref(n),
                                  cnt.ctypes.data_as(_abi.P_i64)))
        return ids[:n.value].copy(), vals[:n.value].copy(), cnt

    def parse_csv_dev(self, d_text, nbytes, d_ids_out, d_values_out, cap, d_status_out=None):
        """Device bytes -> device rows; returns (accepted, counts int64[4])."""
        n = ctypes.c_int64(0)
        cnt = np.zeros(4, np.int64)
        with _Ordered(self.h, self.device, self._bound):
            check(lib().sky_parse_csv_dev(self.h, _tptr(d_text), nbytes, _tptr(d_ids_out), _tptr(d_values_out), cap,
                                          ctypes.byref(n), cnt.ctypes.data_as(_abi.P_i64), _tptr(d_status_out)))
        return n.value, cnt

    def format_csv_dev(self, d_ids, d_values, n, d_text=None, cap=0):
        """The producers' "id,v1,...,vD\n" payload of a device stream; returns its byte count
        (call with d_text=None first to size the buffer)."""
        nb = ctypes.c_int64(0)
        with _Ordered(self.h, self.device, self._bound):
            check(lib().sky_format_csv_dev(self.h, _tptr(d_ids), _tptr(d_values), n, _tptr(d_text), cap,
                                           ctypes.byref(nb)))
        return nb.value

    def profile_sort_dev(self, d_keys, d_vals):
        """Runs the pipeline's radix sort alone on (int64 keys as u64, int32 values as u32),
        in place; returns (passes, ms)."""
        p = ctypes.c_int32(0)
        ms = ctypes.c_double(0)
        with _Ordered(self.h, self.device, self._bound):
            check(lib().sky_profile_sort_dev(self.h, _tptr(d_keys), _tptr(d_vals), d_keys.numel(), ctypes.byref(p),
                                             ctypes.byref(ms)))
        return p.value, ms.value

    def profile_pairs_dev(self, d_values, d_keys, d_fates_out):
        """The small-set route's dense all-pairs kernel alone on device rows with given
        partition keys (int32): fates (bit0 dominated within its partition, bit1 by any row)
        into d_fates_out (int32 view of u32); returns (kind 0 u16 / 1 f32 / 2 f64, kernel ms)."""
        n = d_values.numel() // self.dims
        kind = ctypes.c_int32(0)
        ms = ctypes.c_double(0)
        with _Ordered(self.h, self.device, self._bound):
            check(lib().sky_profile_pairs_dev(self.h, _tptr(d_values), _tptr(d_keys), n, _tptr(d_fates_out),
                                              ctypes.byref(kind), ctypes.byref(ms)))
        return kind.value, ms.value

    def set_stream(self, stream_ptr):
        check(lib().sky_ctx_set_stream(self.h, ctypes.c_void_p(stream_ptr) if stream_ptr else None))
        self._bound = None

    def use_torch_stream(self, stream=None):
        """Run the library on a torch stream (default: the current one) instead of its own:
        the *_dev calls then need no cross-stream events (two HIP event operations and a
        stream lookup per call).  The caller keeps issuing the tensors it passes on that
        stream (or calls use_torch_stream again / set_stream(None) to go back)."""
        t = _abi.torch
        st = stream if stream is not None else t.cuda.current_stream(self.device)
        check(lib().sky_ctx_set_stream(self.h, ctypes.c_void_p(st.cuda_stream)))
        self._bound = st

    def sync(self):
        check(lib().sky_ctx_sync(self.h))

    def profile(self, on=True):
        """on: False/0 off, 1 kernel timers only, True/2 kernel timers + phase events."""
        level = 2 if on is True else int(on)
        check(lib().sky_profile_enable(self.h, level))

    def profile_reset(self):
        check(lib().sky_profile_reset(self.h))

    def phases(self):
        ms = np.zeros(8, np.float64)
        cnt = np.zeros(8, np.int64)
        check(lib().sky_profile_phases(self.h, _ptr(ms), _ptr(cnt)))
        return dict(zip(_abi.PHASES, ms.tolist())), cnt

    def dominance_work(self):
        """Algorithmic pair tests (distinct vectors) of the last query."""
        w = ctypes.c_int64(0)
        check(lib().sky_profile_dominance(self.h, ctypes.byref(w)))
        return w.value

    def kernel_time(self, name):
        ms = ctypes.c_double(0)
        la = ctypes.c_int64(0)
        un = ctypes.c_int64(0)
        check(lib().sky_profile_kernel(self.h, name.encode(), ctypes.byref(ms), ctypes.byref(la), ctypes.byref(un)))
        return ms.value, la.value, un.value


def synth_host(dist, dims, n, seed=1234, id0=0, dmin=0, dmax=1000):
    """Host copy of the device generator (same values bit for bit)."""
    if isinstance(dist, str):
        dist = _abi.DISTS[dist]
    v = np.empty((n, dims), np.float64)
    ids = np.empty(n, np.int64)
    check(lib().sky_synth(dist, dims, dmin, dmax, seed, id0, n, _ptr(v), _ptr(ids)))
    return v, ids


class SkylineStream:
    """Continuous queries over an append-only stream on one engine (sky_stream_*).

    window=0: the reference's landmark window (FlinkSkyline.java:265-316 + :417-444): a
    query covers every tuple appended so far; between queries only the local-skyline
    tuples stay resident.  window=W > 0: count-based sliding window over the last W
    appended tuples (an extension; the reference has no window)."""

    def __init__(self, engine, window=0):
        self.engine = engine
        self.window = int(window)
        h = ctypes.c_void_p()
        check(lib().sky_stream_create(engine.h, self.window, ctypes.byref(h)))
        self.h = h

    def close(self):
        if self.h:
            lib().sky_stream_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def append(self, ids, values):
        """Host arrays (numpy): ids int64[n], values f64[n, D]."""
        ids = np.ascontiguousarray(ids, np.int64)
        v = np.ascontiguousarray(values, np.float64)
        check(lib().sky_stream_append(self.h, _ptr(ids), _ptr(v), len(ids)))

    def append_dev(self, d_ids, d_values, n=None):
        n = d_values.shape[0] if n is None else n
        with _Ordered(self.engine.h, self.engine.device, self.engine._bound):
            check(lib().sky_stream_append_dev(self.h, _tptr(d_ids), _tptr(d_values), n))

    def size(self):
        r, a = ctypes.c_int64(0), ctypes.c_int64(0)
        check(lib().sky_stream_size(self.h, ctypes.byref(r), ctypes.byref(a)))
        return r.value, a.value

    def vectors(self):
        """Rows the next query runs over (sky_stream_vectors): a landmark stream's distinct
        local-skyline vectors + the tuples appended since its last query."""
        v = ctypes.c_int64(0)
        check(lib().sky_stream_vectors(self.h, ctypes.byref(v)))
        return v.value

    def _out(self, cap):
        """Reusable page-locked result buffers (D2H at full PCIe rate), numpy views."""
        if getattr(self, "_cap", 0) < cap:
            cap = max(cap, 2 * getattr(self, "_cap", 0))
            if _abi.torch is not None and _abi.torch.cuda.is_available():
                t = _abi.torch
                self._ids = t.empty(cap, dtype=t.int64, pin_memory=True).numpy()
                self._org = t.empty(cap, dtype=t.int32, pin_memory=True).numpy()
            else:
                self._ids = np.empty(cap, np.int64)
                self._org = np.empty(cap, np.int32)
            self._cap = cap
        return self._ids, self._org

    def query(self):
        """-> (ids int64[g], origin int32[g]) of the global skyline, arrival order (copies)."""
        r, _ = self.size()
        cap = max(r, 1)
        ids, org = self._out(cap)
        g = ctypes.c_int64(0)
        check(lib().sky_stream_query(self.h, _ptr(ids), _ptr(org), cap, ctypes.byref(g)))
        return ids[:g.value].copy(), org[:g.value].copy()

    def reserve(self, cap):
        """Size the page-locked result buffers and the device state once, for up to `cap`
        resident tuples (pinning hundreds of MB takes tens of ms, and every device regrowth
        synchronises the GPU: not something a trigger should pay)."""
        self._out(max(int(cap), 1))
        check(lib().sky_stream_reserve(self.h, max(int(cap), 1)))

    def query_host_view(self):
        """Query into the reusable page-locked buffers; returns g (results in view()[:g])."""
        r, _ = self.size()
        cap = max(r, 1)
        ids, org = self._out(cap)
        g = ctypes.c_int64(0)
        check(lib().sky_stream_query(self.h, _ptr(ids), _ptr(org), cap, ctypes.byref(g)))
        return g.value

    def query_async_host_view(self):
        """sky_stream_query_async into the reusable page-locked buffers: returns g as soon as the
        integers are known (skyline size, engine.stats()); the ids / origins land in view()[:g]
        while the caller goes on appending -- valid after wait()."""
        r, _ = self.size()
        cap = max(r, 1)
        ids, org = self._out(cap)
        g = ctypes.c_int64(0)
        check(lib().sky_stream_query_async(self.h, _ptr(ids), _ptr(org), cap, ctypes.byref(g)))
        return g.value

    def wait(self):
        """Waits for the result copy of the last query_async_host_view; returns its device time
        (ms, from the end of the query's kernels to the last byte in host memory), 0 if none."""
        ms = ctypes.c_double(0)
        check(lib().sky_stream_wait(self.h, ctypes.byref(ms)))
        return ms.value

    def view(self):
        return self._ids, self._org

    def query_dev(self, d_ids_out, d_origin_out, cap):
        g = ctypes.c_int64(0)
        with _Ordered(self.engine.h, self.engine.device, self.engine._bound):
            check(lib().sky_stream_query_dev(self.h, _tptr(d_ids_out), _tptr(d_origin_out), cap, ctypes.byref(g)))
        return g.value
