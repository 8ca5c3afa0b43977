"""Host-side mirror of the reference's operator surface, running on libskyline_hip.

Same class and method names, argument meaning and error behaviour as
/root/reference/java/org.main/FlinkSkyline.java and ServiceTuple.java, so that a
caller of the Java operators finds the same API.  The dominance work (BNL in the
reference) always runs in the library on the GPU; this module only keeps the
operator protocol: buffering, the id barrier, the trigger fan-out, the arrival
count and the JSON payload.

Deliberate, documented differences:
  * the input buffer is per key (the reference's is shared by every key of a
    subtask, FlinkSkyline.java:223,244 — it moves tuples between keys);
  * the JSON carries "query_latency_ms" (computed but never emitted by the
    reference, :588 vs :632-641);
  * NaN values raise (the reference's BNL result is order-dependent for NaN).
"""
import ctypes
import decimal
import time

import numpy as np

from . import _abi
from ._abi import check, lib
from .engine import SkylineEngine


def now_ms():
    return int(time.time() * 1000)


_JAVA_LONG_MAX = (1 << 63) - 1


def java_parse_long(s):
    """Long.parseLong(s): an optional sign and ASCII digits only -- no whitespace, no '_', no
    other digit scripts (Python's int() accepts all three) -- within the long range; anything
    else is a NumberFormatException (raised here as ValueError)."""
    t = s[1:] if s[:1] in ("+", "-") else s
    if not t or any(c not in "0123456789" for c in t):
        raise ValueError('NumberFormatException: For input string: "%s"' % s)
    v = int(s)
    if v > _JAVA_LONG_MAX or v < -_JAVA_LONG_MAX - 1:
        raise ValueError('NumberFormatException: For input string: "%s"' % s)
    return v


def java_format_4f(x):
    """String.format(Locale.US, "%.4f", x): Java rounds HALF_UP on the shortest
    decimal representation of the double (FormattedFloatingDecimal)."""
    if x != x:
        return "NaN"
    if x in (float("inf"), float("-inf")):
        return "Infinity" if x > 0 else "-Infinity"
    d = decimal.Decimal(repr(float(x)))
    return str(d.quantize(decimal.Decimal("0.0001"), rounding=decimal.ROUND_HALF_UP))


def java_split(s, sep=","):
    """String.split(sep) for a one-character separator: trailing empty strings removed."""
    parts = s.split(sep)
    while len(parts) > 1 and parts[-1] == "":
        parts.pop()
    if parts == [""] and s != "":
        return []
    return parts


class ServiceTuple:
    """ServiceTuple.java:15-115 (data model; dominance is evaluated on the device)."""

    __slots__ = ("id", "values", "originPartition", "bad_id")

    def __init__(self, id=None, values=None):
        self.id = id
        self.values = values
        self.originPartition = -1
        self.bad_id = False

    @staticmethod
    def fromStrings(lines, engine):
        """ServiceTuple.fromString (:89-104) over a batch of raw values, decoded on the device
        (sky_parse_csv, k_csv.hip): one entry per line, None where fromString returns null.
        A record whose id is not a Java long yields a tuple flagged `bad_id`; the reference
        only fails on it later, at Long.parseLong (FlinkSkyline.java:276)."""
        lines = list(lines)
        if not lines:
            return []
        text = ("\n".join(lines) + "\n").encode("utf-8", "surrogateescape")
        if any("\n" in x for x in lines):
            raise ValueError("a raw record contains a newline")
        import torch
        dev = torch.device("cuda", engine.device)
        d_text = torch.frombuffer(bytearray(text), dtype=torch.uint8).to(dev)
        R = len(lines)
        ids = torch.empty(R, dtype=torch.int64, device=dev)
        vals = torch.empty((R, engine.dims), dtype=torch.float64, device=dev)
        stat = torch.empty(R, dtype=torch.uint8, device=dev)
        n, _ = engine.parse_csv_dev(d_text, len(text), ids, vals, R, stat)
        st = stat.cpu().numpy()
        ids = ids[:n].cpu().numpy()
        vals = vals[:n].cpu().numpy()
        out, k = [], 0
        for i, c in enumerate(st):
            if c == _abi.CSV_OK:
                out.append(ServiceTuple(str(int(ids[k])), vals[k].tolist()))
                k += 1
            elif c == _abi.CSV_BAD_ID:
                t = ServiceTuple(lines[i].split(",", 1)[0], None)
                t.bad_id = True
                out.append(t)
            else:   # malformed (null) or a value count other than the job's dims
                out.append(None)
        return out

    _engines = {}

    @staticmethod
    def fromString(s):
        """ServiceTuple.fromString (:89-104) for one raw value, decoded on the device."""
        D = len(s.rstrip(",").split(",")) - 1
        if D < 1:
            return None
        if D > _abi.SKY_MAX_DIMS:
            raise ValueError("more than %d values per tuple" % _abi.SKY_MAX_DIMS)
        eng = ServiceTuple._engines.get(D)
        if eng is None:
            eng = ServiceTuple._engines[D] = SkylineEngine(D, 1, "mr-dim", 1000.0, 0)
        return ServiceTuple.fromStrings([s], eng)[0]

    def __repr__(self):
        return "ID:" + str(self.id) + " " + str(self.values)


class PartitioningLogic:
    """FlinkSkyline.PartitioningLogic (:669-877).  getKey runs the bit-exact device
    key function; getKeys batches a whole array (the form the operators use)."""

    class SkylinePartitioner:
        algo = _abi.ALGO_ANGLE

        def __init__(self, partitions, dims, maxVal=1000.0, device=0):
            self.partitions = int(partitions)
            self.dims = int(dims)
            self.engine = SkylineEngine(dims, partitions, self.algo, maxVal, device)

        def getKey(self, t):
            if len(t.values) != self.dims:
                raise IndexError("tuple has %d values, partitioner expects %d" % (len(t.values), self.dims))
            return int(self.engine.partition_keys(np.asarray(t.values, np.float64))[0])

        def getKeys(self, values):
            return self.engine.partition_keys(values)

    class DimPartitioner(SkylinePartitioner):
        algo = _abi.ALGO_DIM

        def __init__(self, partitions, maxVal, dims=1, device=0):
            super().__init__(partitions, dims, maxVal, device)

    class GridPartitioner(SkylinePartitioner):
        algo = _abi.ALGO_GRID

        def __init__(self, partitions, maxVal, dims, device=0):
            super().__init__(partitions, dims, maxVal, device)

    class AnglePartitioner(SkylinePartitioner):
        algo = _abi.ALGO_ANGLE

        def __init__(self, partitions, dims, device=0):
            super().__init__(partitions, dims, 1000.0, device)


def make_partitioner(algo, num_partitions, domain, dims, device=0):
    """The --algo switch of FlinkSkyline.main (:112-134); unknown names fall back to MR-Angle."""
    a = algo.lower()
    if a == "mr-dim":
        return PartitioningLogic.DimPartitioner(num_partitions, domain, dims, device)
    if a == "mr-grid":
        return PartitioningLogic.GridPartitioner(num_partitions, domain, dims, device)
    return PartitioningLogic.AnglePartitioner(num_partitions, dims, device)


def device_count():
    """HIP devices this process sees (sky_device_count; 0 without a GPU)."""
    n = ctypes.c_int32(0)
    check(lib().sky_device_count(ctypes.byref(n)))
    return n.value


def device_for_subtask(subtask, ndev=None):
    """The device of a Flink subtask's context (sky_device_for_subtask): subtask % ndev, as
    HipSkylineOperators.open() maps getIndexOfThisSubtask() over the node's GPUs."""
    ndev = device_count() if ndev is None else ndev
    d = ctypes.c_int32(0)
    check(lib().sky_device_for_subtask(int(subtask), int(ndev), ctypes.byref(d)))
    return d.value


class _LocalPart:
    def __init__(self, engine, key):
        h = ctypes.c_void_p()
        check(lib().sky_part_open(engine.h, key, ctypes.byref(h)))
        self.h = h
        self.dims = engine.dims

    def insert(self, ids, vals):
        ids = np.ascontiguousarray(ids, np.int64)
        vals = np.ascontiguousarray(vals, np.float64)
        check(lib().sky_part_insert(self.h, ids.ctypes.data_as(ctypes.c_void_p),
                                    vals.ctypes.data_as(ctypes.c_void_p), len(ids)))

    @staticmethod
    def insert_many(parts, batches):
        """One sky_parts_insert call: batches[g] = (ids, values) for parts[g] (parts of one engine):
        the full buffers of several keys flushed in one launch set, asynchronously."""
        n = len(parts)
        if n == 0:
            return
        ids = [np.ascontiguousarray(b[0], np.int64) for b in batches]
        vals = [np.ascontiguousarray(b[1], np.float64) for b in batches]
        ph = (ctypes.c_void_p * n)(*[p.h.value for p in parts])
        ip = (ctypes.c_void_p * n)(*[a.ctypes.data for a in ids])
        vp = (ctypes.c_void_p * n)(*[a.ctypes.data for a in vals])
        cnt = np.array([len(a) for a in ids], np.int64)
        check(lib().sky_parts_insert(n, ph, ip, vp, cnt.ctypes.data_as(ctypes.c_void_p)))

    @staticmethod
    def global_merge_many(engine, parts, part_ids=None):
        """sky_parts_global_merge: GlobalSkylineAggregator over the parts' device-resident local
        skylines (no snapshot through host memory) -> (ids, origins), part order then insertion
        order; engine.stats() then holds |L_k| / survivors_k as after engine.global_merge."""
        n = len(parts)
        ph = (ctypes.c_void_p * max(n, 1))(*[p.h.value for p in parts])
        pids = np.ascontiguousarray(part_ids if part_ids is not None else np.arange(n), np.int32)
        g = sum(p.size() for p in parts)          # a bound: every part's local skyline
        out_ids = np.empty(max(g, 1), np.int64)
        out_org = np.empty(max(g, 1), np.int32)
        cnt = ctypes.c_int64(0)
        check(lib().sky_parts_global_merge(engine.h, n, ph, pids.ctypes.data_as(ctypes.c_void_p),
                                           out_ids.ctypes.data_as(ctypes.c_void_p),
                                           out_org.ctypes.data_as(ctypes.c_void_p), g, ctypes.byref(cnt)))
        return out_ids[:cnt.value].copy(), out_org[:cnt.value].copy()

    def size(self):
        n = ctypes.c_int64(0)
        check(lib().sky_part_size(self.h, ctypes.byref(n)))
        return n.value

    def snapshot(self):
        n = ctypes.c_int64(0)
        check(lib().sky_part_size(self.h, ctypes.byref(n)))
        ids = np.empty(max(n.value, 1), np.int64)
        vals = np.empty((max(n.value, 1), self.dims), np.float64)
        check(lib().sky_part_snapshot(self.h, ids.ctypes.data_as(ctypes.c_void_p),
                                      vals.ctypes.data_as(ctypes.c_void_p), n.value, ctypes.byref(n)))
        return ids[:n.value].copy(), vals[:n.value].copy()

    def snapshot_reps(self):
        """sky_part_sizes + sky_part_snapshot_reps: the local skyline as distinct vectors."""
        n, r = ctypes.c_int64(0), ctypes.c_int64(0)
        check(lib().sky_part_sizes(self.h, ctypes.byref(n), ctypes.byref(r)))
        ids = np.empty(max(n.value, 1), np.int64)
        rep = np.empty(max(n.value, 1), np.int32)
        reps = np.empty((max(r.value, 1), self.dims), np.float64)
        rcnt = np.empty(max(r.value, 1), np.int32)
        check(lib().sky_part_snapshot_reps(self.h, ids.ctypes.data_as(ctypes.c_void_p),
                                           rep.ctypes.data_as(ctypes.c_void_p), n.value,
                                           reps.ctypes.data_as(ctypes.c_void_p),
                                           rcnt.ctypes.data_as(ctypes.c_void_p), r.value,
                                           ctypes.byref(n), ctypes.byref(r)))
        return LocalSkyline(ids[:n.value].copy(), rep[:n.value].copy(), reps[:r.value].copy(), rcnt[:r.value].copy())

    def close(self):
        if self.h:
            lib().sky_part_close(self.h)
            self.h = None


class LocalSkyline:
    """The message LocalProcessor.processQuery sends to the aggregator (field 4 of the Tuple6 of
    FlinkSkyline.java:396-403, there a List<ServiceTuple>): the tuples (ids, rep index) in
    insertion order and their distinct vectors with tuple counts -- on the reference streams
    key 0's local skyline is millions of copies of one vector."""

    __slots__ = ("ids", "rep_idx", "reps", "rep_counts")

    def __init__(self, ids, rep_idx, reps, rep_counts):
        self.ids, self.rep_idx, self.reps, self.rep_counts = ids, rep_idx, reps, rep_counts

    def __len__(self):
        return len(self.ids)

    def values(self):
        """The expanded rows (the reference's List<ServiceTuple> values), n x dims."""
        return self.reps[self.rep_idx] if len(self.ids) else self.reps[:0]


class SkylineLocalProcessor:
    """FlinkSkyline.SkylineLocalProcessor (:214-445) over sky_part_* state.

    processElement1(point, key, out)   data input (:265-316)
    processElement2(trigger, out)      trigger input, trigger = (partitionId, payload, dispatchMs) (:330-356)
    Emits Tuple6 = (partitionId, payload, dispatchMs, partitionStartMs, localSkyline, cpuMillis) (:396-403),
    the local skyline as (ids ndarray, values ndarray).
    """

    BUFFER_SIZE = 5000   # :232

    def __init__(self, engine, barrier="per-key"):
        """barrier="per-key": the reference's release rule, per key maxId >= R (:306,351),
        kept with its off-by-one and its wait for a later tuple.  barrier="global" (SURVEY
        §8f row 3): a query "q,R" covers exactly the ids < R -- it is released once every id
        < R has been ingested (ids arrive dense and in order, unified_producer.py:174-185),
        and tuples with id >= R are held back until then, so the answer does not depend on
        timing and no key waits for a tuple it never gets."""
        if barrier not in ("per-key", "global"):
            raise ValueError("barrier must be 'per-key' or 'global'")
        self.barrier = barrier
        self.watermark = 0               # global: every id < watermark has been ingested
        self.held = []                   # global: (point, key) with id >= a pending R
        self.engine = engine
        self.localSkylineState = {}      # key -> _LocalPart
        self.inputBuffer = {}            # key -> list of (id, values)
        self.maxSeenIdState = {}
        self.pendingQueriesState = {}
        self.startTimeState = {}
        self.accumulatedCpuNanosState = {}

    def _state(self, key):
        if key not in self.localSkylineState:
            self.localSkylineState[key] = _LocalPart(self.engine, key)
            self.inputBuffer[key] = []
        return self.localSkylineState[key]

    def _min_pending(self):
        rs = [self._required(q) for qs in self.pendingQueriesState.values() for q in qs]
        return min(rs) if rs else None

    @staticmethod
    def _required(q):
        """requiredCount of a trigger payload "q,R" (FlinkSkyline.java:303-305, :333-334):
        split(",") and Long.parseLong with no trim, so "q, 1000" fails as it does there."""
        parts = java_split(q[1])
        return java_parse_long(parts[1]) if len(parts) > 1 else 0

    # ---- checkpoints (the reference's localSkylineState is Flink keyed state, :243-248) ----
    def snapshot_state(self):
        """What a checkpoint stores: every key's local skyline (ids, values), its buffered
        tuples flushed into the device state first (HipSkylineOperators.snapshotState)."""
        out = {}
        for key in list(self.localSkylineState):
            if self.inputBuffer.get(key):
                self.processBuffer(key)
            out[key] = self.localSkylineState[key].snapshot()
        return out

    def restore_state(self, state):
        """Restore by insert into fresh device state: SKY(empty u S) = S, insertion order kept
        (HipSkylineOperators.initializeState + open)."""
        for key, (ids, vals) in state.items():
            part = self._state(key)
            if len(ids):
                part.insert(ids, vals)

    def _release_global(self, out):
        """Answer every pending query whose ids < R are all in, then replay held tuples."""
        while True:
            released = False
            for key, pending in list(self.pendingQueriesState.items()):
                keep = []
                for q in pending:
                    if self._required(q) <= self.watermark:
                        self.processQuery(q, key, out)
                        released = True
                    else:
                        keep.append(q)
                self.pendingQueriesState[key] = keep
            if not released or not self.held:
                return
            held, self.held = self.held, []
            for point, key in held:
                self._ingest_global(point, key, out)

    def _ingest_global(self, point, key, out):
        if point.bad_id:
            raise ValueError('NumberFormatException: For input string: "%s"' % point.id)
        current_id = int(point.id)
        rmin = self._min_pending()
        if rmin is not None and current_id >= rmin:   # belongs after the pending query
            self.held.append((point, key))
            return
        self._state(key)
        if key not in self.startTimeState:
            self.startTimeState[key] = now_ms()
        if current_id > self.maxSeenIdState.get(key, -1):
            self.maxSeenIdState[key] = current_id
        buf = self.inputBuffer[key]
        buf.append((current_id, point.values))
        if len(buf) >= self.BUFFER_SIZE:
            self.processBuffer(key)
        self.watermark = max(self.watermark, current_id + 1)

    def processElement1(self, point, key, out):
        if self.barrier == "global":
            start = time.perf_counter_ns()
            self._ingest_global(point, key, out)
            self.accumulatedCpuNanosState[key] = self.accumulatedCpuNanosState.get(key, 0) + \
                (time.perf_counter_ns() - start)
            self._release_global(out)
            return
        start = time.perf_counter_ns()
        self._state(key)
        if key not in self.startTimeState:
            self.startTimeState[key] = now_ms()
        if point.bad_id:                                             # Long.parseLong throws (:276)
            raise ValueError('NumberFormatException: For input string: "%s"' % point.id)
        current_id = int(point.id)                                   # Long.parseLong (:276)
        max_id = self.maxSeenIdState.get(key, -1)
        if current_id > max_id:
            self.maxSeenIdState[key] = current_id
            max_id = current_id
        buf = self.inputBuffer[key]
        buf.append((current_id, point.values))
        if len(buf) >= self.BUFFER_SIZE:
            self.processBuffer(key)
        self.accumulatedCpuNanosState[key] = self.accumulatedCpuNanosState.get(key, 0) + \
            (time.perf_counter_ns() - start)
        pending = self.pendingQueriesState.get(key)
        if pending:
            remaining = []
            processed = False
            for q in pending:
                required = self._required(q)
                if max_id >= required:
                    self.processQuery(q, key, out)
                    processed = True
                else:
                    remaining.append(q)
            if processed:
                self.pendingQueriesState[key] = remaining

    def processElement2(self, trigger, out):
        key = trigger[0]
        required = self._required(trigger)
        if self.barrier == "global":
            if self.watermark >= required:
                self.processQuery(trigger, key, out)
            else:
                self.pendingQueriesState.setdefault(key, []).append(trigger)
            return
        current = self.maxSeenIdState.get(key, -1)
        if current >= required or current == -1:
            self.processQuery(trigger, key, out)
        else:
            self.pendingQueriesState.setdefault(key, []).append(trigger)

    def processQuery(self, trigger, key, out):
        start = time.perf_counter_ns()
        self._state(key)
        if self.inputBuffer[key]:
            self.processBuffer(key)
        total = self.accumulatedCpuNanosState.get(key, 0) + (time.perf_counter_ns() - start)
        self.accumulatedCpuNanosState[key] = total
        part_start = self.startTimeState.get(key, now_ms())
        sky = self.localSkylineState[key].snapshot_reps()
        out.append((trigger[0], trigger[1], trigger[2], part_start, sky, total // 1_000_000))

    def processBuffer(self, key):
        """S <- SKY(S u buffer) on the device (the BNL of :417-444)."""
        buf = self.inputBuffer[key]
        if not buf:
            return
        ids = np.fromiter((b[0] for b in buf), np.int64, len(buf))
        vals = np.asarray([b[1] for b in buf], np.float64).reshape(len(buf), self.engine.dims)
        self.localSkylineState[key].insert(ids, vals)
        buf.clear()

    def close(self):
        for p in self.localSkylineState.values():
            p.close()
        self.localSkylineState.clear()


class GlobalSkylineAggregator:
    """FlinkSkyline.GlobalSkylineAggregator (:460-660).  Collects the P local
    skylines of one query key and, on the last arrival, merges them on the
    device (sky_global_merge_reps over the distinct-vector messages) and emits the JSON
    payload (:631-648)."""

    def __init__(self, engine, totalPartitions):
        self.engine = engine
        self.totalPartitions = int(totalPartitions)
        self.state = {}

    def processElement(self, inp, out):
        pid, payload, dispatch_ms, pstart, sky, cpu_ms = inp
        st = self.state.setdefault(payload, {"lists": [], "count": 0, "minStart": None, "lastArr": None,
                                             "maxCpu": None})
        if st["minStart"] is None or (pstart is not None and pstart < st["minStart"]):
            st["minStart"] = pstart
        st["lastArr"] = now_ms()
        if st["maxCpu"] is None or cpu_ms > st["maxCpu"]:
            st["maxCpu"] = cpu_ms
        st["lists"].append((pid, sky))
        st["count"] += 1
        if st["count"] >= self.totalPartitions:
            lists = st["lists"]
            gids, gorg = self.engine.global_merge_reps(
                [l[0] for l in lists], [(l[1].ids, l[1].rep_idx, l[1].reps, l[1].rep_counts) for l in lists])
            finish = now_ms()
            job_start = st["minStart"]
            map_finish = st["lastArr"]
            map_wall = (map_finish - job_start) if job_start is not None else 0
            local_t = st["maxCpu"] or 0
            ingest = max(0, map_wall - local_t)
            global_t = finish - map_finish
            total_t = (finish - job_start) if job_start is not None else 0
            latency = finish - dispatch_ms
            # optimality (:593-608): the local size of partition i is its list size
            sizes = {}
            for l in lists:
                sizes[l[0]] = len(l[1])      # the list's tuple count
            surv = {}
            for o in gorg.tolist():
                surv[o] = surv.get(o, 0) + 1
            s = 0.0
            for i in range(self.totalPartitions):
                if i in sizes and sizes[i] > 0:
                    s += surv.get(i, 0) / sizes[i]
            optimality = s / self.totalPartitions
            parts = java_split(payload)
            qid = parts[0]
            rec = parts[1] if len(parts) > 1 else "unknown"
            js = ('{"query_id": "%s", "record_count": %s, "skyline_size": %d, "optimality": %s, '
                  '"ingestion_time_ms": %d, "local_processing_time_ms": %d, "global_processing_time_ms": %d, '
                  '"total_processing_time_ms": %d, "query_latency_ms": %d}') % (
                qid, rec, len(gids), java_format_4f(optimality), ingest, local_t, global_t, total_t, latency)
            out.append(js)
            st["result_ids"] = gids
            del self.state[payload]
            self.last_result = (gids, gorg)


def run_job(csv_lines, triggers, algo="mr-angle", parallelism=4, dims=2, domain=1000.0, device=0,
            barrier="per-key", out=None):
    """Single-process rendition of the topology of FlinkSkyline.main (:61-186):
    parse -> keyBy(partitioner) -> SkylineLocalProcessor <- broadcast triggers
    -> keyBy(payload) -> GlobalSkylineAggregator.  `triggers` is a list of
    (position, payload): the trigger is injected after that many input lines,
    like unified_producer.py:177-185.  Returns the emitted JSON strings and the
    result ids of the last query.  `out`: an optional list the JSON strings are appended to as
    they are emitted (still filled when a later record fails the job)."""
    P = 2 * parallelism
    part = make_partitioner(algo, P, domain, dims, device)
    eng = part.engine
    local = SkylineLocalProcessor(eng, barrier)
    glob = GlobalSkylineAggregator(eng, P)
    emitted = []
    results = out if out is not None else []
    tuples = ServiceTuple.fromStrings(csv_lines, eng)                 # .map(fromString) (:103), on the device
    valid = [t for t in tuples if t is not None]
    # keys only for tuples with values; a bad-id tuple gets a placeholder key and raises
    # its NumberFormatException in stream order, at processElement1 (:276)
    good = [t for t in valid if not t.bad_id]
    gkeys = part.getKeys(np.asarray([t.values for t in good], np.float64)) if good else []
    keys, gi = [], 0
    for t in valid:
        if t.bad_id:
            keys.append(0)
        else:
            keys.append(int(gkeys[gi]))
            gi += 1
    trig = sorted(triggers)
    ti = 0
    pos = 0

    def fire(payload):
        start = now_ms()
        for i in range(P):                                            # broadcast (:152-154)
            local.processElement2((i, payload, start), emitted)
        drain()

    def drain():
        while emitted:
            glob.processElement(emitted.pop(0), results)

    vi = 0
    for t in tuples:
        while ti < len(trig) and trig[ti][0] <= pos:
            fire(trig[ti][1])
            ti += 1
        if t is not None:
            local.processElement1(t, int(keys[vi]), emitted)
            vi += 1
            drain()
        pos += 1
    while ti < len(trig):
        fire(trig[ti][1])
        ti += 1
    last = getattr(glob, "last_result", None)
    local.close()
    return results, last
