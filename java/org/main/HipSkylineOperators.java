package org.main;

import org.apache.flink.api.common.state.ListState;
import org.apache.flink.api.common.state.ListStateDescriptor;
import org.apache.flink.api.common.state.ValueState;
import org.apache.flink.api.common.state.ValueStateDescriptor;
import org.apache.flink.api.common.typeinfo.TypeHint;
import org.apache.flink.api.common.typeinfo.TypeInformation;
import org.apache.flink.api.java.tuple.Tuple3;
import org.apache.flink.api.java.tuple.Tuple6;
import org.apache.flink.configuration.Configuration;
import org.apache.flink.runtime.state.FunctionInitializationContext;
import org.apache.flink.runtime.state.FunctionSnapshotContext;
import org.apache.flink.runtime.state.KeyGroupRangeAssignment;
import org.apache.flink.streaming.api.checkpoint.CheckpointedFunction;
import org.apache.flink.streaming.api.functions.KeyedProcessFunction;
import org.apache.flink.streaming.api.functions.co.KeyedCoProcessFunction;
import org.apache.flink.util.Collector;

import java.util.ArrayList;
import java.util.HashMap;
import java.util.List;
import java.util.Locale;
import java.util.Map;

/**
 * Drop-in replacements for the two hot-path operators of FlinkSkyline.java, running their
 * dominance work in libskyline_hip.so on the MI355X (through SkylineHip / JNI).
 *
 * Devices: every subtask creates its context on SkylineHip.deviceForSubtask(getIndexOfThisSubtask(),
 * deviceCount()), so the `parallelism` subtasks of an operator (FlinkSkyline.java:66,76,138)
 * spread round-robin over the node's GPUs; a TaskManager without a GPU fails in open().
 *
 * The local skylines travel between the two operators as LocalSkyline messages (field 4 of the
 * Tuple6, a List<ServiceTuple> in the reference, :396-403): the tuples as (id, index of their
 * vector) and the distinct vectors with their tuple counts -- on the reference streams key 0's
 * 4.4M skyline tuples are one all-zero vector, so the message is 12 bytes per tuple and no
 * ServiceTuple objects are built on either side.
 *
 * Topology change in FlinkSkyline.main (:162-176):
 *   keyedData.connect(keyedTriggers).process(new HipSkylineOperators.LocalProcessor(dims, P, algo, domain))
 *   ...keyBy(t -> t.f1).process(new HipSkylineOperators.GlobalAggregator(P, dims, algo, domain))
 * Everything else (Kafka source and sink, fromString, the partitioners, the trigger
 * broadcast) is unchanged.  Not compiled in the build container (no JDK); the identical C
 * call sequence runs in tests/operator_replay.c on the GPU box.
 *
 * Deliberate differences from the reference (DESIGN.md §5): the input buffer is per key (the
 * reference's is shared by a subtask's keys, :223,244); NaN values fail the task
 * (ArithmeticException); the JSON adds "query_latency_ms" (computed at :588, never emitted).
 * Trigger payloads are parsed exactly as the reference does (split(","), Long.parseLong without
 * trim, :303-305, :333-334, :627-629): "q, 1000" throws NumberFormatException in both.
 * Checkpoints: the reference keeps localSkylineState in Flink keyed state (:243-248); the device
 * state is written into union operator state at every checkpoint (snapshotState) and re-inserted
 * into fresh device state on restore (initializeState + open), each subtask taking its keys.
 */
public final class HipSkylineOperators {
    private HipSkylineOperators() {}

    static final int BUFFER_SIZE = 5000;   // FlinkSkyline.java:232

    /** Per-key tuple buffer flattened for one JNI call. */
    static final class KeyBuffer {
        final long[] ids = new long[BUFFER_SIZE];
        final double[] values;
        final int dims;
        int n;

        KeyBuffer(int dims) {
            this.dims = dims;
            this.values = new double[BUFFER_SIZE * dims];
        }

        boolean add(long id, double[] v) {
            ids[n] = id;
            System.arraycopy(v, 0, values, n * dims, dims);
            return ++n == BUFFER_SIZE;
        }
    }

    /** A local skyline as distinct vectors (sky_part_snapshot_reps): tuple i is ids[i] with the
     *  values reps[repIdx[i] * dims ..]; repCounts[r] = tuples on vector r.  A Flink POJO. */
    public static final class LocalSkyline {
        public long[] ids;
        public int[] repIdx;
        public double[] reps;
        public int[] repCounts;

        public LocalSkyline() {}

        LocalSkyline(long[] ids, int[] repIdx, double[] reps, int[] repCounts) {
            this.ids = ids;
            this.repIdx = repIdx;
            this.reps = reps;
            this.repCounts = repCounts;
        }

        public int size() {
            return ids.length;
        }
    }

    /** The context of this subtask, on its GPU (see the class comment). */
    static long openContext(org.apache.flink.api.common.functions.RuntimeContext rc, int dims, int partitions,
                            int algo, double domain) {
        final int ndev = SkylineHip.deviceCount();
        if (ndev < 1) throw new IllegalStateException("no HIP device visible to this TaskManager");
        final long ctx = SkylineHip.ctxCreate(SkylineHip.deviceForSubtask(rc.getIndexOfThisSubtask(), ndev), dims,
                partitions, algo, domain);
        SkylineHip.ctxWarmup(ctx);                     // first kernel launches off the query path
        return ctx;
    }

    /**
     * SkylineLocalProcessor (FlinkSkyline.java:214-445) with the per-key skyline held on the
     * device: processBuffer's BNL (:417-444) is an asynchronous sky_parts_insert of the full
     * buffers of up to FLUSH_GROUP keys; processQuery's snapshot (:387-392) is
     * sky_part_snapshot_reps (after every waiting buffer).  The id barrier (:276-356) is unchanged.
     * A device error or NaN in a buffer held back for its flush group surfaces at the flush, from
     * whichever element, query or checkpoint triggers it; its message names the key whose batch
     * failed ("batch of key k").
     */
    public static class LocalProcessor extends KeyedCoProcessFunction<Integer, ServiceTuple,
            Tuple3<Integer, String, Long>, Tuple6<Integer, String, Long, Long, LocalSkyline, Long>>
            implements CheckpointedFunction {
        private final int dims, partitions, algo;
        private final double domain;
        private transient long ctx;
        private transient Map<Integer, Long> parts;          // key -> sky_part handle
        private transient Map<Integer, KeyBuffer> buffers;   // key -> pending tuples
        private transient ValueState<Long> maxSeenIdState;
        private transient ListState<Tuple3<Integer, String, Long>> pendingQueriesState;
        private transient ValueState<Long> startTimeState;
        private transient ValueState<Long> accumulatedCpuNanosState;
        // the device skylines at the last checkpoint: (key, ids, values row-major), union-redistributed
        private transient ListState<Tuple3<Integer, long[], double[]>> checkpointedSkylines;
        private transient List<Tuple3<Integer, long[], double[]>> restored;

        public LocalProcessor(int dims, int partitions, String algo, double domain) {
            this.dims = dims;
            this.partitions = partitions;
            this.algo = SkylineHip.algoOf(algo);
            this.domain = domain;
        }

        @Override
        public void open(Configuration config) {
            ctx = openContext(getRuntimeContext(), dims, partitions, algo, domain);
            parts = new HashMap<>();
            buffers = new HashMap<>();
            maxSeenIdState = getRuntimeContext().getState(new ValueStateDescriptor<>("maxId", Long.class));
            pendingQueriesState = getRuntimeContext().getListState(new ListStateDescriptor<>("pendingQs",
                    TypeInformation.of(new TypeHint<Tuple3<Integer, String, Long>>() {})));
            startTimeState = getRuntimeContext().getState(new ValueStateDescriptor<>("jobStartTime", Long.class));
            accumulatedCpuNanosState = getRuntimeContext().getState(new ValueStateDescriptor<>("cpuTime", Long.class));
            restoreInto();
        }

        /** Checkpoint: every key's device skyline (its buffered tuples flushed first, so nothing
         *  that arrived before the barrier is lost) into union operator state. */
        @Override
        public void snapshotState(FunctionSnapshotContext fc) throws Exception {
            checkpointedSkylines.clear();
            drainFull();
            for (int key : new ArrayList<>(buffers.keySet())) flush(key);
            for (Map.Entry<Integer, Long> e : parts.entrySet()) {
                final long p = e.getValue();
                int n = (int) SkylineHip.partSize(p);
                long[] ids = new long[n];
                double[] vals = new double[n * dims];
                n = SkylineHip.partSnapshot(p, ids, vals);
                checkpointedSkylines.add(Tuple3.of(e.getKey(), ids, vals));
            }
        }

        @Override
        public void initializeState(FunctionInitializationContext fc) throws Exception {
            checkpointedSkylines = fc.getOperatorStateStore().getUnionListState(new ListStateDescriptor<>(
                    "hipLocalSky", TypeInformation.of(new TypeHint<Tuple3<Integer, long[], double[]>>() {})));
            restored = new ArrayList<>();
            if (fc.isRestored())
                for (Tuple3<Integer, long[], double[]> t : checkpointedSkylines.get()) restored.add(t);
        }

        /** Restore by insert: SKY(empty u S) = S for a skyline S, insertion order kept; each
         *  subtask takes the keys of its key-group range (the state is union-redistributed). */
        private void restoreInto() {
            if (restored == null || restored.isEmpty()) return;
            final int maxPar = getRuntimeContext().getMaxNumberOfParallelSubtasks();
            final int par = getRuntimeContext().getNumberOfParallelSubtasks();
            final int idx = getRuntimeContext().getIndexOfThisSubtask();
            for (Tuple3<Integer, long[], double[]> t : restored) {
                if (KeyGroupRangeAssignment.assignKeyToParallelOperator(t.f0, maxPar, par) != idx) continue;
                if (t.f1.length > 0) SkylineHip.partInsert(part(t.f0), t.f1, t.f2, t.f1.length);
            }
            restored.clear();
        }

        @Override
        public void close() {   // the reference has no close(); device state is released here
            full = null;
            for (long p : parts.values()) SkylineHip.partClose(p);
            parts.clear();
            if (ctx != 0) SkylineHip.ctxDestroy(ctx);
            ctx = 0;
        }

        private long part(int key) {
            return parts.computeIfAbsent(key, k -> SkylineHip.partOpen(ctx, k));
        }

        // full buffers waiting to go to the device together (one partsInsert per round of keys)
        private static final int FLUSH_GROUP = 8;
        private transient List<Tuple3<Integer, KeyBuffer, Integer>> full;

        /** processBuffer for every full buffer waiting: S <- SKY(S u buffer) per key, in one
         *  asynchronous launch set per round (a key appears once per round, in arrival order). */
        private void drainFull() {
            if (full == null || full.isEmpty()) return;
            while (!full.isEmpty()) {
                List<Tuple3<Integer, KeyBuffer, Integer>> round = new ArrayList<>(), later = new ArrayList<>();
                java.util.Set<Integer> seen = new java.util.HashSet<>();
                for (Tuple3<Integer, KeyBuffer, Integer> t : full) (seen.add(t.f0) ? round : later).add(t);
                long[] ps = new long[round.size()];
                long[][] is = new long[round.size()][];
                double[][] vs = new double[round.size()][];
                int[] cs = new int[round.size()];
                for (int g = 0; g < round.size(); g++) {
                    Tuple3<Integer, KeyBuffer, Integer> t = round.get(g);
                    ps[g] = part(t.f0);
                    is[g] = t.f1.ids;
                    vs[g] = t.f1.values;
                    cs[g] = t.f2;
                }
                SkylineHip.partsInsert(ps, is, vs, cs);    // copied before it returns
                full = later;
            }
        }

        private void flush(int key) {
            drainFull();
            KeyBuffer b = buffers.get(key);
            if (b != null && b.n > 0) {
                SkylineHip.partInsert(part(key), b.ids, b.values, b.n);   // S <- SKY(S u buffer)
                b.n = 0;
            }
        }

        private static long required(Tuple3<Integer, String, Long> q) {   // :303-305, :333-334
            String[] parts = q.f1.split(",");
            return parts.length > 1 ? Long.parseLong(parts[1]) : 0L;
        }

        private void addCpu(long startNano) throws Exception {
            Long acc = accumulatedCpuNanosState.value();
            accumulatedCpuNanosState.update((acc == null ? 0L : acc) + (System.nanoTime() - startNano));
        }

        @Override
        public void processElement1(ServiceTuple point, Context c,
                                    Collector<Tuple6<Integer, String, Long, Long, LocalSkyline, Long>> out)
                throws Exception {
            final long startNano = System.nanoTime();
            final int key = c.getCurrentKey();
            if (startTimeState.value() == null) startTimeState.update(System.currentTimeMillis());
            final long id = Long.parseLong(point.id);                // throws as the reference does (:276)
            Long maxId = maxSeenIdState.value();
            if (maxId == null || id > maxId) {
                maxSeenIdState.update(id);
                maxId = id;
            }
            if (buffers.computeIfAbsent(key, k -> new KeyBuffer(dims)).add(id, point.values)) {
                // the full buffer waits for FLUSH_GROUP of them; the key continues in a fresh one
                if (full == null) full = new ArrayList<>();
                full.add(Tuple3.of(key, buffers.get(key), BUFFER_SIZE));
                buffers.put(key, new KeyBuffer(dims));
                if (full.size() >= FLUSH_GROUP) drainFull();
            }
            addCpu(startNano);
            List<Tuple3<Integer, String, Long>> remaining = new ArrayList<>();
            boolean released = false;
            for (Tuple3<Integer, String, Long> q : pendingQueriesState.get()) {
                if (maxId >= required(q)) {
                    processQuery(q, key, out);
                    released = true;
                } else {
                    remaining.add(q);
                }
            }
            if (released) pendingQueriesState.update(remaining);
        }

        @Override
        public void processElement2(Tuple3<Integer, String, Long> trigger, Context c,
                                    Collector<Tuple6<Integer, String, Long, Long, LocalSkyline, Long>> out)
                throws Exception {
            Long current = maxSeenIdState.value();
            long cur = current == null ? -1L : current;
            if (cur >= required(trigger) || cur == -1L) processQuery(trigger, c.getCurrentKey(), out);
            else pendingQueriesState.add(trigger);
        }

        private void processQuery(Tuple3<Integer, String, Long> trigger, int key,
                                  Collector<Tuple6<Integer, String, Long, Long, LocalSkyline, Long>> out)
                throws Exception {
            final long startNano = System.nanoTime();
            flush(key);
            final long p = part(key);
            final long[] sizes = new long[2];
            SkylineHip.partSizes(p, sizes);                // the one synchronisation of the query
            final int n = (int) sizes[0], r = (int) sizes[1];
            final LocalSkyline sky = new LocalSkyline(new long[n], new int[n], new double[r * dims], new int[r]);
            SkylineHip.partSnapshotReps(p, sky.ids, sky.repIdx, sky.reps, sky.repCounts);
            addCpu(startNano);
            Long start = startTimeState.value();
            Long cpu = accumulatedCpuNanosState.value();
            out.collect(new Tuple6<>(trigger.f0, trigger.f1, trigger.f2,
                    start == null ? System.currentTimeMillis() : start, sky, cpu == null ? 0L : cpu / 1_000_000L));
        }
    }

    /**
     * GlobalSkylineAggregator (FlinkSkyline.java:460-660): collects the P local skylines of one
     * query, then ONE sky_global_merge_reps (the BNL merge of :548-566 over the distinct-vector
     * messages) and sky_global_stats (the optimality integers of :593-608) on the last arrival,
     * and the JSON payload of :631-648.
     */
    public static class GlobalAggregator extends KeyedProcessFunction<String,
            Tuple6<Integer, String, Long, Long, LocalSkyline, Long>, String> {
        private final int totalPartitions, dims, algo;
        private final double domain;
        private transient long ctx;
        private transient ValueState<List<Tuple6<Integer, String, Long, Long, LocalSkyline, Long>>> arrived;
        private transient ValueState<Long> minStartTimeState;

        public GlobalAggregator(int totalPartitions, int dims, String algo, double domain) {
            this.totalPartitions = totalPartitions;
            this.dims = dims;
            this.algo = SkylineHip.algoOf(algo);
            this.domain = domain;
        }

        @Override
        public void open(Configuration config) {
            ctx = openContext(getRuntimeContext(), dims, totalPartitions, algo, domain);
            arrived = getRuntimeContext().getState(new ValueStateDescriptor<>("arrived",
                    TypeInformation.of(new TypeHint<List<Tuple6<Integer, String, Long, Long, LocalSkyline, Long>>>() {})));
            minStartTimeState = getRuntimeContext().getState(new ValueStateDescriptor<>("minStart", Long.class));
        }

        @Override
        public void close() {
            if (ctx != 0) SkylineHip.ctxDestroy(ctx);
            ctx = 0;
        }

        @Override
        public void processElement(Tuple6<Integer, String, Long, Long, LocalSkyline, Long> in, Context c,
                                   Collector<String> out) throws Exception {
            Long minStart = minStartTimeState.value();
            if (minStart == null || in.f3 < minStart) minStartTimeState.update(in.f3);
            List<Tuple6<Integer, String, Long, Long, LocalSkyline, Long>> lists = arrived.value();
            if (lists == null) lists = new ArrayList<>();
            lists.add(in);
            if (lists.size() < totalPartitions) {
                arrived.update(lists);
                return;
            }
            final long lastArrival = System.currentTimeMillis();
            final int np = lists.size();
            int[] partIds = new int[np];
            long[][] ids = new long[np][];
            int[][] repIdx = new int[np][];
            double[][] reps = new double[np][];
            int[][] repCounts = new int[np][];
            long maxCpu = 0;
            int total = 0;
            for (int k = 0; k < np; k++) {
                Tuple6<Integer, String, Long, Long, LocalSkyline, Long> t = lists.get(k);
                partIds[k] = t.f0;
                ids[k] = t.f4.ids;
                repIdx[k] = t.f4.repIdx;
                reps[k] = t.f4.reps;
                repCounts[k] = t.f4.repCounts;
                total += t.f4.size();
                maxCpu = Math.max(maxCpu, t.f5);
            }
            long[] gids = new long[Math.max(total, 1)];
            int[] gorg = new int[Math.max(total, 1)];
            final int g = SkylineHip.globalMergeReps(ctx, partIds, ids, repIdx, reps, repCounts, gids, gorg);
            // the integers are indexed by list, like partIds; their count K comes from the library
            final int K = SkylineHip.globalStats(ctx, null, null);
            long[] lsz = new long[Math.max(K, 1)], surv = new long[Math.max(K, 1)];
            final int k2 = SkylineHip.globalStats(ctx, lsz, surv);
            if (K < 0 || k2 != K)
                throw new IllegalStateException("globalStats returned " + k2 + " (expected " + K + ")");
            double sum = 0.0;
            for (int k = 0; k < Math.min(np, K); k++)
                if (partIds[k] < totalPartitions && lsz[k] > 0) sum += (double) surv[k] / lsz[k];
            final double optimality = sum / totalPartitions;
            final long finish = System.currentTimeMillis();
            final long jobStart = minStartTimeState.value();
            final long mapWall = lastArrival - jobStart;
            final long ingest = Math.max(0, mapWall - maxCpu);
            String[] payload = in.f1.split(",");                       // :627-629
            String records = payload.length > 1 ? payload[1] : "unknown";
            out.collect("{\"query_id\": \"" + payload[0] + "\", \"record_count\": " + records
                    + ", \"skyline_size\": " + g
                    + ", \"optimality\": " + String.format(Locale.US, "%.4f", optimality)
                    + ", \"ingestion_time_ms\": " + ingest
                    + ", \"local_processing_time_ms\": " + maxCpu
                    + ", \"global_processing_time_ms\": " + (finish - lastArrival)
                    + ", \"total_processing_time_ms\": " + (finish - jobStart)
                    + ", \"query_latency_ms\": " + (finish - in.f2) + "}");
            arrived.clear();   // minStart survives, as in the reference (:653-657)
        }
    }
}
