package org.main;

/**
 * JNI entry points of libskyline_hip.so (include/skyline_hip.h, via jni/skyline_hip_jni.c).
 *
 * Not compiled in the build container (no JDK there); the same call sequence is exercised by
 * tests/operator_replay.c (C) and by the Python binding (flink-skyline-qos_amd/skyline/).
 *
 * Handles are opaque longs.  Arrays: ids long[n], values double[n * dims] row-major.
 * Failures throw RuntimeException(sky_last_error()); a NaN value throws ArithmeticException;
 * arrays shorter than the call needs throw IllegalArgumentException.
 * Methods returning an int count return -required when an output array is too small.
 */
public final class SkylineHip {
    static {
        System.loadLibrary("skyline_hip_jni");   // links libskyline_hip.so
    }

    private SkylineHip() {}

    /** FlinkSkyline.main --algo values (FlinkSkyline.java:112-134). */
    public static final int ALGO_DIM = 0, ALGO_GRID = 1, ALGO_ANGLE = 2;
    public static final int SEM_REFERENCE = 0, SEM_COMPLETE = 1;
    public static final int CSV_MALFORMED = 1, CSV_BAD_ID = 2, CSV_ARITY = 3;

    public static int algoOf(String flag) {
        switch (flag.toLowerCase()) {
            case "mr-dim": return ALGO_DIM;
            case "mr-grid": return ALGO_GRID;
            default: return ALGO_ANGLE;            // the reference's default branch
        }
    }

    /** HIP devices this TaskManager process sees (0 without a GPU). */
    public static native int deviceCount();
    /** The device of subtask `subtask`: subtask % ndev (sky_device_for_subtask). */
    public static native int deviceForSubtask(int subtask, int ndev);

    public static native long ctxCreate(int device, int dims, int partitions, int algo, double domain);
    public static native void ctxDestroy(long ctx);
    public static native void ctxWarmup(long ctx);            // once in open(): first launches off the query path
    public static native void ctxSetSemantics(long ctx, int semantics);
    public static native void ctxSetGridFilter(long ctx, boolean on);

    public static native void partitionKeys(long ctx, double[] values, int n, int[] keysOut);

    public static native long partOpen(long ctx, int key);
    public static native void partClose(long part);
    public static native void partInsert(long part, long[] ids, double[] values, int n);
    /** the full buffers of several keys (parts of one context) in one launch set */
    public static native void partsInsert(long[] parts, long[][] ids, double[][] values, int[] counts);
    public static native long partSize(long part);
    public static native int partSnapshot(long part, long[] idsOut, double[] valuesOut);
    /** sizesOut[0] = tuples T, sizesOut[1] = distinct vectors R of the local skyline. */
    public static native void partSizes(long part, long[] sizesOut);
    /** The local skyline as distinct vectors: ids[T], repIdx[T], reps[R * dims], repCounts[R];
     *  returns T, or -T when an array is too small. */
    public static native int partSnapshotReps(long part, long[] idsOut, int[] repIdxOut, double[] repsOut,
                                              int[] repCountsOut);

    /** GlobalSkylineAggregator over the parts' device-resident states (co-located aggregator):
     *  the skyline size, or -(needed) when idsOut is too short. */
    public static native int partsGlobalMerge(long ctx, long[] parts, int[] partIds, long[] idsOut, int[] originOut);
    public static native int globalMerge(long ctx, int[] partIds, long[][] ids, double[][] values,
                                         long[] idsOut, int[] originOut);
    /** globalMerge over partSnapshotReps messages: same ids, order, origins and stats. */
    public static native int globalMergeReps(long ctx, int[] partIds, long[][] ids, int[][] repIdx, double[][] reps,
                                             int[][] repCounts, long[] idsOut, int[] originOut);
    /** The optimality integers of the last merge / query (FlinkSkyline.java:593-608), indexed like
     *  its lists.  Returns K; with null arrays only K (size the arrays from it).  Arrays shorter
     *  than K are left untouched and -K is returned: callers must treat a negative return as an
     *  error. */
    public static native int globalStats(long ctx, long[] localSizes, long[] survivors);

    public static native int query(long ctx, long[] ids, double[] values, int n, long[] idsOut, int[] originOut);

    public static native int parseCsv(long ctx, byte[] text, int nbytes, long[] idsOut, double[] valuesOut,
                                      long[] countsOut);

    public static native long streamCreate(long ctx, long window);
    public static native void streamDestroy(long stream);
    public static native void streamAppend(long stream, long[] ids, double[] values, int n);
    public static native int streamQuery(long stream, long[] idsOut, int[] originOut);
    public static native void streamReserve(long stream, long tuples);
    public static native long streamResident(long stream);
}
