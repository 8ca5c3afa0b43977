/*
 * jni/skyline_hip_jni.c — the JNI layer between the Java operators (java/org/main/SkylineHip.java)
 * and libskyline_hip.so (include/skyline_hip.h).  One native per ABI entry point the operators
 * use; every status != SKY_OK becomes a java.lang.RuntimeException carrying sky_last_error(),
 * except SKY_E_NAN, which becomes an ArithmeticException (the reference accepts NaN, and its
 * BNL result then depends on arrival order: FlinkSkyline.java:417-444).
 *
 * Build (on a host with a JDK; this container has none, so this file is not compiled here):
 *   gcc -O2 -shared -fPIC -I"$JAVA_HOME/include" -I"$JAVA_HOME/include/linux" -Iinclude \
 *       jni/skyline_hip_jni.c -Lflink-skyline-qos_amd/build -lskyline_hip \
 *       -Wl,-rpath,'$ORIGIN' -o libskyline_hip_jni.so
 *
 * Arrays cross as Java primitive arrays: ids long[n], values double[n*dims] (row-major, the
 * layout of ServiceTuple.values concatenated).  Every array is checked against what the C call
 * reads or writes (IllegalArgumentException otherwise), and a NULL from Get*Critical leaves the
 * pending OutOfMemoryError.  The library copies host buffers before it returns, so arrays are
 * pinned only for the duration of one call (GetPrimitiveArrayCritical, no JNI calls in
 * between).  Handles are jlong (uintptr_t) values of the C pointers.
 *
 * The C call sequence these natives produce is replayed by tests/operator_replay.c, which the
 * GPU test tests/test_gpu_replay.py runs on the golden streams.
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

#include "skyline_hip.h"

static jboolean fail(JNIEnv *env, int rc) {
    if (rc == SKY_OK) return JNI_FALSE;
    const char *cls = rc == SKY_E_NAN ? "java/lang/ArithmeticException" : "java/lang/RuntimeException";
    (*env)->ThrowNew(env, (*env)->FindClass(env, cls), sky_last_error());
    return JNI_TRUE;
}

static jboolean throw_arg(JNIEnv *env, const char *msg) {
    (*env)->ThrowNew(env, (*env)->FindClass(env, "java/lang/IllegalArgumentException"), msg);
    return JNI_TRUE;
}

/* every array a native reads or writes is checked against what the C call will touch: a
 * misuse from Java is an IllegalArgumentException, never an out-of-bounds native access */
static jboolean bad_len(JNIEnv *env, jarray a, jlong need, const char *what) {
    if (!a) return throw_arg(env, what);
    if ((jlong)(*env)->GetArrayLength(env, a) < need) return throw_arg(env, what);
    return JNI_FALSE;
}

/* GetPrimitiveArrayCritical may return NULL (out of memory): an OutOfMemoryError is pending */
#define CRIT(arr) ((*env)->GetPrimitiveArrayCritical(env, (arr), NULL))
#define UNCRIT(arr, p, mode) do { if (p) (*env)->ReleasePrimitiveArrayCritical(env, (arr), (p), (mode)); } while (0)

#define CTX(h) ((sky_ctx *)(uintptr_t)(h))
#define PART(h) ((sky_part *)(uintptr_t)(h))
#define STREAM(h) ((sky_stream *)(uintptr_t)(h))

static int ctx_dims(sky_ctx *c) {
    int32_t d = 0;
    return sky_ctx_info(c, &d, NULL, NULL) == SKY_OK ? d : -1;
}
static int part_dims(sky_part *p) {
    int32_t d = 0;
    return sky_part_info(p, NULL, &d) == SKY_OK ? d : -1;
}

/* ---- device map: which GPU a subtask's context goes on (FlinkSkyline.java:66,76,138) ---- */
JNIEXPORT jint JNICALL Java_org_main_SkylineHip_deviceCount(JNIEnv *env, jclass cls) {
    int32_t n = 0;
    if (fail(env, sky_device_count(&n))) return 0;
    return n;
}

JNIEXPORT jint JNICALL Java_org_main_SkylineHip_deviceForSubtask(JNIEnv *env, jclass cls, jint subtask, jint ndev) {
    int32_t d = 0;
    if (fail(env, sky_device_for_subtask(subtask, ndev, &d))) return 0;
    return d;
}

/* ---- context: SkylineLocalProcessor.open() / GlobalSkylineAggregator.open() ---- */
JNIEXPORT jlong JNICALL Java_org_main_SkylineHip_ctxCreate(JNIEnv *env, jclass cls, jint device, jint dims,
                                                            jint partitions, jint algo, jdouble domain) {
    sky_ctx *ctx = NULL;
    int dev = device;
    if (fail(env, sky_ctx_create(&dev, 1, dims, partitions, algo, domain, &ctx))) return 0;
    return (jlong)(uintptr_t)ctx;
}

JNIEXPORT void JNICALL Java_org_main_SkylineHip_ctxDestroy(JNIEnv *env, jclass cls, jlong ctx) {
    fail(env, sky_ctx_destroy(CTX(ctx)));
}

JNIEXPORT void JNICALL Java_org_main_SkylineHip_ctxWarmup(JNIEnv *env, jclass cls, jlong ctx) {
    fail(env, sky_ctx_warmup(CTX(ctx)));
}

JNIEXPORT void JNICALL Java_org_main_SkylineHip_ctxSetSemantics(JNIEnv *env, jclass cls, jlong ctx, jint sem) {
    fail(env, sky_ctx_set_semantics(CTX(ctx), sem));
}

JNIEXPORT void JNICALL Java_org_main_SkylineHip_ctxSetGridFilter(JNIEnv *env, jclass cls, jlong ctx, jboolean on) {
    fail(env, sky_ctx_set_grid_filter(CTX(ctx), on ? 1 : 0));
}

/* ---- partitioners: SkylinePartitioner.getKey over a batch (FlinkSkyline.java:675) ---- */
JNIEXPORT void JNICALL Java_org_main_SkylineHip_partitionKeys(JNIEnv *env, jclass cls, jlong ctx,
                                                               jdoubleArray values, jint n, jintArray keys_out) {
    const int D = ctx_dims(CTX(ctx));
    if (n < 0 || D < 1) { throw_arg(env, "partitionKeys: bad n or context"); return; }
    if (bad_len(env, values, (jlong)n * D, "partitionKeys: values shorter than n * dims") ||
        bad_len(env, keys_out, n, "partitionKeys: keysOut shorter than n"))
        return;
    jdouble *v = CRIT(values);
    jint *k = CRIT(keys_out);
    const int rc = v && k ? sky_partition_keys(CTX(ctx), v, n, (int32_t *)k) : SKY_E_NOMEM;
    UNCRIT(keys_out, k, 0);
    UNCRIT(values, v, JNI_ABORT);
    if (v && k) fail(env, rc);
}

/* ---- local operator state: localSkylineState + processBuffer (FlinkSkyline.java:221, :417-444) ---- */
JNIEXPORT jlong JNICALL Java_org_main_SkylineHip_partOpen(JNIEnv *env, jclass cls, jlong ctx, jint key) {
    sky_part *p = NULL;
    if (fail(env, sky_part_open(CTX(ctx), key, &p))) return 0;
    return (jlong)(uintptr_t)p;
}

JNIEXPORT void JNICALL Java_org_main_SkylineHip_partClose(JNIEnv *env, jclass cls, jlong part) {
    fail(env, sky_part_close(PART(part)));
}

JNIEXPORT void JNICALL Java_org_main_SkylineHip_partInsert(JNIEnv *env, jclass cls, jlong part, jlongArray ids,
                                                            jdoubleArray values, jint n) {
    const int D = part_dims(PART(part));
    if (n < 0 || D < 1) { throw_arg(env, "partInsert: bad n or part"); return; }
    if (n == 0) return;
    if (bad_len(env, ids, n, "partInsert: ids shorter than n") ||
        bad_len(env, values, (jlong)n * D, "partInsert: values shorter than n * dims"))
        return;
    jlong *pi = CRIT(ids);
    jdouble *pv = CRIT(values);
    const int rc = pi && pv ? sky_part_insert(PART(part), (const int64_t *)pi, pv, n) : SKY_E_NOMEM;   /* copies */
    UNCRIT(values, pv, JNI_ABORT);
    UNCRIT(ids, pi, JNI_ABORT);
    if (pi && pv) fail(env, rc);
}

/* the full buffers of several keys in one call (sky_parts_insert): parts[g] gets
 * ids[g][0..counts[g]) / values[g][0..counts[g] * dims) */
JNIEXPORT void JNICALL Java_org_main_SkylineHip_partsInsert(JNIEnv *env, jclass cls, jlongArray parts,
                                                             jobjectArray ids, jobjectArray values, jintArray counts) {
    if (!parts || !ids || !values || !counts) { throw_arg(env, "partsInsert: null argument"); return; }
    const jsize np = (*env)->GetArrayLength(env, parts);
    if ((*env)->GetArrayLength(env, ids) != np || (*env)->GetArrayLength(env, values) != np ||
        (*env)->GetArrayLength(env, counts) != np) {
        throw_arg(env, "partsInsert: arrays of different lengths");
        return;
    }
    if (np == 0) return;
    sky_part **pp = calloc((size_t)np, sizeof(sky_part *));
    const int64_t **pids = calloc((size_t)np, sizeof(int64_t *));
    const double **pvals = calloc((size_t)np, sizeof(double *));
    int64_t *cnt = calloc((size_t)np, sizeof(int64_t));
    jlongArray *ja = calloc((size_t)np, sizeof(jlongArray));
    jdoubleArray *jv = calloc((size_t)np, sizeof(jdoubleArray));
    jsize got = 0;
    if (!pp || !pids || !pvals || !cnt || !ja || !jv) {
        (*env)->ThrowNew(env, (*env)->FindClass(env, "java/lang/OutOfMemoryError"), "partsInsert");
        goto out;
    }
    {
        jlong *ph = (*env)->GetLongArrayElements(env, parts, NULL);
        jint *pc = (*env)->GetIntArrayElements(env, counts, NULL);
        if (ph && pc)
            for (jsize g = 0; g < np; g++) { pp[g] = PART(ph[g]); cnt[g] = pc[g]; }
        /* each released on its own: one of them may have failed (OutOfMemoryError pending) */
        if (pc) (*env)->ReleaseIntArrayElements(env, counts, pc, JNI_ABORT);
        if (ph) (*env)->ReleaseLongArrayElements(env, parts, ph, JNI_ABORT);
        if (!ph || !pc) goto out;
    }
    for (jsize g = 0; g < np; g++) {   /* Get*ArrayElements: several arrays stay pinned/copied at once */
        const int D = part_dims(pp[g]);
        ja[g] = (jlongArray)(*env)->GetObjectArrayElement(env, ids, g);
        jv[g] = (jdoubleArray)(*env)->GetObjectArrayElement(env, values, g);
        if (D < 1 || cnt[g] < 0 || bad_len(env, ja[g], cnt[g], "partsInsert: ids[g] shorter than counts[g]") ||
            bad_len(env, jv[g], cnt[g] * D, "partsInsert: values[g] shorter than counts[g] * dims")) {
            if (!(*env)->ExceptionCheck(env)) throw_arg(env, "partsInsert: bad part or count");
            goto release;
        }
        pids[g] = (const int64_t *)(*env)->GetLongArrayElements(env, ja[g], NULL);
        pvals[g] = (*env)->GetDoubleArrayElements(env, jv[g], NULL);
        got = g + 1;
        if (!pids[g] || !pvals[g]) goto release;
    }
    fail(env, sky_parts_insert(np, pp, pids, pvals, cnt));   /* copies before it returns */
release:
    for (jsize g = 0; g < np; g++) {
        if (g < got) {
            if (pvals[g]) (*env)->ReleaseDoubleArrayElements(env, jv[g], (jdouble *)pvals[g], JNI_ABORT);
            if (pids[g]) (*env)->ReleaseLongArrayElements(env, ja[g], (jlong *)pids[g], JNI_ABORT);
        }
        if (jv[g]) (*env)->DeleteLocalRef(env, jv[g]);
        if (ja[g]) (*env)->DeleteLocalRef(env, ja[g]);
    }
out:
    free(pp);
    free(pids);
    free(pvals);
    free(cnt);
    free(ja);
    free(jv);
}

JNIEXPORT jlong JNICALL Java_org_main_SkylineHip_partSize(JNIEnv *env, jclass cls, jlong part) {
    int64_t n = 0;
    if (fail(env, sky_part_size(PART(part), &n))) return -1;
    return (jlong)n;
}

/* processQuery's snapshot (:387-392): returns n, or -required if the arrays are too small */
JNIEXPORT jint JNICALL Java_org_main_SkylineHip_partSnapshot(JNIEnv *env, jclass cls, jlong part,
                                                              jlongArray ids_out, jdoubleArray values_out) {
    const int D = part_dims(PART(part));
    if (D < 1 || !ids_out || !values_out) { throw_arg(env, "partSnapshot: bad part or null array"); return 0; }
    jsize cap = (*env)->GetArrayLength(env, ids_out);
    const jsize vcap = (*env)->GetArrayLength(env, values_out) / D;
    if (vcap < cap) cap = vcap;            /* both arrays must hold the snapshot */
    jlong *pi = CRIT(ids_out);
    jdouble *pv = CRIT(values_out);
    int64_t n = 0;
    const int rc = pi && pv ? sky_part_snapshot(PART(part), (int64_t *)pi, pv, cap, &n) : SKY_E_NOMEM;
    UNCRIT(values_out, pv, 0);
    UNCRIT(ids_out, pi, 0);
    if (!pi || !pv) return 0;
    if (rc == SKY_E_CAPACITY) return (jint)-n;
    if (fail(env, rc)) return 0;
    return (jint)n;
}

/* exact tuple and distinct-vector counts: sizes_out[0] = T, sizes_out[1] = R */
JNIEXPORT void JNICALL Java_org_main_SkylineHip_partSizes(JNIEnv *env, jclass cls, jlong part, jlongArray sizes_out) {
    if (bad_len(env, sizes_out, 2, "partSizes: sizesOut shorter than 2")) return;
    int64_t t = 0, r = 0;
    if (fail(env, sky_part_sizes(PART(part), &t, &r))) return;
    const jlong v[2] = {(jlong)t, (jlong)r};
    (*env)->SetLongArrayRegion(env, sizes_out, 0, 2, v);
}

/* processQuery's message as distinct vectors: ids[T], repIdx[T], reps[R * dims], repCounts[R];
 * returns T, or -T when an array is too small (partSizes gives T and R) */
JNIEXPORT jint JNICALL Java_org_main_SkylineHip_partSnapshotReps(JNIEnv *env, jclass cls, jlong part,
                                                                  jlongArray ids_out, jintArray rep_out,
                                                                  jdoubleArray reps_out, jintArray rep_count_out) {
    const int D = part_dims(PART(part));
    if (D < 1 || !ids_out || !rep_out || !reps_out || !rep_count_out) {
        throw_arg(env, "partSnapshotReps: bad part or null array");
        return 0;
    }
    jsize cap = (*env)->GetArrayLength(env, ids_out);
    if ((*env)->GetArrayLength(env, rep_out) < cap) cap = (*env)->GetArrayLength(env, rep_out);
    jsize rcap = (*env)->GetArrayLength(env, rep_count_out);
    if ((*env)->GetArrayLength(env, reps_out) / D < rcap) rcap = (*env)->GetArrayLength(env, reps_out) / D;
    jlong *pi = CRIT(ids_out);
    jint *pr = CRIT(rep_out);
    jdouble *pv = CRIT(reps_out);
    jint *pc = CRIT(rep_count_out);
    int64_t n = 0, r = 0;
    const int ok = pi && pr && pv && pc;
    const int rc = ok ? sky_part_snapshot_reps(PART(part), (int64_t *)pi, (int32_t *)pr, cap, pv, (int32_t *)pc, rcap,
                                               &n, &r)
                      : SKY_E_NOMEM;
    UNCRIT(rep_count_out, pc, 0);
    UNCRIT(reps_out, pv, 0);
    UNCRIT(rep_out, pr, 0);
    UNCRIT(ids_out, pi, 0);
    if (!ok) return 0;
    if (rc == SKY_E_CAPACITY) return (jint)-n;
    if (fail(env, rc)) return 0;
    return (jint)n;
}

/* ---- global merge: GlobalSkylineAggregator.processElement (:515-569), on the last arrival ---- */
/* over the distinct-vector messages (partSnapshotReps output of each local processor):
 * returns the skyline size, or -(needed) when idsOut is too short */
JNIEXPORT jint JNICALL Java_org_main_SkylineHip_globalMergeReps(JNIEnv *env, jclass cls, jlong ctx, jintArray part_ids,
                                                                 jobjectArray ids, jobjectArray rep_idx,
                                                                 jobjectArray reps, jobjectArray rep_counts,
                                                                 jlongArray ids_out, jintArray origin_out) {
    (void)cls;
    const int D = ctx_dims(CTX(ctx));
    if (D < 1 || !part_ids || !ids || !rep_idx || !reps || !rep_counts || !ids_out || !origin_out) {
        throw_arg(env, "globalMergeReps: bad context or null array");
        return 0;
    }
    const jsize np = (*env)->GetArrayLength(env, part_ids);
    if ((*env)->GetArrayLength(env, ids) != np || (*env)->GetArrayLength(env, rep_idx) != np ||
        (*env)->GetArrayLength(env, reps) != np || (*env)->GetArrayLength(env, rep_counts) != np) {
        throw_arg(env, "globalMergeReps: arrays of different lengths");
        return 0;
    }
    const size_t m = np ? (size_t)np : 1;
    const int64_t **pid = calloc(m, sizeof(int64_t *));
    const int32_t **prx = calloc(m, sizeof(int32_t *));
    const double **prp = calloc(m, sizeof(double *));
    const int32_t **prc = calloc(m, sizeof(int32_t *));
    int64_t *cnt = calloc(m, sizeof(int64_t)), *nrep = calloc(m, sizeof(int64_t));
    jarray *jo = calloc(4 * m, sizeof(jarray));          /* [4k + 0..3]: ids, repIdx, reps, repCounts of list k */
    jint g = 0;
    jsize got = 0;
    if (!pid || !prx || !prp || !prc || !cnt || !nrep || !jo) {
        (*env)->ThrowNew(env, (*env)->FindClass(env, "java/lang/OutOfMemoryError"), "globalMergeReps");
        goto out;
    }
    for (jsize k = 0; k < np; k++) {    /* Get*ArrayElements: several arrays stay pinned/copied at once */
        jo[4 * k] = (*env)->GetObjectArrayElement(env, ids, k);
        jo[4 * k + 1] = (*env)->GetObjectArrayElement(env, rep_idx, k);
        jo[4 * k + 2] = (*env)->GetObjectArrayElement(env, reps, k);
        jo[4 * k + 3] = (*env)->GetObjectArrayElement(env, rep_counts, k);
        if (!jo[4 * k] || !jo[4 * k + 3]) { throw_arg(env, "globalMergeReps: null list"); goto release; }
        cnt[k] = (*env)->GetArrayLength(env, jo[4 * k]);
        nrep[k] = (*env)->GetArrayLength(env, jo[4 * k + 3]);
        if (bad_len(env, jo[4 * k + 1], cnt[k], "globalMergeReps: repIdx[k] shorter than ids[k]") ||
            bad_len(env, jo[4 * k + 2], nrep[k] * D, "globalMergeReps: reps[k] shorter than repCounts[k] * dims"))
            goto release;
        pid[k] = (const int64_t *)(*env)->GetLongArrayElements(env, (jlongArray)jo[4 * k], NULL);
        prx[k] = (const int32_t *)(*env)->GetIntArrayElements(env, (jintArray)jo[4 * k + 1], NULL);
        prp[k] = (*env)->GetDoubleArrayElements(env, (jdoubleArray)jo[4 * k + 2], NULL);
        prc[k] = (const int32_t *)(*env)->GetIntArrayElements(env, (jintArray)jo[4 * k + 3], NULL);
        got = k + 1;
        if (!pid[k] || !prx[k] || !prp[k] || !prc[k]) goto release;
    }
    {
        const jsize cap = (*env)->GetArrayLength(env, ids_out);
        if ((*env)->GetArrayLength(env, origin_out) < cap) {
            throw_arg(env, "globalMergeReps: originOut shorter than idsOut");
            goto release;
        }
        jint *pk = (*env)->GetIntArrayElements(env, part_ids, NULL);
        jlong *oi = (*env)->GetLongArrayElements(env, ids_out, NULL);
        jint *oo = (*env)->GetIntArrayElements(env, origin_out, NULL);
        if (pk && oi && oo) {
            int64_t n = 0;
            const int rc = sky_global_merge_reps(CTX(ctx), np, (const int32_t *)pk, pid, prx, cnt, prp, prc, nrep,
                                                 (int64_t *)oi, (int32_t *)oo, cap, &n);
            if (rc == SKY_E_CAPACITY) g = (jint)-n;
            else if (!fail(env, rc)) g = (jint)n;
        }
        if (oo) (*env)->ReleaseIntArrayElements(env, origin_out, oo, 0);
        if (oi) (*env)->ReleaseLongArrayElements(env, ids_out, oi, 0);
        if (pk) (*env)->ReleaseIntArrayElements(env, part_ids, pk, JNI_ABORT);
    }
release:
    for (jsize k = 0; k < np; k++) {
        if (k < got) {
            if (prc[k]) (*env)->ReleaseIntArrayElements(env, (jintArray)jo[4 * k + 3], (jint *)prc[k], JNI_ABORT);
            if (prp[k]) (*env)->ReleaseDoubleArrayElements(env, (jdoubleArray)jo[4 * k + 2], (jdouble *)prp[k], JNI_ABORT);
            if (prx[k]) (*env)->ReleaseIntArrayElements(env, (jintArray)jo[4 * k + 1], (jint *)prx[k], JNI_ABORT);
            if (pid[k]) (*env)->ReleaseLongArrayElements(env, (jlongArray)jo[4 * k], (jlong *)pid[k], JNI_ABORT);
        }
        for (int q = 0; q < 4; q++)
            if (jo[4 * k + q]) (*env)->DeleteLocalRef(env, jo[4 * k + q]);
    }
out:
    free(pid);
    free(prx);
    free(prp);
    free(prc);
    free(cnt);
    free(nrep);
    free(jo);
    return g;
}

/* the co-located aggregator's merge over the parts' device-resident states (no snapshot through
 * the JVM heap); returns the skyline size, or -(needed) when idsOut is too short */
JNIEXPORT jint JNICALL Java_org_main_SkylineHip_partsGlobalMerge(JNIEnv *env, jclass cls, jlong ctx, jlongArray parts,
                                                                  jintArray part_ids, jlongArray ids_out,
                                                                  jintArray origin_out) {
    (void)cls;
    if (!parts || !part_ids || !ids_out || !origin_out) {
        throw_arg(env, "partsGlobalMerge: null array");
        return 0;
    }
    const jsize np = (*env)->GetArrayLength(env, parts);
    if (bad_len(env, part_ids, np, "partsGlobalMerge: partIds shorter than parts")) return 0;
    const jsize cap = (*env)->GetArrayLength(env, ids_out);
    if (bad_len(env, origin_out, cap, "partsGlobalMerge: originOut shorter than idsOut")) return 0;
    jlong *ph = (*env)->GetLongArrayElements(env, parts, NULL);
    jint *pk = (*env)->GetIntArrayElements(env, part_ids, NULL);
    jlong *oi = (*env)->GetLongArrayElements(env, ids_out, NULL);
    jint *oo = (*env)->GetIntArrayElements(env, origin_out, NULL);
    jint g = 0;
    if (ph && pk && oi && oo) {
        sky_part **pp = calloc(np ? np : 1, sizeof(sky_part *));
        if (!pp) {
            (*env)->ThrowNew(env, (*env)->FindClass(env, "java/lang/OutOfMemoryError"), "partsGlobalMerge");
        } else {
            for (jsize k = 0; k < np; k++) pp[k] = PART(ph[k]);
            int64_t n = 0;
            const int rc = sky_parts_global_merge(CTX(ctx), np, pp, (const int32_t *)pk, (int64_t *)oi,
                                                  (int32_t *)oo, cap, &n);
            if (rc == SKY_E_CAPACITY) g = (jint)-n;
            else if (!fail(env, rc)) g = (jint)n;
            free(pp);
        }
    }
    if (oo) (*env)->ReleaseIntArrayElements(env, origin_out, oo, 0);
    if (oi) (*env)->ReleaseLongArrayElements(env, ids_out, oi, 0);
    if (pk) (*env)->ReleaseIntArrayElements(env, part_ids, pk, JNI_ABORT);
    if (ph) (*env)->ReleaseLongArrayElements(env, parts, ph, JNI_ABORT);
    return g;
}

JNIEXPORT jint JNICALL Java_org_main_SkylineHip_globalMerge(JNIEnv *env, jclass cls, jlong ctx, jintArray part_ids,
                                                             jobjectArray ids, jobjectArray values,
                                                             jlongArray ids_out, jintArray origin_out) {
    const jsize np = (*env)->GetArrayLength(env, part_ids);
    const int64_t **pids = calloc(np ? np : 1, sizeof(int64_t *));
    const double **pvals = calloc(np ? np : 1, sizeof(double *));
    int64_t *counts = calloc(np ? np : 1, sizeof(int64_t));
    jlongArray *ja = calloc(np ? np : 1, sizeof(jlongArray));
    jdoubleArray *jv = calloc(np ? np : 1, sizeof(jdoubleArray));
    jint g = 0;
    if (!pids || !pvals || !counts || !ja || !jv) {
        (*env)->ThrowNew(env, (*env)->FindClass(env, "java/lang/OutOfMemoryError"), "globalMerge");
        goto out;
    }
    const int D = ctx_dims(CTX(ctx));
    jsize got = 0;
    if (D < 1 || !ids || !values || !ids_out || !origin_out || (*env)->GetArrayLength(env, ids) != np ||
        (*env)->GetArrayLength(env, values) != np) {
        throw_arg(env, "globalMerge: bad context or arrays");
        goto out;
    }
    for (jsize k = 0; k < np; k++) {   /* Get*ArrayElements: several arrays stay pinned/copied at once */
        ja[k] = (jlongArray)(*env)->GetObjectArrayElement(env, ids, k);
        jv[k] = (jdoubleArray)(*env)->GetObjectArrayElement(env, values, k);
        if (!ja[k] || bad_len(env, jv[k], (jlong)(*env)->GetArrayLength(env, ja[k]) * D,
                               "globalMerge: values[k] shorter than ids[k].length * dims"))
            goto release;
        counts[k] = (*env)->GetArrayLength(env, ja[k]);
        pids[k] = (const int64_t *)(*env)->GetLongArrayElements(env, ja[k], NULL);
        pvals[k] = (*env)->GetDoubleArrayElements(env, jv[k], NULL);
        got = k + 1;
        if (!pids[k] || !pvals[k]) goto release;
    }
    {
        const jsize cap = (*env)->GetArrayLength(env, ids_out);
        if ((*env)->GetArrayLength(env, origin_out) < cap) { throw_arg(env, "globalMerge: originOut shorter than idsOut"); goto release; }
        jint *pk = (*env)->GetIntArrayElements(env, part_ids, NULL);
        jlong *oi = (*env)->GetLongArrayElements(env, ids_out, NULL);
        jint *oo = (*env)->GetIntArrayElements(env, origin_out, NULL);
        if (pk && oi && oo) {
            int64_t n = 0;
            const int rc = sky_global_merge(CTX(ctx), np, (const int32_t *)pk, pids, pvals, counts, (int64_t *)oi,
                                            (int32_t *)oo, cap, &n);
            if (rc == SKY_E_CAPACITY) g = (jint)-n;
            else if (!fail(env, rc)) g = (jint)n;
        }
        if (oo) (*env)->ReleaseIntArrayElements(env, origin_out, oo, 0);
        if (oi) (*env)->ReleaseLongArrayElements(env, ids_out, oi, 0);
        if (pk) (*env)->ReleaseIntArrayElements(env, part_ids, pk, JNI_ABORT);
    }
release:
    for (jsize k = 0; k < np; k++) {
        if (k < got) {
            if (pvals[k]) (*env)->ReleaseDoubleArrayElements(env, jv[k], (jdouble *)pvals[k], JNI_ABORT);
            if (pids[k]) (*env)->ReleaseLongArrayElements(env, ja[k], (jlong *)pids[k], JNI_ABORT);
        }
        if (jv[k]) (*env)->DeleteLocalRef(env, jv[k]);
        if (ja[k]) (*env)->DeleteLocalRef(env, ja[k]);
    }
out:
    free(pids);
    free(pvals);
    free(counts);
    free(ja);
    free(jv);
    return g;
}

/* the optimality integers (:593-608): returns K, fills |L_k| and survivors_k for k < K; with both
 * arrays null it only returns K; arrays shorter than K: -K, nothing written */
JNIEXPORT jint JNICALL Java_org_main_SkylineHip_globalStats(JNIEnv *env, jclass cls, jlong ctx,
                                                             jlongArray local_sizes, jlongArray survivors) {
    int32_t K = 0;
    if (fail(env, sky_global_stats(CTX(ctx), NULL, NULL, &K))) return 0;
    if (!local_sizes && !survivors) return K;
    if (!local_sizes || !survivors) { throw_arg(env, "globalStats: one array null"); return 0; }
    if ((*env)->GetArrayLength(env, local_sizes) < K || (*env)->GetArrayLength(env, survivors) < K) return -K;
    jlong *ls = (*env)->GetLongArrayElements(env, local_sizes, NULL);
    jlong *sv = (*env)->GetLongArrayElements(env, survivors, NULL);
    const int rc = ls && sv ? sky_global_stats(CTX(ctx), (int64_t *)ls, (int64_t *)sv, &K) : SKY_E_NOMEM;
    if (sv) (*env)->ReleaseLongArrayElements(env, survivors, sv, 0);
    if (ls) (*env)->ReleaseLongArrayElements(env, local_sizes, ls, 0);
    if (ls && sv) fail(env, rc);
    return K;
}

/* ---- whole-stream query (batch / replay jobs): keyBy -> local -> global (:138-174) ---- */
JNIEXPORT jint JNICALL Java_org_main_SkylineHip_query(JNIEnv *env, jclass cls, jlong ctx, jlongArray ids,
                                                       jdoubleArray values, jint n, jlongArray ids_out,
                                                       jintArray origin_out) {
    const int D = ctx_dims(CTX(ctx));
    if (n < 0 || D < 1 || bad_len(env, ids, n, "query: ids shorter than n") ||
        bad_len(env, values, (jlong)n * D, "query: values shorter than n * dims") ||
        bad_len(env, ids_out, 0, "query: null idsOut") || bad_len(env, origin_out, 0, "query: null originOut")) {
        if (!(*env)->ExceptionCheck(env)) throw_arg(env, "query: bad n or context");
        return 0;
    }
    jsize cap = (*env)->GetArrayLength(env, ids_out);
    if ((*env)->GetArrayLength(env, origin_out) < cap) cap = (*env)->GetArrayLength(env, origin_out);
    jlong *pi = CRIT(ids);
    jdouble *pv = CRIT(values);
    jlong *oi = CRIT(ids_out);
    jint *oo = CRIT(origin_out);
    int64_t g = 0;
    const int ok = pi && pv && oi && oo;
    const int rc = ok ? sky_query(CTX(ctx), (const int64_t *)pi, pv, n, (int64_t *)oi, (int32_t *)oo, cap, &g)
                      : SKY_E_NOMEM;
    UNCRIT(origin_out, oo, 0);
    UNCRIT(ids_out, oi, 0);
    UNCRIT(values, pv, JNI_ABORT);
    UNCRIT(ids, pi, JNI_ABORT);
    if (!ok) return 0;
    if (rc == SKY_E_CAPACITY) return (jint)-g;
    if (fail(env, rc)) return 0;
    return (jint)g;
}

/* ---- bulk ingest: .map(ServiceTuple::fromString).filter(nonNull) + Long.parseLong (:102-104, :276).
 * text: raw Kafka values joined with '\n'.  counts_out[4] = records, malformed, bad id, arity.
 * Returns the accepted records (ids_out / values_out), or -required. */
JNIEXPORT jint JNICALL Java_org_main_SkylineHip_parseCsv(JNIEnv *env, jclass cls, jlong ctx, jbyteArray text,
                                                          jint nbytes, jlongArray ids_out, jdoubleArray values_out,
                                                          jlongArray counts_out) {
    const int D = ctx_dims(CTX(ctx));
    if (nbytes < 0 || D < 1 || bad_len(env, text, nbytes, "parseCsv: text shorter than nbytes") ||
        bad_len(env, counts_out, 4, "parseCsv: countsOut shorter than 4") ||
        bad_len(env, ids_out, 0, "parseCsv: null idsOut") || bad_len(env, values_out, 0, "parseCsv: null valuesOut")) {
        if (!(*env)->ExceptionCheck(env)) throw_arg(env, "parseCsv: bad nbytes or context");
        return 0;
    }
    jsize cap = (*env)->GetArrayLength(env, ids_out);
    if ((*env)->GetArrayLength(env, values_out) / D < cap) cap = (*env)->GetArrayLength(env, values_out) / D;
    jbyte *t = CRIT(text);
    jlong *oi = CRIT(ids_out);
    jdouble *ov = CRIT(values_out);
    jlong *oc = CRIT(counts_out);
    int64_t n = 0;
    const int ok = t && oi && ov && oc;
    const int rc = ok ? sky_parse_csv(CTX(ctx), (const char *)t, nbytes, (int64_t *)oi, ov, cap, &n, (int64_t *)oc)
                      : SKY_E_NOMEM;
    UNCRIT(counts_out, oc, 0);
    UNCRIT(values_out, ov, 0);
    UNCRIT(ids_out, oi, 0);
    UNCRIT(text, t, JNI_ABORT);
    if (!ok) return 0;
    if (rc == SKY_E_CAPACITY) return (jint)-n;
    if (fail(env, rc)) return 0;
    return (jint)n;
}

/* ---- continuous queries (landmark window = the reference; window > 0 = sliding extension) ---- */
JNIEXPORT jlong JNICALL Java_org_main_SkylineHip_streamCreate(JNIEnv *env, jclass cls, jlong ctx, jlong window) {
    sky_stream *s = NULL;
    if (fail(env, sky_stream_create(CTX(ctx), window, &s))) return 0;
    return (jlong)(uintptr_t)s;
}

JNIEXPORT void JNICALL Java_org_main_SkylineHip_streamDestroy(JNIEnv *env, jclass cls, jlong s) {
    fail(env, sky_stream_destroy(STREAM(s)));
}

JNIEXPORT void JNICALL Java_org_main_SkylineHip_streamAppend(JNIEnv *env, jclass cls, jlong s, jlongArray ids,
                                                              jdoubleArray values, jint n) {
    int32_t D = 0;
    if (n < 0 || sky_stream_info(STREAM(s), &D) != SKY_OK || D < 1) { throw_arg(env, "streamAppend: bad n or stream"); return; }
    if (n == 0) return;
    if (bad_len(env, ids, n, "streamAppend: ids shorter than n") ||
        bad_len(env, values, (jlong)n * D, "streamAppend: values shorter than n * dims"))
        return;
    jlong *pi = CRIT(ids);
    jdouble *pv = CRIT(values);
    const int rc = pi && pv ? sky_stream_append(STREAM(s), (const int64_t *)pi, pv, n) : SKY_E_NOMEM;
    UNCRIT(values, pv, JNI_ABORT);
    UNCRIT(ids, pi, JNI_ABORT);
    if (pi && pv) fail(env, rc);
}

JNIEXPORT jint JNICALL Java_org_main_SkylineHip_streamQuery(JNIEnv *env, jclass cls, jlong s, jlongArray ids_out,
                                                             jintArray origin_out) {
    if (!ids_out || !origin_out) { throw_arg(env, "streamQuery: null array"); return 0; }
    jsize cap = (*env)->GetArrayLength(env, ids_out);
    if ((*env)->GetArrayLength(env, origin_out) < cap) cap = (*env)->GetArrayLength(env, origin_out);
    jlong *oi = CRIT(ids_out);
    jint *oo = CRIT(origin_out);
    int64_t g = 0;
    const int rc = oi && oo ? sky_stream_query(STREAM(s), (int64_t *)oi, (int32_t *)oo, cap, &g) : SKY_E_NOMEM;
    UNCRIT(origin_out, oo, 0);
    UNCRIT(ids_out, oi, 0);
    if (!oi || !oo) return 0;
    if (rc == SKY_E_CAPACITY) return (jint)-g;
    if (fail(env, rc)) return 0;
    return (jint)g;
}

JNIEXPORT void JNICALL Java_org_main_SkylineHip_streamReserve(JNIEnv *env, jclass cls, jlong s, jlong tuples) {
    (void)cls;
    if (tuples < 0) {
        throw_arg(env, "tuples must be >= 0");
        return;
    }
    (void)fail(env, sky_stream_reserve(STREAM(s), (int64_t)tuples));
}

JNIEXPORT jlong JNICALL Java_org_main_SkylineHip_streamResident(JNIEnv *env, jclass cls, jlong s) {
    int64_t r = 0, a = 0;
    if (fail(env, sky_stream_size(STREAM(s), &r, &a))) return -1;
    return (jlong)r;
}
