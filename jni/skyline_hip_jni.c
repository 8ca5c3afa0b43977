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
 * layout of ServiceTuple.values concatenated).  The library copies host buffers before it
 * returns, so arrays are pinned only for the duration of one call (GetPrimitiveArrayCritical,
 * no JNI calls in between).  Handles are jlong (uintptr_t) values of the C pointers.
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

#define CTX(h) ((sky_ctx *)(uintptr_t)(h))
#define PART(h) ((sky_part *)(uintptr_t)(h))
#define STREAM(h) ((sky_stream *)(uintptr_t)(h))

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
    jdouble *v = (*env)->GetPrimitiveArrayCritical(env, values, NULL);
    jint *k = (*env)->GetPrimitiveArrayCritical(env, keys_out, NULL);
    const int rc = sky_partition_keys(CTX(ctx), v, n, (int32_t *)k);
    (*env)->ReleasePrimitiveArrayCritical(env, keys_out, k, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, values, v, JNI_ABORT);
    fail(env, rc);
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
    jlong *pi = (*env)->GetPrimitiveArrayCritical(env, ids, NULL);
    jdouble *pv = (*env)->GetPrimitiveArrayCritical(env, values, NULL);
    const int rc = sky_part_insert(PART(part), (const int64_t *)pi, pv, n);   /* copies before return */
    (*env)->ReleasePrimitiveArrayCritical(env, values, pv, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, ids, pi, JNI_ABORT);
    fail(env, rc);
}

JNIEXPORT jlong JNICALL Java_org_main_SkylineHip_partSize(JNIEnv *env, jclass cls, jlong part) {
    int64_t n = 0;
    if (fail(env, sky_part_size(PART(part), &n))) return -1;
    return (jlong)n;
}

/* processQuery's snapshot (:387-392): returns n, or -required if the arrays are too small */
JNIEXPORT jint JNICALL Java_org_main_SkylineHip_partSnapshot(JNIEnv *env, jclass cls, jlong part,
                                                              jlongArray ids_out, jdoubleArray values_out) {
    const jsize cap = (*env)->GetArrayLength(env, ids_out);
    jlong *pi = (*env)->GetPrimitiveArrayCritical(env, ids_out, NULL);
    jdouble *pv = (*env)->GetPrimitiveArrayCritical(env, values_out, NULL);
    int64_t n = 0;
    const int rc = sky_part_snapshot(PART(part), (int64_t *)pi, pv, cap, &n);
    (*env)->ReleasePrimitiveArrayCritical(env, values_out, pv, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, ids_out, pi, 0);
    if (rc == SKY_E_CAPACITY) return (jint)-n;
    if (fail(env, rc)) return 0;
    return (jint)n;
}

/* ---- global merge: GlobalSkylineAggregator.processElement (:515-569), on the last arrival ---- */
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
    for (jsize k = 0; k < np; k++) {   /* Get*ArrayElements: several arrays stay pinned/copied at once */
        ja[k] = (jlongArray)(*env)->GetObjectArrayElement(env, ids, k);
        jv[k] = (jdoubleArray)(*env)->GetObjectArrayElement(env, values, k);
        counts[k] = (*env)->GetArrayLength(env, ja[k]);
        pids[k] = (const int64_t *)(*env)->GetLongArrayElements(env, ja[k], NULL);
        pvals[k] = (*env)->GetDoubleArrayElements(env, jv[k], NULL);
    }
    {
        jint *pk = (*env)->GetIntArrayElements(env, part_ids, NULL);
        jlong *oi = (*env)->GetLongArrayElements(env, ids_out, NULL);
        jint *oo = (*env)->GetIntArrayElements(env, origin_out, NULL);
        const jsize cap = (*env)->GetArrayLength(env, ids_out);
        int64_t n = 0;
        const int rc = sky_global_merge(CTX(ctx), np, (const int32_t *)pk, pids, pvals, counts, (int64_t *)oi,
                                        (int32_t *)oo, cap, &n);
        (*env)->ReleaseIntArrayElements(env, origin_out, oo, 0);
        (*env)->ReleaseLongArrayElements(env, ids_out, oi, 0);
        (*env)->ReleaseIntArrayElements(env, part_ids, pk, JNI_ABORT);
        if (rc == SKY_E_CAPACITY) g = (jint)-n;
        else if (!fail(env, rc)) g = (jint)n;
    }
    for (jsize k = 0; k < np; k++) {
        (*env)->ReleaseDoubleArrayElements(env, jv[k], (jdouble *)pvals[k], JNI_ABORT);
        (*env)->ReleaseLongArrayElements(env, ja[k], (jlong *)pids[k], JNI_ABORT);
        (*env)->DeleteLocalRef(env, jv[k]);
        (*env)->DeleteLocalRef(env, ja[k]);
    }
out:
    free(pids);
    free(pvals);
    free(counts);
    free(ja);
    free(jv);
    return g;
}

/* the optimality integers (:593-608): returns K, fills |L_k| and survivors_k for k < K */
JNIEXPORT jint JNICALL Java_org_main_SkylineHip_globalStats(JNIEnv *env, jclass cls, jlong ctx,
                                                             jlongArray local_sizes, jlongArray survivors) {
    int32_t K = 0;
    if (fail(env, sky_global_stats(CTX(ctx), NULL, NULL, &K))) return 0;
    if ((*env)->GetArrayLength(env, local_sizes) < K || (*env)->GetArrayLength(env, survivors) < K) return -K;
    jlong *ls = (*env)->GetLongArrayElements(env, local_sizes, NULL);
    jlong *sv = (*env)->GetLongArrayElements(env, survivors, NULL);
    const int rc = sky_global_stats(CTX(ctx), (int64_t *)ls, (int64_t *)sv, &K);
    (*env)->ReleaseLongArrayElements(env, survivors, sv, 0);
    (*env)->ReleaseLongArrayElements(env, local_sizes, ls, 0);
    fail(env, rc);
    return K;
}

/* ---- whole-stream query (batch / replay jobs): keyBy -> local -> global (:138-174) ---- */
JNIEXPORT jint JNICALL Java_org_main_SkylineHip_query(JNIEnv *env, jclass cls, jlong ctx, jlongArray ids,
                                                       jdoubleArray values, jint n, jlongArray ids_out,
                                                       jintArray origin_out) {
    const jsize cap = (*env)->GetArrayLength(env, ids_out);
    jlong *pi = (*env)->GetPrimitiveArrayCritical(env, ids, NULL);
    jdouble *pv = (*env)->GetPrimitiveArrayCritical(env, values, NULL);
    jlong *oi = (*env)->GetPrimitiveArrayCritical(env, ids_out, NULL);
    jint *oo = (*env)->GetPrimitiveArrayCritical(env, origin_out, NULL);
    int64_t g = 0;
    const int rc = sky_query(CTX(ctx), (const int64_t *)pi, pv, n, (int64_t *)oi, (int32_t *)oo, cap, &g);
    (*env)->ReleasePrimitiveArrayCritical(env, origin_out, oo, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, ids_out, oi, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, values, pv, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, ids, pi, JNI_ABORT);
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
    const jsize cap = (*env)->GetArrayLength(env, ids_out);
    jbyte *t = (*env)->GetPrimitiveArrayCritical(env, text, NULL);
    jlong *oi = (*env)->GetPrimitiveArrayCritical(env, ids_out, NULL);
    jdouble *ov = (*env)->GetPrimitiveArrayCritical(env, values_out, NULL);
    jlong *oc = (*env)->GetPrimitiveArrayCritical(env, counts_out, NULL);
    int64_t n = 0;
    const int rc = sky_parse_csv(CTX(ctx), (const char *)t, nbytes, (int64_t *)oi, ov, cap, &n, (int64_t *)oc);
    (*env)->ReleasePrimitiveArrayCritical(env, counts_out, oc, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, values_out, ov, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, ids_out, oi, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, text, t, JNI_ABORT);
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
    jlong *pi = (*env)->GetPrimitiveArrayCritical(env, ids, NULL);
    jdouble *pv = (*env)->GetPrimitiveArrayCritical(env, values, NULL);
    const int rc = sky_stream_append(STREAM(s), (const int64_t *)pi, pv, n);
    (*env)->ReleasePrimitiveArrayCritical(env, values, pv, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, ids, pi, JNI_ABORT);
    fail(env, rc);
}

JNIEXPORT jint JNICALL Java_org_main_SkylineHip_streamQuery(JNIEnv *env, jclass cls, jlong s, jlongArray ids_out,
                                                             jintArray origin_out) {
    const jsize cap = (*env)->GetArrayLength(env, ids_out);
    jlong *oi = (*env)->GetPrimitiveArrayCritical(env, ids_out, NULL);
    jint *oo = (*env)->GetPrimitiveArrayCritical(env, origin_out, NULL);
    int64_t g = 0;
    const int rc = sky_stream_query(STREAM(s), (int64_t *)oi, (int32_t *)oo, cap, &g);
    (*env)->ReleasePrimitiveArrayCritical(env, origin_out, oo, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, ids_out, oi, 0);
    if (rc == SKY_E_CAPACITY) return (jint)-g;
    if (fail(env, rc)) return 0;
    return (jint)g;
}

JNIEXPORT jlong JNICALL Java_org_main_SkylineHip_streamResident(JNIEnv *env, jclass cls, jlong s) {
    int64_t r = 0, a = 0;
    if (fail(env, sky_stream_size(STREAM(s), &r, &a))) return -1;
    return (jlong)r;
}
