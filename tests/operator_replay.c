/*
 * tests/operator_replay.c — a C caller of libskyline_hip.so that replays the reference
 * operators' call sequence, the way the JNI shim (jni/skyline_hip_jni.c) drives the library
 * from the Java operators.  Run by tests/test_gpu_replay.py on the golden streams.
 *
 *   input     the producers' payload "id,v1,...,vD\n" (python/unified_producer.py:174), read
 *             from a file and decoded on the device: sky_parse_csv
 *             (.map(ServiceTuple::fromString).filter(nonNull), FlinkSkyline.java:102-104)
 *   keyBy     sky_partition_keys (getKey, FlinkSkyline.java:138, :707-712/:774-789/:827-875)
 *   device    sky_device_count + sky_device_for_subtask (the subtask's GPU, HipSkylineOperators.open)
 *   local     SkylineLocalProcessor: per key, buffer 5000 tuples then sky_part_insert
 *             (processElement1 + processBuffer, :265-316, :417-444); a trigger "q,N" after the
 *             last tuple: per key 0..P-1 flush + sky_part_sizes + sky_part_snapshot_reps
 *             (processQuery, :367-404: the LocalSkyline message, distinct vectors)
 *   global    GlobalSkylineAggregator: sky_global_merge_reps over the P messages +
 *             sky_global_stats (:515-608), then the JSON payload of :631-648 plus
 *             "query_latency_ms".  proto 1: the round-3 messages instead (sky_part_snapshot of
 *             ids + values, sky_global_merge)
 *
 *   batching  full buffers wait until G of them are pending (default 8, as HipSkylineOperators'
 *             FLUSH_GROUP) and go to the device as drainFull does: rounds in arrival order,
 *             each round the first waiting buffer of every key, one sky_parts_insert per round
 *   checkpoint after C tuples (optional): every key's buffer flushed and its skyline snapshot
 *             taken (snapshotState), every part and the context closed (a failure), a fresh
 *             context opened and each snapshot re-inserted (initializeState + open); the stream
 *             then continues, and the answer must not change
 *
 * usage: operator_replay <csv file> <dims> <parallelism> <algo 0|1|2> [domain] [checkpoint C | -1] [G] [proto]
 *        proto 0: distinct-vector messages; 1: ids + values messages; 2: as 0, plus empty messages of
 *        the keys >= P the trigger does not reach (a merge whose stats K differs from P)
 * stdout: the JSON line, then "ids" and the sorted global skyline ids, then "lsz" / "surv";
 * stderr: "calls" -- the sky_parts_insert calls and their part counts (the call sequence).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "skyline_hip.h"

#define BUFFER_SIZE 5000   /* FlinkSkyline.java:232 */

static void die(const char *what, int rc) {
    fprintf(stderr, "%s failed: status %d: %s\n", what, rc, sky_last_error());
    exit(1);
}
#define CHECK(call)                       \
    do {                                  \
        int rc_ = (call);                 \
        if (rc_ != SKY_OK) die(#call, rc_); \
    } while (0)

static int64_t now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    return (int64_t)ts.tv_sec * 1000 + ts.tv_nsec / 1000000;
}

/* String.format(Locale.US, "%.4f", x): Java rounds HALF_UP on the shortest decimal string
 * that reads back as x (FormattedFloatingDecimal); x in [0, 1] here. */
static void java_format_4f(double x, char *out, size_t cap) {
    char s[64];
    for (int p = 1; p <= 17; p++) {   /* shortest %e string that reads back as x */
        snprintf(s, sizeof s, "%.*e", p - 1, x);
        if (strtod(s, NULL) == x) break;
    }
    char dg[32];
    int nd = 0;
    const char *c = s;
    for (; *c && *c != 'e'; c++)
        if (*c >= '0' && *c <= '9') dg[nd++] = *c;
    const int e = atoi(c + 1);   /* x = d0.d1d2... x 10^e, x >= 0 */
    long long ip = 0;
    int fr[6] = {0};             /* fr[j]: digit of 10^-j */
    for (int pw = e; pw >= 0; pw--) {
        const int i = e - pw;
        ip = ip * 10 + (i < nd ? dg[i] - '0' : 0);
    }
    for (int i = 0; i < nd; i++) {
        const int pw = e - i;
        if (pw < 0 && pw >= -5) fr[-pw] = dg[i] - '0';
    }
    int f4 = fr[1] * 1000 + fr[2] * 100 + fr[3] * 10 + fr[4];
    if (fr[5] >= 5 && ++f4 == 10000) {   /* HALF_UP: the discarded part is >= half a unit */
        f4 = 0;
        ip++;
    }
    snprintf(out, cap, "%lld.%04d", ip, f4);
}

typedef struct {
    int32_t key;
    sky_part *part;
    int64_t *ids;
    double *vals;
    int64_t n;
} keyed_state;

/* the full buffers waiting for drainFull, in arrival order (HipSkylineOperators.LocalProcessor.full) */
typedef struct {
    int key;
    int64_t *ids;
    double *vals;
} full_buf;
static full_buf *g_full;
static int g_nfull, g_capfull;
static long g_calls, g_call_parts;

/* drainFull: while buffers wait, one round = the first waiting buffer of every key in arrival
 * order (a key appears once per round), one sky_parts_insert per round, the rest keep their order */
static void drain_full(keyed_state *ks) {
    while (g_nfull) {
        sky_part *pp[256];
        const int64_t *pi[256];
        const double *pv[256];
        int64_t cnt[256];
        char seen[256] = {0};
        int np = 0, nlater = 0;
        full_buf *later = (full_buf *)malloc((size_t)g_nfull * sizeof(full_buf));
        full_buf *round = (full_buf *)malloc((size_t)g_nfull * sizeof(full_buf));
        for (int i = 0; i < g_nfull; i++) {
            const int k = g_full[i].key;
            if (k < 256 && !seen[k] && np < 256) {
                seen[k] = 1;
                pp[np] = ks[k].part;
                pi[np] = g_full[i].ids;
                pv[np] = g_full[i].vals;
                cnt[np] = BUFFER_SIZE;
                round[np++] = g_full[i];
            } else {
                later[nlater++] = g_full[i];
            }
        }
        CHECK(sky_parts_insert(np, pp, pi, pv, cnt));   /* copied before it returns */
        g_calls++;
        g_call_parts += np;
        for (int g = 0; g < np; g++) {
            free(round[g].ids);
            free(round[g].vals);
        }
        memcpy(g_full, later, (size_t)nlater * sizeof(full_buf));
        g_nfull = nlater;
        free(later);
        free(round);
    }
}

static void push_full(keyed_state *s, int D) {
    if (g_nfull == g_capfull) {
        g_capfull = g_capfull ? 2 * g_capfull : 64;
        g_full = (full_buf *)realloc(g_full, (size_t)g_capfull * sizeof(full_buf));
    }
    full_buf *b = &g_full[g_nfull++];
    b->key = s->key;
    b->ids = (int64_t *)malloc(BUFFER_SIZE * 8);
    b->vals = (double *)malloc((size_t)BUFFER_SIZE * D * 8);
    memcpy(b->ids, s->ids, BUFFER_SIZE * 8);
    memcpy(b->vals, s->vals, (size_t)BUFFER_SIZE * D * 8);
}

int main(int argc, char **argv) {
    if (argc >= 2 && strcmp(argv[1], "--fmt") == 0) {   /* formatter self-check (no device) */
        for (int i = 2; i < argc; i++) {
            char o[64];
            java_format_4f(strtod(argv[i], NULL), o, sizeof o);
            printf("%s\n", o);
        }
        return 0;
    }
    if (argc < 5) {
        fprintf(stderr, "usage: %s <csv> <dims> <parallelism> <algo> [domain]\n", argv[0]);
        return 2;
    }
    const int D = atoi(argv[2]), par = atoi(argv[3]), algo = atoi(argv[4]);
    const double domain = argc > 5 ? atof(argv[5]) : 1000.0;
    const int64_t ckpt_at = argc > 6 ? atoll(argv[6]) : -1;
    const int group = argc > 7 ? atoi(argv[7]) : 8;
    const int proto = argc > 8 ? atoi(argv[8]) : 0;
    const int P = 2 * par;   /* FlinkSkyline.java:76 */
    FILE *f = fopen(argv[1], "rb");
    if (!f) { perror("open"); return 2; }
    fseek(f, 0, SEEK_END);
    const long nbytes = ftell(f);
    fseek(f, 0, SEEK_SET);
    char *text = (char *)malloc((size_t)nbytes + 1);
    if (fread(text, 1, (size_t)nbytes, f) != (size_t)nbytes) { perror("read"); return 2; }
    fclose(f);

    int32_t ndev = 0, dev32 = 0;
    CHECK(sky_device_count(&ndev));
    if (ndev < 1) { fprintf(stderr, "no HIP device\n"); return 4; }
    CHECK(sky_device_for_subtask(0, ndev, &dev32));   /* the one subtask of this replay */
    int dev = dev32;
    sky_ctx *ctx = NULL;
    CHECK(sky_ctx_create(&dev, 1, D, P, algo, domain, &ctx));
    const int64_t rmax = nbytes / 2 + 1;
    int64_t *ids = (int64_t *)malloc((size_t)rmax * 8);
    double *vals = (double *)malloc((size_t)rmax * D * 8);
    int64_t n = 0, counts[4] = {0};
    CHECK(sky_parse_csv(ctx, text, nbytes, ids, vals, rmax, &n, counts));
    if (counts[SKY_CSV_BAD_ID]) { fprintf(stderr, "NumberFormatException\n"); return 3; }
    int32_t *keys = (int32_t *)malloc((size_t)(n > 0 ? n : 1) * 4);
    CHECK(sky_partition_keys(ctx, vals, n, keys));

    /* keyed state: every key that receives a tuple (MR-Grid keys may exceed P) */
    int kmax = P;
    for (int64_t i = 0; i < n; i++)
        if (keys[i] + 1 > kmax) kmax = keys[i] + 1;
    keyed_state *ks = (keyed_state *)calloc((size_t)kmax, sizeof(keyed_state));
    for (int k = 0; k < kmax; k++) {
        ks[k].key = k;
        ks[k].ids = (int64_t *)malloc(BUFFER_SIZE * 8);
        ks[k].vals = (double *)malloc((size_t)BUFFER_SIZE * D * 8);
        CHECK(sky_part_open(ctx, k, &ks[k].part));
    }
    /* processElement1: buffer; a full buffer waits for its group, then processBuffer */
    for (int64_t i = 0; i < n; i++) {
        if (i == ckpt_at) {
            /* snapshotState: the waiting and partial buffers flushed, every key's skyline saved */
            drain_full(ks);
            int64_t *sn = (int64_t *)calloc((size_t)kmax, 8);
            int64_t **sid = (int64_t **)calloc((size_t)kmax, sizeof(int64_t *));
            double **sval = (double **)calloc((size_t)kmax, sizeof(double *));
            for (int k = 0; k < kmax; k++) {
                keyed_state *s = &ks[k];
                if (s->n) CHECK(sky_part_insert(s->part, s->ids, s->vals, s->n));
                s->n = 0;
                int64_t m = 0;
                int rc = sky_part_snapshot(s->part, NULL, NULL, 0, &m);
                if (rc != SKY_OK && rc != SKY_E_CAPACITY) die("sky_part_snapshot (size)", rc);
                sid[k] = (int64_t *)malloc((size_t)(m > 0 ? m : 1) * 8);
                sval[k] = (double *)malloc((size_t)(m > 0 ? m : 1) * D * 8);
                CHECK(sky_part_snapshot(s->part, sid[k], sval[k], m, &m));
                sn[k] = m;
            }
            /* the failure: every handle gone */
            for (int k = 0; k < kmax; k++) CHECK(sky_part_close(ks[k].part));
            CHECK(sky_ctx_destroy(ctx));
            /* restore: a fresh context, each key's skyline re-inserted (SKY(empty u S) = S) */
            CHECK(sky_ctx_create(&dev, 1, D, P, algo, domain, &ctx));
            for (int k = 0; k < kmax; k++) {
                CHECK(sky_part_open(ctx, k, &ks[k].part));
                if (sn[k]) CHECK(sky_part_insert(ks[k].part, sid[k], sval[k], sn[k]));
                free(sid[k]);
                free(sval[k]);
            }
            free(sn);
            free(sid);
            free(sval);
        }
        const int k = keys[i];
        if (k < 0) continue;   /* removed by the (optional) grid dominance filter */
        keyed_state *s = &ks[k];
        s->ids[s->n] = ids[i];
        memcpy(s->vals + s->n * D, vals + i * D, (size_t)D * 8);
        if (++s->n == BUFFER_SIZE) {
            if (group <= 1) {
                CHECK(sky_part_insert(s->part, s->ids, s->vals, s->n));
            } else {
                push_full(s, D);
                if (g_nfull >= group) drain_full(ks);
            }
            s->n = 0;
        }
    }
    /* trigger "1,N" after the last tuple, broadcast to keys 0..P-1 (:145-157) */
    const int64_t dispatch = now_ms();
    /* proto 2: the aggregator also receives empty messages of the keys the trigger does not reach
     * (MR-Grid keys >= P): a merge over nl > P lists, whose sky_global_stats K is not P */
    const int nl = proto == 2 ? kmax : P;
    int32_t *part_ids = (int32_t *)malloc((size_t)nl * 4);
    int64_t **lid = (int64_t **)calloc((size_t)nl, sizeof(int64_t *));
    double **lval = (double **)calloc((size_t)nl, sizeof(double *));
    int32_t **lrep = (int32_t **)calloc((size_t)nl, sizeof(int32_t *));
    int32_t **lrc = (int32_t **)calloc((size_t)nl, sizeof(int32_t *));
    int64_t *lcnt = (int64_t *)calloc((size_t)nl, 8), *lnr = (int64_t *)calloc((size_t)nl, 8);
    int64_t total = 0;
    for (int k = P; k < nl; k++) {   /* the untriggered keys' empty messages */
        part_ids[k] = k;
        lid[k] = (int64_t *)malloc(8);
        lrep[k] = (int32_t *)malloc(4);
        lval[k] = (double *)malloc((size_t)D * 8);
        lrc[k] = (int32_t *)malloc(4);
    }
    for (int k = 0; k < P; k++) {   /* processQuery: flush (drainFull first), then the local skyline message */
        keyed_state *s = &ks[k];
        drain_full(ks);
        if (s->n) {
            CHECK(sky_part_insert(s->part, s->ids, s->vals, s->n));
            s->n = 0;
        }
        int64_t m = 0, r = 0;
        if (proto != 1) {
            CHECK(sky_part_sizes(s->part, &m, &r));
            lid[k] = (int64_t *)malloc((size_t)(m > 0 ? m : 1) * 8);
            lrep[k] = (int32_t *)malloc((size_t)(m > 0 ? m : 1) * 4);
            lval[k] = (double *)malloc((size_t)(r > 0 ? r : 1) * D * 8);
            lrc[k] = (int32_t *)malloc((size_t)(r > 0 ? r : 1) * 4);
            CHECK(sky_part_snapshot_reps(s->part, lid[k], lrep[k], m, lval[k], lrc[k], r, &m, &r));
        } else {
            CHECK(sky_part_size(s->part, &m));
            lid[k] = (int64_t *)malloc((size_t)(m > 0 ? m : 1) * 8);
            lval[k] = (double *)malloc((size_t)(m > 0 ? m : 1) * D * 8);
            lrep[k] = lrc[k] = NULL;
            CHECK(sky_part_snapshot(s->part, lid[k], lval[k], m, &m));
        }
        part_ids[k] = k;
        lcnt[k] = m;
        lnr[k] = r;
        total += m;
    }
    fprintf(stderr, "calls %ld parts %ld\n", g_calls, g_call_parts);
    /* GlobalSkylineAggregator: merge on the last arrival, optimality integers */
    int64_t *gids = (int64_t *)malloc((size_t)(total > 0 ? total : 1) * 8);
    int32_t *gorg = (int32_t *)malloc((size_t)(total > 0 ? total : 1) * 4);
    int64_t g = 0;
    if (proto != 1)
        CHECK(sky_global_merge_reps(ctx, nl, part_ids, (const int64_t *const *)lid, (const int32_t *const *)lrep, lcnt,
                                    (const double *const *)lval, (const int32_t *const *)lrc, lnr, gids, gorg, total,
                                    &g));
    else
        CHECK(sky_global_merge(ctx, P, part_ids, (const int64_t *const *)lid, (const double *const *)lval, lcnt, gids,
                               gorg, total, &g));
    /* the integers' count K from the library (as HipSkylineOperators sizes its arrays), then the
     * integers; indexed by list, like part_ids */
    int32_t K = 0, K2 = 0;
    CHECK(sky_global_stats(ctx, NULL, NULL, &K));
    if (K < 0 || K < P) { fprintf(stderr, "sky_global_stats: K = %d\n", K); return 5; }
    int64_t *lsz = (int64_t *)malloc((size_t)K * 8 + 8), *surv = (int64_t *)malloc((size_t)K * 8 + 8);
    CHECK(sky_global_stats(ctx, lsz, surv, &K2));
    if (K2 != K) { fprintf(stderr, "sky_global_stats: K changed %d -> %d\n", K, K2); return 5; }
    fprintf(stderr, "stats K %d lists %d\n", K, nl);
    const int64_t finish = now_ms();
    double opt = 0.0;
    for (int k = 0; k < (K < nl ? K : nl); k++)
        if (part_ids[k] < P && lsz[k] > 0) opt += (double)surv[k] / (double)lsz[k];
    opt /= P;
    char ostr[64];
    java_format_4f(opt, ostr, sizeof ostr);
    printf("{\"query_id\": \"1\", \"record_count\": %lld, \"skyline_size\": %lld, \"optimality\": %s, "
           "\"ingestion_time_ms\": 0, \"local_processing_time_ms\": 0, \"global_processing_time_ms\": %lld, "
           "\"total_processing_time_ms\": %lld, \"query_latency_ms\": %lld}\n",
           (long long)n, (long long)g, ostr, (long long)(finish - dispatch), (long long)(finish - dispatch),
           (long long)(finish - dispatch));
    /* sorted global ids (insertion sort is enough for golden sizes; qsort otherwise) */
    int cmp_i64(const void *a, const void *b);
    qsort(gids, (size_t)g, 8, cmp_i64);
    printf("ids");
    for (int64_t j = 0; j < g; j++) printf(" %lld", (long long)gids[j]);
    printf("\nlsz");
    for (int k = 0; k < P; k++) printf(" %lld", (long long)lsz[k]);
    printf("\nsurv");
    for (int k = 0; k < P; k++) printf(" %lld", (long long)surv[k]);
    printf("\n");
    for (int k = 0; k < kmax; k++) {
        CHECK(sky_part_close(ks[k].part));
        free(ks[k].ids);
        free(ks[k].vals);
    }
    for (int k = 0; k < nl; k++) { free(lid[k]); free(lval[k]); free(lrep[k]); free(lrc[k]); }
    CHECK(sky_ctx_destroy(ctx));
    free(ks); free(lid); free(lval); free(lrep); free(lrc); free(lcnt); free(lnr); free(part_ids); free(g_full); free(gids); free(gorg); free(lsz); free(surv);
    free(keys); free(ids); free(vals); free(text);
    return 0;
}

int cmp_i64(const void *a, const void *b) {
    const int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
    return x < y ? -1 : x > y;
}
