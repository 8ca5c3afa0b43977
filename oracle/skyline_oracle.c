/*
 * oracle/skyline_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference skyline hot path, used solely as the
 * checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
 * The product (flink-skyline-qos_amd/, libskyline_hip.so) never links, loads or
 * calls anything in this directory.
 *
 * Every function cites the reference line it restates (paths relative to
 * /root/reference/java/org.main/).
 *
 * Parity status: the reference hot path is Java/Flink and there is no JDK in
 * this container, so this restatement could not be run against
 * the reference binary: parity of the OPERATOR OUTPUTS is "unpinned" against
 * the Java job.  What IS pinned: the input streams (tests/golden/ holds streams
 * emitted by the reference's own generator functions), the fdlibm constants
 * (hex words), and the PDF p.15 qualitative KAT (correlated skyline = all
 * [0,...,0] duplicates).  BNL, brute force and SFS are cross-checked here.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

double orc_fdlibm_atan2(double y, double x);

enum { ALGO_DIM = 0, ALGO_GRID = 1, ALGO_ANGLE = 2 };
enum { SEM_REFERENCE = 0, SEM_COMPLETE = 1 };

/* ServiceTuple.dominates (ServiceTuple.java:67-77): minimisation, early exit
 * on the first a[i] > b[i]; NaN compares false both ways. */
int orc_dominates(const double *a, const double *b, int d) {
    int better = 0;
    for (int i = 0; i < d; i++) {
        if (a[i] > b[i]) return 0;
        if (a[i] < b[i]) better = 1;
    }
    return better;
}

/* Java (int) narrowing of a double (JLS 5.1.3): NaN -> 0, saturating, else
 * truncation toward zero. */
int32_t orc_java_d2i(double x) {
    if (x != x) return 0;
    if (x >= 2147483647.0) return 2147483647;
    if (x <= -2147483648.0) return (int32_t)0x80000000u;
    return (int32_t)x;
}

/* DimPartitioner.getKey (FlinkSkyline.java:707-712) */
int32_t orc_key_dim(const double *v, int P, double maxVal) {
    int32_t p = orc_java_d2i(v[0] / (maxVal / P));
    if (p > P - 1) p = P - 1;
    if (p < 0) p = 0;
    return p;
}

/* GridPartitioner (FlinkSkyline.java:750-789): mids[i] = maxVal/2.0 (:756);
 * mask |= (1 << i) when values[i] >= mids[i] (:780-785).  Java's int shift
 * uses (i & 31).  No clamp and no modulo: keys lie in [0, 2^D). */
/* GridDominanceFilter (FlinkSkyline.java:716-733, commented out in the reference):
 * when enabled, a tuple is kept iff some value is < maxVal/2 ("!allWorse"); a removed
 * tuple never reaches keyBy (key -1 here).  Process-wide switch for the tests. */
static int g_grid_filter = 0;
void orc_set_grid_filter(int on) { g_grid_filter = on; }

int32_t orc_key_grid(const double *v, int D, double maxVal) {
    double mid = maxVal / 2.0;
    uint32_t mask = 0;
    int allWorse = 1;
    for (int i = 0; i < D; i++) {
        if (v[i] >= mid) mask |= (1u << (i & 31));
        if (v[i] < mid) allWorse = 0;                 /* :726-729 */
    }
    if (g_grid_filter && allWorse) return -1;
    return (int32_t)mask;
}

/* AnglePartitioner.getKey (FlinkSkyline.java:827-875) */
int32_t orc_key_angle(const double *v, int D, int P) {
    int numAngles = D - 1;
    if (numAngles < 1) return 0;                       /* :832 */
    double normalizedSum = 0.0;
    const double maxAngle = 3.141592653589793 / 2.0;   /* Math.PI / 2.0, :856 */
    for (int i = 0; i < numAngles; i++) {
        double v_i = v[i];
        double sumSqRest = 0.0;
        for (int j = i + 1; j < D; j++) {
            double sq = v[j] * v[j];
            sumSqRest += sq;                           /* :844-846, no FMA */
        }
        double hyp = sqrt(sumSqRest);                  /* :847, correctly rounded */
        double angle = orc_fdlibm_atan2(hyp, v_i);     /* :850 */
        normalizedSum += angle / maxAngle;             /* :860-863 */
    }
    double avgPosition = normalizedSum / numAngles;    /* :866 */
    int32_t p = orc_java_d2i(avgPosition * P);         /* :870 */
    if (p > P - 1) p = P - 1;
    if (p < 0) p = 0;
    return p;
}

void orc_keys(int algo, const double *vals, int64_t n, int D, int P, double domain, int32_t *out) {
    for (int64_t i = 0; i < n; i++) {
        const double *v = vals + i * D;
        out[i] = algo == ALGO_DIM ? orc_key_dim(v, P, domain)
               : algo == ALGO_GRID ? orc_key_grid(v, D, domain)
               : orc_key_angle(v, D, P);
    }
}

/* ------------------------------------------------------------------------ */
/* BNL list (an ArrayList<ServiceTuple> of row indices)                      */

typedef struct { int64_t *a; int64_t len, cap; } ilist;

static void il_push(ilist *l, int64_t x) {
    if (l->len == l->cap) {
        l->cap = l->cap ? l->cap * 2 : 64;
        l->a = (int64_t *)realloc(l->a, (size_t)l->cap * sizeof(int64_t));
    }
    l->a[l->len++] = x;
}

/* One BNL step for candidate c against list S, in the exact iteration order of
 * SkylineLocalProcessor.processBuffer (FlinkSkyline.java:424-441) and of the
 * GlobalSkylineAggregator merge (:549-565): scan; break when an existing point
 * dominates c; Iterator.remove() each existing point c dominates; append c if
 * it survived. */
static void bnl_step(ilist *S, int64_t c, const double *vals, int D) {
    const double *cv = vals + c * D;
    int64_t w = 0;
    int dominated = 0;
    for (int64_t r = 0; r < S->len; r++) {
        int64_t e = S->a[r];
        if (!dominated) {
            const double *ev = vals + e * D;
            if (orc_dominates(ev, cv, D)) { dominated = 1; S->a[w++] = e; continue; }
            if (orc_dominates(cv, ev, D)) continue;          /* it.remove() */
        }
        S->a[w++] = e;
    }
    S->len = w;
    if (!dominated) il_push(S, c);
}

/*
 * Whole-stream query with reference semantics (the trigger arrives after the
 * last tuple):
 *   keyBy(partitioner) (:138) -> per key: buffer, BNL flush every
 *   buffer_size tuples (:286-289, :232) -> processQuery flushes the rest and
 *   emits the key's list tagged originPartition = key (:372-392) ->
 *   GlobalSkylineAggregator merges the lists of keys 0..P-1 (:152-154, :548-566)
 *   -> optimality integers (:593-608).
 * Reference semantics only query keys 0..P-1; for MR-Grid keys >= P are
 * never merged.  SEM_COMPLETE queries every key in [0, K).
 * Deviation kept from the build: the buffer is per key (the reference shares
 * one buffer across all keys of a subtask, :223,244 — a bug that moves tuples
 * between keys; for Dim/Angle it does not change the skyline set).
 *
 * Outputs: global skyline ids (merge order) + origin key, |L_k| for k < K and
 * survivors_k.  Returns |G| (or -1 if cap is too small / bad args).
 */
int64_t orc_query_bnl(int algo, const double *vals, const int64_t *ids, int64_t n, int D, int P,
                      double domain, int buffer_size, int semantics,
                      int64_t *out_ids, int32_t *out_origin, int64_t cap,
                      int64_t *local_sizes, int64_t *survivors) {
    int K = P;
    if (algo == ALGO_GRID && semantics == SEM_COMPLETE) {
        if (D > 16) return -1;
        K = (1 << D) > P ? (1 << D) : P;
    }
    int32_t *keys = (int32_t *)malloc((size_t)(n > 0 ? n : 1) * sizeof(int32_t));
    orc_keys(algo, vals, n, D, P, domain, keys);
    ilist *state = (ilist *)calloc((size_t)K, sizeof(ilist));
    ilist *buf = (ilist *)calloc((size_t)K, sizeof(ilist));
    for (int64_t i = 0; i < n; i++) {
        int32_t k = keys[i];
        if (k < 0 || k >= K) continue;        /* a key nobody ever queries */
        il_push(&buf[k], i);
        if (buf[k].len >= buffer_size) {
            for (int64_t j = 0; j < buf[k].len; j++) bnl_step(&state[k], buf[k].a[j], vals, D);
            buf[k].len = 0;
        }
    }
    ilist G = {0};
    int32_t *origin_of = (int32_t *)malloc((size_t)(n > 0 ? n : 1) * sizeof(int32_t));
    for (int k = 0; k < K; k++) {
        for (int64_t j = 0; j < buf[k].len; j++) bnl_step(&state[k], buf[k].a[j], vals, D);
        buf[k].len = 0;
        local_sizes[k] = state[k].len;
        survivors[k] = 0;
        for (int64_t j = 0; j < state[k].len; j++) {
            origin_of[state[k].a[j]] = k;
            bnl_step(&G, state[k].a[j], vals, D);
        }
    }
    int64_t g = G.len;
    for (int64_t j = 0; j < g; j++) {
        int64_t r = G.a[j];
        survivors[origin_of[r]]++;
        if (j < cap) { out_ids[j] = ids[r]; out_origin[j] = origin_of[r]; }
    }
    for (int k = 0; k < K; k++) { free(state[k].a); free(buf[k].a); }
    free(state); free(buf); free(G.a); free(keys); free(origin_of);
    return g <= cap ? g : -1;
}

/*
 * The same query with the local phase run the way the Flink job parallelises it:
 * one thread per operator subtask, each owning the keys k with k % nthreads == t
 * (Flink's murmur key-group assignment is not vendored; round-robin stands in for
 * it), running the per-key buffer + BNL of processElement1/processBuffer
 * (FlinkSkyline.java:265-316, :417-444) over its keys' tuples in stream order.
 * The global merge stays single-threaded, as GlobalSkylineAggregator is keyed by
 * the query (:515-569).  Used only as the multi-core CPU baseline of bench.py;
 * results are identical to orc_query_bnl (the keys are independent).
 */
#include <pthread.h>

typedef struct {
    const double *vals;
    const int32_t *keys;
    int64_t n;
    int D, K, buffer_size, t, T;
    ilist *state;
} bnl_task;

static void *bnl_worker(void *arg) {
    bnl_task *a = (bnl_task *)arg;
    ilist *buf = (ilist *)calloc((size_t)a->K, sizeof(ilist));
    for (int64_t i = 0; i < a->n; i++) {
        int32_t k = a->keys[i];
        if (k < 0 || k >= a->K || k % a->T != a->t) continue;
        il_push(&buf[k], i);
        if (buf[k].len >= a->buffer_size) {
            for (int64_t j = 0; j < buf[k].len; j++) bnl_step(&a->state[k], buf[k].a[j], a->vals, a->D);
            buf[k].len = 0;
        }
    }
    for (int k = a->t; k < a->K; k += a->T) {
        for (int64_t j = 0; j < buf[k].len; j++) bnl_step(&a->state[k], buf[k].a[j], a->vals, a->D);
        free(buf[k].a);
    }
    free(buf);
    return NULL;
}

int64_t orc_query_bnl_mt(int algo, const double *vals, const int64_t *ids, int64_t n, int D, int P, double domain,
                         int buffer_size, int nthreads, int64_t *out_ids, int32_t *out_origin, int64_t cap,
                         int64_t *local_sizes, int64_t *survivors) {
    const int K = P;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    int32_t *keys = (int32_t *)malloc((size_t)(n > 0 ? n : 1) * sizeof(int32_t));
    orc_keys(algo, vals, n, D, P, domain, keys);
    ilist *state = (ilist *)calloc((size_t)K, sizeof(ilist));
    pthread_t th[256];
    bnl_task task[256];
    for (int t = 0; t < nthreads; t++) {
        task[t] = (bnl_task){vals, keys, n, D, K, buffer_size, t, nthreads, state};
        pthread_create(&th[t], NULL, bnl_worker, &task[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    ilist G = {0};
    int32_t *origin_of = (int32_t *)malloc((size_t)(n > 0 ? n : 1) * sizeof(int32_t));
    for (int k = 0; k < K; k++) {
        local_sizes[k] = state[k].len;
        survivors[k] = 0;
        for (int64_t j = 0; j < state[k].len; j++) {
            origin_of[state[k].a[j]] = k;
            bnl_step(&G, state[k].a[j], vals, D);
        }
    }
    int64_t g = G.len;
    for (int64_t j = 0; j < g; j++) {
        int64_t r = G.a[j];
        survivors[origin_of[r]]++;
        if (j < cap) { out_ids[j] = ids[r]; out_origin[j] = origin_of[r]; }
    }
    for (int k = 0; k < K; k++) free(state[k].a);
    free(state); free(G.a); free(keys); free(origin_of);
    return g <= cap ? g : -1;
}

/* Definition check: brute-force skyline membership (test oracle for BNL). */
void orc_skyline_brute(const double *vals, int64_t n, int D, uint8_t *in_sky) {
    for (int64_t i = 0; i < n; i++) {
        int dom = 0;
        for (int64_t j = 0; j < n && !dom; j++)
            if (j != i && orc_dominates(vals + j * D, vals + i * D, D)) dom = 1;
        in_sky[i] = (uint8_t)!dom;
    }
}

/* ------------------------------------------------------------------------ */
/* SFS restatement for larger streams: the skyline SET equals BNL's (the BNL  */
/* result is order-independent for a strict partial order), so per key:      */
/* sort by (sum, lex), collapse exact duplicates, scan against the survivors.  */

typedef struct { double s; int64_t i; } sfs_item;
static const double *g_sfs_vals;
static int g_sfs_D;

static int sfs_cmp(const void *pa, const void *pb) {
    const sfs_item *a = (const sfs_item *)pa, *b = (const sfs_item *)pb;
    if (a->s < b->s) return -1;
    if (a->s > b->s) return 1;
    const double *va = g_sfs_vals + a->i * g_sfs_D, *vb = g_sfs_vals + b->i * g_sfs_D;
    for (int d = 0; d < g_sfs_D; d++) {
        if (va[d] < vb[d]) return -1;
        if (va[d] > vb[d]) return 1;
    }
    return a->i < b->i ? -1 : a->i > b->i;
}

/* in_sky[j] for the rows listed in idx[0..m).  Rows must be NaN-free: the
 * (sum, lex) order is then a linear extension of dominance among distinct
 * vectors (a dominates b => sum(a) <= sum(b) by monotone rounding, and on a
 * tie the first differing coordinate is smaller). */
static void sfs_subset(const double *vals, int D, const int64_t *idx, int64_t m, uint8_t *in_sky_rows) {
    sfs_item *it = (sfs_item *)malloc((size_t)(m > 0 ? m : 1) * sizeof(sfs_item));
    for (int64_t j = 0; j < m; j++) {
        const double *v = vals + idx[j] * D;
        double s = 0.0;   /* clamped: +inf and -inf never meet, the sum stays monotone */
        for (int d = 0; d < D; d++) s += v[d] > 1e300 ? 1e300 : (v[d] < -1e300 ? -1e300 : v[d]);
        it[j].s = s; it[j].i = idx[j];
    }
    g_sfs_vals = vals; g_sfs_D = D;
    qsort(it, (size_t)m, sizeof(sfs_item), sfs_cmp);
    int64_t *sky = (int64_t *)malloc((size_t)(m > 0 ? m : 1) * sizeof(int64_t));
    int64_t ns = 0;
    int64_t j = 0;
    while (j < m) {
        int64_t e = j + 1;       /* run of exact duplicates shares one fate */
        while (e < m) {
            const double *a = vals + it[j].i * D, *b = vals + it[e].i * D;
            int eq = 1;
            for (int d = 0; d < D; d++) if (!(a[d] == b[d])) { eq = 0; break; }
            if (!eq) break;
            e++;
        }
        const double *v = vals + it[j].i * D;
        int dom = 0;
        for (int64_t q = 0; q < ns && !dom; q++) dom = orc_dominates(vals + sky[q] * D, v, D);
        if (!dom) sky[ns++] = it[j].i;
        for (int64_t q = j; q < e; q++) in_sky_rows[it[q].i] = (uint8_t)!dom;
        j = e;
    }
    free(it); free(sky);
}

/* Same outputs as orc_query_bnl, as per-row flags: in_local[i] (row i is in
 * its key's local skyline) and in_global[i].  keys_out[i] = partition key. */
int64_t orc_query_sfs(int algo, const double *vals, int64_t n, int D, int P, double domain,
                      int semantics, int32_t *keys_out, uint8_t *in_local, uint8_t *in_global,
                      int64_t *local_sizes, int64_t *survivors) {
    int K = P;
    if (algo == ALGO_GRID && semantics == SEM_COMPLETE) {
        if (D > 16) return -1;
        K = (1 << D) > P ? (1 << D) : P;
    }
    orc_keys(algo, vals, n, D, P, domain, keys_out);
    int64_t *cnt = (int64_t *)calloc((size_t)K + 1, sizeof(int64_t));
    for (int64_t i = 0; i < n; i++) {
        in_local[i] = 0; in_global[i] = 0;
        if (keys_out[i] >= 0 && keys_out[i] < K) cnt[keys_out[i] + 1]++;
    }
    for (int k = 0; k < K; k++) cnt[k + 1] += cnt[k];
    int64_t *order = (int64_t *)malloc((size_t)(cnt[K] > 0 ? cnt[K] : 1) * sizeof(int64_t));
    int64_t *fill = (int64_t *)malloc((size_t)K * sizeof(int64_t));
    for (int k = 0; k < K; k++) fill[k] = cnt[k];
    for (int64_t i = 0; i < n; i++)
        if (keys_out[i] >= 0 && keys_out[i] < K) order[fill[keys_out[i]]++] = i;
    for (int k = 0; k < K; k++) sfs_subset(vals, D, order + cnt[k], cnt[k + 1] - cnt[k], in_local);
    int64_t nl = 0;
    for (int64_t j = 0; j < cnt[K]; j++) if (in_local[order[j]]) order[nl++] = order[j];
    sfs_subset(vals, D, order, nl, in_global);
    int64_t g = 0;
    for (int k = 0; k < K; k++) { local_sizes[k] = 0; survivors[k] = 0; }
    for (int64_t j = 0; j < nl; j++) {
        int64_t i = order[j];
        local_sizes[keys_out[i]]++;
        if (in_global[i]) { survivors[keys_out[i]]++; g++; }
    }
    /* rows that never reached the merge must not be flagged global */
    free(cnt); free(order); free(fill);
    return g;
}

/* ------------------------------------------------------------------------ */
/* Synthetic streams: restatement of python/unified_producer.py:50-123 with a */
/* counter-based RNG so that the device generator of the product            */
/* (flink-skyline-qos_amd/csrc/k_synth.hip) can be checked value-for-value.    */
/* dist: 0 uniform, 1 correlated, 2 anti_correlated (reference formula),       */
/* 3 std_anti (Borzsonyi-style plane band; EXTENSION, not in the reference),  */
/* 4 mixed (blocks of 65536 tuples cycling 0,1,2; EXTENSION for config C5).   */

static inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static inline double rnd(uint64_t seed, uint64_t i, uint32_t j) {
    uint64_t h = mix64(mix64(seed) ^ (i * 0xD1B54A32D192ED03ull) ^ ((uint64_t)j * 0x8CB92BA72F3D8DD7ull));
    return (double)(h >> 11) * (1.0 / 9007199254740992.0);   /* [0,1), as random.random() */
}
static inline double clamp_trunc(double v, int dmin, int dmax) {
    int64_t t = (int64_t)v;                                 /* Python int(): toward zero */
    if (t > dmax) t = dmax;
    if (t < dmin) t = dmin;
    return (double)t;
}
static double anti_eps(int D) {                              /* unified_producer.py:93-104 */
    if (D == 2) return 0.0005;
    if (D == 3) return 0.05;
    if (D == 4) return 0.9;
    return (double)D * 0.005 * 100;
}

void orc_synth(int dist, int D, int dmin, int dmax, uint64_t seed, int64_t id0, int64_t n, double *out) {
    for (int64_t r = 0; r < n; r++) {
        uint64_t i = (uint64_t)(id0 + r);
        double *v = out + r * D;
        int dd = dist;
        if (dist == 4) dd = (int)((i >> 16) % 3);
        if (dd == 0) {                                       /* :50-51 */
            double range = (double)(dmax - dmin + 1);
            for (int d = 0; d < D; d++) v[d] = (double)(dmin + (int64_t)floor(rnd(seed, i, d) * range));
        } else if (dd == 1) {                                /* :63-76, rho = 0.9 */
            double a = (double)dmin, b = (double)dmax;
            double base = a + (b - a) * rnd(seed, i, 0);
            double lo = -(1 - 0.9) * (double)(dmax - dmin);
            double hi = +(1 - 0.9) * (double)(dmax - dmin);
            for (int d = 0; d < D; d++) {
                double noise = lo + (hi - lo) * rnd(seed, i, 1 + d);
                v[d] = clamp_trunc(base + noise, dmin, dmax);
            }
        } else if (dd == 2) {                                /* :89-123 */
            double eps = anti_eps(D);
            double total = 0.0;
            for (int d = 0; d < D; d++) { v[d] = rnd(seed, i, d); total += v[d]; }
            double mean = (double)(dmin + dmax) / 2.0 * D;
            double slack = eps * (double)(dmax - dmin) * D;
            double lo = mean - slack, hi = mean + slack;
            double target = lo + (hi - lo) * rnd(seed, i, 32);
            double scale = total != 0 ? target / total : 1.0;
            for (int d = 0; d < D; d++) v[d] = clamp_trunc(v[d] * scale, dmin, dmax);
        } else {                                             /* std_anti extension */
            /* plane sum/D ~ 0.5 + 0.05*IrwinHall4-centred; points spread on the
             * plane by a symmetric shift; rows outside the cube are re-drawn. */
            double c = 0.5 + 0.05 * ((rnd(seed, i, 40) + rnd(seed, i, 41) + rnd(seed, i, 42) + rnd(seed, i, 43)) - 2.0);
            int ok = 0;
            for (uint32_t att = 0; att < 8 && !ok; att++) {
                double mean = 0.0;
                for (int d = 0; d < D; d++) { v[d] = rnd(seed, i, 64 + att * 32 + d); mean += v[d]; }
                mean = mean / D;
                ok = 1;
                for (int d = 0; d < D; d++) {
                    v[d] = v[d] + (c - mean);
                    if (v[d] < 0.0 || v[d] >= 1.0) ok = 0;
                }
            }
            double range = (double)(dmax - dmin);
            for (int d = 0; d < D; d++) {
                double x = v[d] < 0.0 ? 0.0 : (v[d] >= 1.0 ? 0.9999999999999999 : v[d]);
                v[d] = (double)(dmin + (int64_t)floor(x * range));
            }
        }
    }
}
