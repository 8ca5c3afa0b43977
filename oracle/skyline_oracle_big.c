/*
 * oracle/skyline_oracle_big.c — TEST INFRASTRUCTURE ONLY (the checker; the product never
 * links it).  The same query as orc_query_sfs (skyline_oracle.c), sized for the BASELINE
 * configurations C2-C4 (10M-100M tuples), where the single-threaded SFS restatement would
 * take minutes:
 *
 *   keys            orc_keys (FlinkSkyline.java:707-712 / :774-789 / :827-875), in slices
 *                   on T threads
 *   chunk phase     every chunk of `chunk` tuples: per key, the skyline of the chunk's tuples
 *                   of that key (a tuple dominated inside its chunk is dominated in the
 *                   stream: SKY(U_c SKY(chunk_c)) = SKY(U_c chunk_c))
 *   key phase       per key k < K: SKY_k over the chunk survivors of key k = L_k
 *                   (processBuffer's BNL result as a set, FlinkSkyline.java:417-444)
 *   global phase    SKY over the union of the L_k = G (the merge, :548-566)
 *   stats           |L_k|, survivors_k (:593-608)
 *
 * Each skyline is computed over DISTINCT vectors: the rows are hashed (−0.0 and +0.0 are
 * one value, as Java's < and > see them), the distinct vectors are sorted by (sum, lex) and
 * scanned against the confirmed skyline (the SFS restatement, dominance =
 * ServiceTuple.dominates, ServiceTuple.java:67-77); a vector's fate is every duplicate's
 * fate (equal vectors never dominate each other).  Rows must be NaN-free.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

int orc_dominates(const double *a, const double *b, int d);
void orc_keys(int algo, const double *vals, int64_t n, int D, int P, double domain, int32_t *out);

enum { ALGO_GRID_ = 1, SEM_COMPLETE_ = 1 };

static inline uint64_t mixh(uint64_t z) {
    z ^= z >> 33;
    z *= 0xff51afd7ed558ccdull;
    z ^= z >> 33;
    z *= 0xc4ceb9fe1a85ec53ull;
    return z ^ (z >> 33);
}

static uint64_t row_hash(const double *v, int D) {
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (int d = 0; d < D; d++) {
        double x = v[d] + 0.0;   /* -0.0 -> +0.0 */
        uint64_t b;
        memcpy(&b, &x, 8);
        h = mixh(h ^ b) + (uint64_t)d;
    }
    return h;
}

static int row_eq(const double *a, const double *b, int D) {
    for (int d = 0; d < D; d++)
        if (!(a[d] == b[d])) return 0;
    return 1;
}

typedef struct { double s; int64_t r; } rep_item;   /* r = representative index */
static __thread const double *t_vals;
static __thread const int64_t *t_rep_row;
static __thread int t_D;

static int rep_cmp(const void *pa, const void *pb) {
    const rep_item *a = (const rep_item *)pa, *b = (const rep_item *)pb;
    if (a->s < b->s) return -1;
    if (a->s > b->s) return 1;
    const double *va = t_vals + t_rep_row[a->r] * t_D, *vb = t_vals + t_rep_row[b->r] * t_D;
    for (int d = 0; d < t_D; d++) {
        if (va[d] < vb[d]) return -1;
        if (va[d] > vb[d]) return 1;
    }
    return a->r < b->r ? -1 : a->r > b->r;
}

/* flag[idx[j]] = 1 iff row idx[j] is in the skyline of the rows idx[0..m) */
static void sky_subset_hashed(const double *vals, int D, const int64_t *idx, int64_t m, uint8_t *flag) {
    if (m <= 0) return;
    int64_t cap = 64;
    while (cap < 2 * m) cap <<= 1;
    int64_t *slot = (int64_t *)malloc((size_t)cap * sizeof(int64_t));   /* rep index or -1 */
    for (int64_t q = 0; q < cap; q++) slot[q] = -1;
    int64_t *rep_of = (int64_t *)malloc((size_t)m * sizeof(int64_t));
    int64_t *rep_row = (int64_t *)malloc((size_t)m * sizeof(int64_t));
    int64_t nrep = 0;
    for (int64_t j = 0; j < m; j++) {      /* distinct vectors: first row of each is its rep */
        const double *v = vals + idx[j] * D;
        int64_t q = (int64_t)(row_hash(v, D) & (uint64_t)(cap - 1));
        for (;;) {
            if (slot[q] < 0) {
                slot[q] = nrep;
                rep_row[nrep] = idx[j];
                rep_of[j] = nrep++;
                break;
            }
            if (row_eq(vals + rep_row[slot[q]] * D, v, D)) {
                rep_of[j] = slot[q];
                break;
            }
            q = (q + 1) & (cap - 1);
        }
    }
    free(slot);
    rep_item *it = (rep_item *)malloc((size_t)nrep * sizeof(rep_item));
    for (int64_t r = 0; r < nrep; r++) {
        const double *v = vals + rep_row[r] * D;
        double s = 0.0;   /* clamped: the sum stays monotone under dominance */
        for (int d = 0; d < D; d++) s += v[d] > 1e300 ? 1e300 : (v[d] < -1e300 ? -1e300 : v[d]);
        it[r].s = s;
        it[r].r = r;
    }
    t_vals = vals;
    t_rep_row = rep_row;
    t_D = D;
    qsort(it, (size_t)nrep, sizeof(rep_item), rep_cmp);
    /* SFS: (sum, lex) is a linear extension of dominance among distinct vectors */
    int64_t *sky = (int64_t *)malloc((size_t)nrep * sizeof(int64_t));
    uint8_t *rep_alive = (uint8_t *)calloc((size_t)nrep, 1);
    int64_t ns = 0;
    for (int64_t p = 0; p < nrep; p++) {
        const double *v = vals + rep_row[it[p].r] * D;
        int dom = 0;
        for (int64_t q = 0; q < ns && !dom; q++) dom = orc_dominates(vals + sky[q] * D, v, D);
        if (!dom) {
            sky[ns++] = rep_row[it[p].r];
            rep_alive[it[p].r] = 1;
        }
    }
    for (int64_t j = 0; j < m; j++) flag[idx[j]] = rep_alive[rep_of[j]];
    free(it);
    free(sky);
    free(rep_alive);
    free(rep_of);
    free(rep_row);
}

/* ---- a minimal work queue over T threads ---- */
typedef struct {
    void (*fn)(void *ctx, int64_t item);
    void *ctx;
    int64_t nitems;
    int64_t next;
    pthread_mutex_t mu;
} wq;

static void *wq_worker(void *arg) {
    wq *q = (wq *)arg;
    for (;;) {
        pthread_mutex_lock(&q->mu);
        int64_t i = q->next++;
        pthread_mutex_unlock(&q->mu);
        if (i >= q->nitems) return NULL;
        q->fn(q->ctx, i);
    }
}

static void run_parallel(int T, int64_t nitems, void (*fn)(void *, int64_t), void *ctx) {
    wq q;
    q.fn = fn;
    q.ctx = ctx;
    q.nitems = nitems;
    q.next = 0;
    pthread_mutex_init(&q.mu, NULL);
    if (T < 1) T = 1;
    if (T > 64) T = 64;
    pthread_t th[64];
    for (int t = 0; t < T; t++) pthread_create(&th[t], NULL, wq_worker, &q);
    for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
    pthread_mutex_destroy(&q.mu);
}

typedef struct {
    int algo, D, P, K;
    double domain;
    const double *vals;
    int64_t n, chunk;
    int32_t *keys;
    uint8_t *in_local;
    /* key phase */
    int64_t *kbeg;
    int64_t *korder;
} big_ctx;

static void keys_item(void *cp, int64_t c) {
    big_ctx *b = (big_ctx *)cp;
    int64_t lo = c * b->chunk, hi = lo + b->chunk < b->n ? lo + b->chunk : b->n;
    orc_keys(b->algo, b->vals + lo * b->D, hi - lo, b->D, b->P, b->domain, b->keys + lo);
}

static void chunk_item(void *cp, int64_t c) {
    big_ctx *b = (big_ctx *)cp;
    int64_t lo = c * b->chunk, hi = lo + b->chunk < b->n ? lo + b->chunk : b->n;
    int K = b->K;
    int64_t *cnt = (int64_t *)calloc((size_t)K + 1, sizeof(int64_t));
    for (int64_t i = lo; i < hi; i++)
        if (b->keys[i] >= 0 && b->keys[i] < K) cnt[b->keys[i] + 1]++;
    for (int k = 0; k < K; k++) cnt[k + 1] += cnt[k];
    int64_t *order = (int64_t *)malloc((size_t)(cnt[K] > 0 ? cnt[K] : 1) * sizeof(int64_t));
    int64_t *fill = (int64_t *)malloc((size_t)K * sizeof(int64_t));
    for (int k = 0; k < K; k++) fill[k] = cnt[k];
    for (int64_t i = lo; i < hi; i++)
        if (b->keys[i] >= 0 && b->keys[i] < K) order[fill[b->keys[i]]++] = i;
    for (int k = 0; k < K; k++) sky_subset_hashed(b->vals, b->D, order + cnt[k], cnt[k + 1] - cnt[k], b->in_local);
    free(cnt);
    free(order);
    free(fill);
}

static void key_item(void *cp, int64_t k) {
    big_ctx *b = (big_ctx *)cp;
    sky_subset_hashed(b->vals, b->D, b->korder + b->kbeg[k], b->kbeg[k + 1] - b->kbeg[k], b->in_local);
}

/* Returns |G|, or -1 for bad arguments.  keys_out[n], in_local[n], in_global[n],
 * local_sizes[K], survivors[K] (K = P, or max(P, 2^D) for complete MR-Grid). */
int64_t orc_query_sfs_chunked(int algo, const double *vals, int64_t n, int D, int P, double domain, int semantics,
                              int64_t chunk, int nthreads, int32_t *keys_out, uint8_t *in_local, uint8_t *in_global,
                              int64_t *local_sizes, int64_t *survivors) {
    int K = P;
    if (algo == ALGO_GRID_ && semantics == SEM_COMPLETE_) {
        if (D > 16) return -1;
        K = (1 << D) > P ? (1 << D) : P;
    }
    if (chunk < 1) chunk = 1 << 20;
    big_ctx b = {algo, D, P, K, domain, vals, n, chunk, keys_out, in_local, NULL, NULL};
    const int64_t nch = (n + chunk - 1) / chunk;
    memset(in_local, 0, (size_t)n);
    memset(in_global, 0, (size_t)n);
    run_parallel(nthreads, nch, keys_item, &b);
    run_parallel(nthreads, nch, chunk_item, &b);
    /* key phase over the chunk survivors, stream order within a key */
    int64_t *kbeg = (int64_t *)calloc((size_t)K + 1, sizeof(int64_t));
    for (int64_t i = 0; i < n; i++)
        if (in_local[i]) kbeg[keys_out[i] + 1]++;
    for (int k = 0; k < K; k++) kbeg[k + 1] += kbeg[k];
    int64_t *korder = (int64_t *)malloc((size_t)(kbeg[K] > 0 ? kbeg[K] : 1) * sizeof(int64_t));
    int64_t *fill = (int64_t *)malloc((size_t)K * sizeof(int64_t));
    for (int k = 0; k < K; k++) fill[k] = kbeg[k];
    for (int64_t i = 0; i < n; i++)
        if (in_local[i]) {
            korder[fill[keys_out[i]]++] = i;
            in_local[i] = 0;
        }
    b.kbeg = kbeg;
    b.korder = korder;
    run_parallel(nthreads, K, key_item, &b);
    /* global phase over the union of the local skylines */
    int64_t nl = 0;
    for (int64_t j = 0; j < kbeg[K]; j++)
        if (in_local[korder[j]]) korder[nl++] = korder[j];
    sky_subset_hashed(vals, D, korder, nl, in_global);
    int64_t g = 0;
    for (int k = 0; k < K; k++) { local_sizes[k] = 0; survivors[k] = 0; }
    for (int64_t j = 0; j < nl; j++) {
        int64_t i = korder[j];
        local_sizes[keys_out[i]]++;
        if (in_global[i]) { survivors[keys_out[i]]++; g++; }
    }
    free(kbeg);
    free(korder);
    free(fill);
    return g;
}
