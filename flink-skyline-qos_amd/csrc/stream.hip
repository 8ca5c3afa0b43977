// stream.hip — continuous queries (sky_stream_*, config C5): a query's resident state in HBM,
// micro-batch appends, and a query over everything that counts at the trigger.
//
// Landmark window (the reference: every tuple since the job started counts,
// FlinkSkyline.java:221-249, 265-316): after a query only the tuples of the local skylines
// matter, SKY_k(L_k u new_k) = SKY_k(every tuple of key k).  The state holds them as DISTINCT
// VECTORS, as the per-key operator state does (part.hip): R reps (f64 row, partition key, tuple
// count) plus the tuples (id, rep) in arrival order.  On the reference streams the local
// skylines are mostly copies of one all-zero vector, so the next query runs over R + N rows
// (N = appended since) instead of every resident tuple.  A query:
//   1. the new rows' keys (launch_keys); the reps keep theirs (given keys)
//   2. pipe_run over [reps ; new rows], weights = [tuple counts ; 1]: weighted |L_k| /
//      survivors_k, and a fate per row (bit 0: in L_k, bit 1: in G)
//   3. the output, arrival order: the resident tuples whose rep is in G, then the new tuples in G
//   4. the next state: the reps in L_k (compacted) and the new rows in L_k, merged into them by
//      (key, row bits) in a device hash table; the resident tuples of surviving reps, then the
//      new local tuples, in arrival order.
// Sliding window (count-based, the last W appended tuples; a labelled extension): all W stay
// resident (expiry needs the non-skyline tuples) in a 2W ring, and each query runs over them.
#include "abi_common.h"
#include "knobs.h"

#include <algorithm>
#include <vector>

namespace sky {
namespace {

constexpr uint64_t kHashEmpty = ~0ull;

__device__ __forceinline__ uint32_t row_hash(const double *r, int D, int32_t key) {
    uint64_t h = 0x9e3779b97f4a7c15ull ^ (uint64_t)(uint32_t)key;
    for (int d = 0; d < D; d++) {
        h ^= (uint64_t)__double_as_longlong(r[d]);
        h *= 0xff51afd7ed558ccdull;
        h ^= h >> 33;
    }
    return (uint32_t)(h ^ (h >> 32));
}
// a published rep's row, read past this CU's L1 (another workgroup wrote it during this kernel;
// a line cached here earlier for a neighbouring rep would be stale)
__device__ __forceinline__ bool same_row(const double *pub, const double *b, int D) {
    bool eq = true;
    const unsigned long long *a = reinterpret_cast<const unsigned long long *>(pub);
    for (int d = 0; d < D; d++)
        eq &= __hip_atomic_load(a + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
              (unsigned long long)__double_as_longlong(b[d]);
    return eq;
}

// output selection over [resident tuples ; new rows]: t < T -> its rep's fate, else new row R + t - T
__global__ __launch_bounds__(kThreads) void k_ls_select(uint32_t T, uint32_t N, uint32_t R,
                                                        const uint32_t *__restrict__ trep,
                                                        const uint8_t *__restrict__ rowf, uint32_t bit,
                                                        uint32_t *__restrict__ flag) {
    const uint32_t t = blockIdx.x * kThreads + threadIdx.x;
    if (t >= T + N) return;
    const uint32_t row = t < T ? trep[t] : R + (t - T);
    flag[t] = (rowf[row] & bit) ? 1u : 0u;
}
// the global skyline's ids / origins (the rep's or the row's partition key) in arrival order
__global__ __launch_bounds__(kThreads) void k_ls_write_out(uint32_t T, uint32_t N, uint32_t R,
                                                           const int64_t *__restrict__ tid,
                                                           const uint32_t *__restrict__ trep,
                                                           const int64_t *__restrict__ qids,
                                                           const int32_t *__restrict__ qkey,
                                                           const uint32_t *__restrict__ flag,
                                                           const uint32_t *__restrict__ pos, int64_t cap,
                                                           int64_t *__restrict__ ids_out,
                                                           int32_t *__restrict__ org_out) {
    const uint32_t t = blockIdx.x * kThreads + threadIdx.x;
    if (t >= T + N || !flag[t]) return;
    const uint32_t o = pos[t];
    if ((int64_t)o >= cap) return;
    const uint32_t row = t < T ? trep[t] : R + (t - T);
    if (ids_out) ids_out[o] = t < T ? tid[t] : qids[row];
    if (org_out) org_out[o] = qkey[row];
}
// the reps in L_k: flags for the scan that numbers them
__global__ __launch_bounds__(kThreads) void k_ls_rep_flag(uint32_t R, const uint8_t *__restrict__ rowf,
                                                          uint32_t *__restrict__ flag) {
    const uint32_t r = blockIdx.x * kThreads + threadIdx.x;
    if (r < R) flag[r] = (rowf[r] & 1u) ? 1u : 0u;
}
// kept reps -> the next state's first rows (distinct already), and into the hash table
__global__ __launch_bounds__(kThreads) void k_ls_rep_keep(int D, uint32_t R, const uint32_t *__restrict__ flag,
                                                          const uint32_t *__restrict__ pos,
                                                          const double *__restrict__ qrows,
                                                          const int32_t *__restrict__ qkey,
                                                          const int64_t *__restrict__ qw, double *__restrict__ rows2,
                                                          int32_t *__restrict__ key2, int64_t *__restrict__ w2,
                                                          unsigned long long *__restrict__ table, uint32_t hmask) {
    const uint32_t r = blockIdx.x * kThreads + threadIdx.x;
    if (r >= R || !flag[r]) return;
    const uint32_t o = pos[r];
    const double *src = qrows + (size_t)r * D;
    for (int d = 0; d < D; d++) rows2[(size_t)o * D + d] = src[d];
    key2[o] = qkey[r];
    w2[o] = qw[r];
    const uint32_t h = row_hash(src, D, qkey[r]);
    const unsigned long long v = ((unsigned long long)h << 32) | o;
    for (uint32_t s = h & hmask;; s = (s + 1) & hmask)
        if (atomicCAS(&table[s], kHashEmpty, v) == kHashEmpty) break;
}
// the next rep count starts at the kept reps' count; the hole count (ctr[2]) at zero
__global__ void k_ls_set_ctr(const uint32_t *__restrict__ kept, uint32_t *__restrict__ ctr) {
    if (threadIdx.x == 0) {
        ctr[0] = kept[0];
        ctr[2] = 0u;
    }
}
// new rows in L_k: the rep of their (key, row), created when absent.  A row that loses the race
// to publish a new vector keeps its reserved slot as an inert hole (key -1: dropped by the next
// query, weight 0).  Reps below *kept were published by an earlier kernel (plain loads see them);
// reps created by this kernel are read past the CU's L1.  Tuple counts: per wave for lanes that
// share a rep, then per workgroup in an LDS table over its grid-stride rows, one global atomic per
// (workgroup, rep) — the reference streams put most new local tuples on one vector.
constexpr int kLsSlots = 64;
__global__ __launch_bounds__(kThreads) void k_ls_new_reps(int D, uint32_t N, uint32_t R,
                                                          const uint8_t *__restrict__ rowf,
                                                          const double *__restrict__ qrows,
                                                          const int32_t *__restrict__ qkey,
                                                          double *__restrict__ rows2, int32_t *__restrict__ key2,
                                                          unsigned long long *__restrict__ w2,
                                                          unsigned long long *__restrict__ table, uint32_t hmask,
                                                          const uint32_t *__restrict__ kept,
                                                          uint32_t *__restrict__ ctr, uint32_t *__restrict__ holes,
                                                          uint32_t *__restrict__ newrep) {
    __shared__ uint32_t s_rep[kLsSlots];
    __shared__ unsigned long long s_cnt[kLsSlots];
    if (threadIdx.x < kLsSlots) {
        s_rep[threadIdx.x] = 0xffffffffu;
        s_cnt[threadIdx.x] = 0;
    }
    __syncthreads();
    const uint32_t base = __builtin_amdgcn_readfirstlane(kept[0]);
    const int lane = (int)(threadIdx.x & 63);
    for (uint32_t i0 = blockIdx.x * kThreads; i0 < N; i0 += gridDim.x * kThreads) {   // block-uniform
    const uint32_t i = i0 + threadIdx.x;
    const bool local = i < N && (rowf[R + i] & 1u);
    const double *src = qrows + (size_t)(R + min(i, N - 1u)) * D;
    const int32_t k = local ? qkey[R + i] : 0;
    const uint32_t h = local ? row_hash(src, D, k) : 0u;
    auto lookup = [&]() -> uint32_t {
        uint32_t mine = 0xffffffffu, rep = 0xffffffffu;   // reserved rep slot (written before publishing)
        for (uint32_t s = h & hmask;; s = (s + 1) & hmask) {
            unsigned long long cur = table[s];
            if (cur == kHashEmpty) {
                if (mine == 0xffffffffu) {
                    mine = atomicAdd(ctr, 1u);
                    for (int d = 0; d < D; d++) rows2[(size_t)mine * D + d] = src[d];
                    key2[mine] = k;
                    __threadfence();
                }
                cur = atomicCAS(&table[s], kHashEmpty, ((unsigned long long)h << 32) | mine);
                if (cur == kHashEmpty) {
                    rep = mine;
                    break;
                }
            }
            if ((uint32_t)(cur >> 32) == h) {
                const uint32_t r2 = (uint32_t)cur;
                bool eq;
                if (r2 < base) {                           // an earlier kernel's rep
                    eq = key2[r2] == k;
                    for (int d = 0; d < D; d++)
                        eq &= __double_as_longlong(rows2[(size_t)r2 * D + d]) == __double_as_longlong(src[d]);
                } else {
                    eq = __hip_atomic_load(key2 + r2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == k &&
                         same_row(rows2 + (size_t)r2 * D, src, D);
                }
                if (eq) {
                    rep = r2;
                    break;
                }
            }
        }
        if (mine != 0xffffffffu && mine != rep) {   // lost the race: an inert hole, counted
            key2[mine] = -1;
            atomicAdd(holes, 1u);
        }
        return rep;
    };
    // duplicates first resolved inside the wave: up to two leaders look their row up and every lane
    // holding the same (key, row) takes the leader's rep, so a vector repeated across the stream (the
    // zero vector of the reference streams) costs one table probe per wave, not one per tuple on
    // the same table slot
    uint32_t rep = 0xffffffffu;
    bool done = !local;
    uint64_t pend = __ballot(local);
    for (int round = 0; round < 2 && pend; round++) {
        const int leader = __ffsll((unsigned long long)pend) - 1;
        bool same = !done && h == (uint32_t)__shfl((int)h, leader, 64) && k == __shfl(k, leader, 64);
        for (int d = 0; d < D; d++) {
            const long long x = __double_as_longlong(src[d]);   // bits: the table's notion of one vector
            same &= __shfl(x, leader, 64) == x;
        }
        uint32_t r = 0;
        if (lane == leader) r = lookup();
        r = (uint32_t)__shfl((int)r, leader, 64);
        if (same) {
            rep = r;
            done = true;
        }
        pend = __ballot(!done);
    }
    if (!done) rep = lookup();
    if (local) newrep[i] = rep;
    // tuple counts: per group of lanes sharing a rep, into the workgroup's table (or global)
    uint64_t pw = __ballot(local);
    while (pw) {
        const int leader = __ffsll((unsigned long long)pw) - 1;
        const uint32_t r0 = __shfl(rep, leader, 64);
        const uint64_t same = __ballot(local && rep == r0);
        if (lane == leader) {
            const uint32_t sl = r0 & (kLsSlots - 1);
            uint32_t cur = s_rep[sl];
            if (cur == 0xffffffffu) cur = atomicCAS(&s_rep[sl], 0xffffffffu, r0) == 0xffffffffu ? r0 : s_rep[sl];
            if (cur == r0) atomicAdd(&s_cnt[sl], (unsigned long long)__popcll(same));
            else atomicAdd(&w2[r0], (unsigned long long)__popcll(same));
        }
        pw &= ~same;
    }
    }                                                      // next rows of this workgroup
    __syncthreads();
    if (threadIdx.x < kLsSlots && s_rep[threadIdx.x] != 0xffffffffu)
        atomicAdd(&w2[s_rep[threadIdx.x]], s_cnt[threadIdx.x]);
}
// the next state's tuples: resident tuples of kept reps (rep renumbered), then the new local
// tuples with their reps, arrival order kept
__global__ __launch_bounds__(kThreads) void k_ls_tuples(uint32_t T, uint32_t N, uint32_t R,
                                                        const int64_t *__restrict__ tid,
                                                        const uint32_t *__restrict__ trep,
                                                        const int64_t *__restrict__ qids,
                                                        const uint32_t *__restrict__ rpos,
                                                        const uint32_t *__restrict__ newrep,
                                                        const uint32_t *__restrict__ flag,
                                                        const uint32_t *__restrict__ pos, int64_t *__restrict__ tid2,
                                                        uint32_t *__restrict__ trep2) {
    const uint32_t t = blockIdx.x * kThreads + threadIdx.x;
    if (t >= T + N || !flag[t]) return;
    const uint32_t o = pos[t];
    if (t < T) {
        tid2[o] = tid[t];
        trep2[o] = rpos[trep[t]];
    } else {
        tid2[o] = qids[R + (t - T)];
        trep2[o] = newrep[t - T];
    }
}
__global__ __launch_bounds__(kThreads) void k_ls_ones(int64_t *__restrict__ w, uint32_t n) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i < n) w[i] = 1;
}

inline unsigned nblk(size_t n) { return (unsigned)((n + kThreads - 1) / kThreads); }

}  // namespace
}  // namespace sky

// the landmark state and its query workspace (one set per stream)
struct sky_stream_landmark {
    sky::DevBuf qrows, qids, qkey, qw;      // [reps ; new rows]: capacity qcap rows
    sky::DevBuf tid, trep;                  // resident tuples (arrival order): capacity tcap
    sky::DevBuf rows2, key2, w2, tid2, trep2;   // the next state, swapped in after a query
    sky::DevBuf rowf, flag, pos, rflag, rpos, newrep, table, words, scratch;
    sky::DevBuf lb;                         // the query's one-pass scans' look-back words (scan_excl_u32_lb)
    const void *lb_at = nullptr;            // ... the buffer zeroed last, and the last scan's epoch
    uint32_t lb_epoch = 0;
    int64_t R = 0, N = 0, T = 0, holes = 0;
    int64_t qcap = 0, tcap = 0;
};

namespace {

using sky::DevBuf;

// the landmark's row buffers hold at least `rows` rows, its tuple buffers `tuples` tuples
// (both state sets, so a query's swap never allocates)
int lm_reserve(sky_stream *s, int64_t rows, int64_t tuples) {
    sky_stream_landmark &L = *s->lm;
    sky_ctx *c = s->ctx;
    const int D = c->D;
    if (rows > L.qcap) {
        int64_t cap = std::max<int64_t>(L.qcap, 1024);
        while (cap < rows) cap *= 2;
        ARG_CHECK(cap < (int64_t)0x7fffffffLL, "stream state too large");
        // keep [0, R + N) of the row-side buffers
        const int64_t used = L.R + L.N;
        DevBuf nr, ni, nk, nw;
        SKY_TRY(nr.ensure((size_t)cap * D * 8));
        SKY_TRY(ni.ensure((size_t)cap * 8));
        SKY_TRY(nk.ensure((size_t)cap * 4));
        SKY_TRY(nw.ensure((size_t)cap * 8));
        if (used) {
            HIP_TRY(hipMemcpyAsync(nr.p, L.qrows.p, (size_t)used * D * 8, hipMemcpyDeviceToDevice, c->st));
            HIP_TRY(hipMemcpyAsync(ni.p, L.qids.p, (size_t)used * 8, hipMemcpyDeviceToDevice, c->st));
            HIP_TRY(hipMemcpyAsync(nk.p, L.qkey.p, (size_t)used * 4, hipMemcpyDeviceToDevice, c->st));
            HIP_TRY(hipMemcpyAsync(nw.p, L.qw.p, (size_t)used * 8, hipMemcpyDeviceToDevice, c->st));
        }
        HIP_TRY(hipStreamSynchronize(c->st));
        L.qrows = std::move(nr);
        L.qids = std::move(ni);
        L.qkey = std::move(nk);
        L.qw = std::move(nw);
        SKY_TRY(L.rows2.ensure((size_t)cap * D * 8));
        SKY_TRY(L.key2.ensure((size_t)cap * 4));
        SKY_TRY(L.w2.ensure((size_t)cap * 8));
        SKY_TRY(L.rowf.ensure((size_t)cap));
        SKY_TRY(L.rflag.ensure((size_t)cap * 4));
        SKY_TRY(L.rpos.ensure((size_t)cap * 4 + 64));
        SKY_TRY(L.newrep.ensure((size_t)cap * 4));
        SKY_TRY(L.table.ensure((size_t)2 * cap * 8 * 2));
        L.qcap = cap;
    }
    if (tuples > L.tcap) {
        int64_t cap = std::max<int64_t>(L.tcap, 1024);
        while (cap < tuples) cap *= 2;
        ARG_CHECK(cap < (int64_t)0x7fffffffLL, "stream state too large");
        DevBuf ti, tr;
        SKY_TRY(ti.ensure((size_t)cap * 8));
        SKY_TRY(tr.ensure((size_t)cap * 4));
        if (L.T) {
            HIP_TRY(hipMemcpyAsync(ti.p, L.tid.p, (size_t)L.T * 8, hipMemcpyDeviceToDevice, c->st));
            HIP_TRY(hipMemcpyAsync(tr.p, L.trep.p, (size_t)L.T * 4, hipMemcpyDeviceToDevice, c->st));
        }
        HIP_TRY(hipStreamSynchronize(c->st));
        L.tid = std::move(ti);
        L.trep = std::move(tr);
        SKY_TRY(L.tid2.ensure((size_t)cap * 8));
        SKY_TRY(L.trep2.ensure((size_t)cap * 4));
        L.tcap = cap;
    }
    // the output / next-state scans run over [resident tuples ; new rows]
    const size_t tn = (size_t)std::max<int64_t>(L.tcap + L.qcap, 1);
    SKY_TRY(L.flag.ensure(tn * 4));
    SKY_TRY(L.pos.ensure(tn * 4 + 64));
    SKY_TRY(L.scratch.ensure(sky::scan_scratch_words(tn + 1) * 4 + 64));
    SKY_TRY(L.words.ensure(256));
    SKY_TRY(L.lb.ensure(sky::scan_lb_words(tn + 1) * 8));
    if (L.lb.p != L.lb_at) {                  // new words: zeroed (no epoch yet), the error word too
        HIP_TRY(hipMemsetAsync(L.lb.p, 0, L.lb.cap, c->st));
        HIP_TRY(hipMemsetAsync(L.words.as<uint32_t>() + 6, 0, 4, c->st));
        L.lb_at = L.lb.p;
        L.lb_epoch = 0;
    }
    return SKY_OK;
}

// the next one-pass scan's epoch on the landmark's look-back words (re-zeroed at the 30-bit wrap)
int lm_scan_epoch(sky_stream *s, uint32_t *epoch) {
    sky_stream_landmark &L = *s->lm;
    if (++L.lb_epoch >= (1u << 30)) {
        HIP_TRY(hipMemsetAsync(L.lb.p, 0, L.lb.cap, s->ctx->st));
        L.lb_epoch = 1;
    }
    *epoch = L.lb_epoch;
    return SKY_OK;
}

// the sliding window's ring: compact the live range to the front of the other buffer, growing both
int ring_reserve(sky_stream *s, int64_t extra) {
    sky_ctx *c = s->ctx;
    const int D = c->D;
    if (s->off + s->n + extra <= s->cap) return SKY_OK;
    int64_t want = s->n + extra;
    int64_t cap = std::max<int64_t>(s->cap, 1024);
    while (cap < want) cap *= 2;
    cap = std::max<int64_t>(cap, std::min<int64_t>(2 * s->window + extra, (int64_t)0x7ffffffe));
    ARG_CHECK(cap < (int64_t)0x7fffffffLL, "stream state too large");
    const int o = 1 - s->cur;
    if (cap > s->cap) {
        SKY_TRY(s->ids[o].ensure((size_t)cap * 8));
        SKY_TRY(s->rows[o].ensure((size_t)cap * D * 8));
    }
    if (s->n) {
        HIP_TRY(hipMemcpyAsync(s->ids[o].p, s->ids[s->cur].as<int64_t>() + s->off, (size_t)s->n * 8,
                               hipMemcpyDeviceToDevice, c->st));
        HIP_TRY(hipMemcpyAsync(s->rows[o].p, s->rows[s->cur].as<double>() + s->off * D, (size_t)s->n * D * 8,
                               hipMemcpyDeviceToDevice, c->st));
    }
    HIP_TRY(hipStreamSynchronize(c->st));
    if (cap > s->cap) {
        SKY_TRY(s->ids[s->cur].ensure((size_t)cap * 8));
        SKY_TRY(s->rows[s->cur].ensure((size_t)cap * D * 8));
        s->cap = cap;
    }
    s->cur = o;
    s->off = 0;
    return SKY_OK;
}

// NaN admission of rows just copied in: the batch is rejected whole (the state stays queryable)
int nan_check(sky_stream *s, const double *rows, int64_t n) {
    sky_ctx *c = s->ctx;
    SKY_TRY(s->nanflag.ensure(64));
    if (!s->nan_host) HIP_TRY(hipHostMalloc(&s->nan_host, 64, hipHostMallocDefault));
    HIP_TRY(hipMemsetAsync(s->nanflag.p, 0, 4, c->st));
    sky::launch_nan_any(rows, (size_t)n * c->D, s->nanflag.as<uint32_t>(), c->st);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(s->nan_host, s->nanflag.p, 4, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));   // also: the caller's host buffer is free
    if (*(volatile uint32_t *)s->nan_host) {
        set_error("a tuple value is NaN: the reference BNL result is order-dependent for NaN; batch rejected");
        return SKY_E_NAN;
    }
    return SKY_OK;
}

int stream_append(sky_stream *s, const int64_t *ids, const double *values, int64_t n, hipMemcpyKind kind) {
    GUARD_BEGIN
    ARG_CHECK(s && (n == 0 || (ids && values)), "null argument");
    ARG_CHECK(n >= 0, "negative n");
    if (n == 0) return SKY_OK;
    sky_ctx *c = s->ctx;
    SKY_TRY(bind(c));
    const int D = c->D;
    if (s->window == 0) {
        sky_stream_landmark &L = *s->lm;
        ARG_CHECK(L.R + L.N + n < (int64_t)0x7fffffffLL, "stream state too large");
        SKY_TRY(lm_reserve(s, L.R + L.N + n, L.T));
        const int64_t at = L.R + L.N;
        HIP_TRY(hipMemcpyAsync(L.qids.as<int64_t>() + at, ids, (size_t)n * 8, kind, c->st));
        HIP_TRY(hipMemcpyAsync(L.qrows.as<double>() + at * D, values, (size_t)n * D * 8, kind, c->st));
        sky::k_ls_ones<<<sky::nblk((size_t)n), sky::kThreads, 0, c->st>>>(L.qw.as<int64_t>() + at, (uint32_t)n);
        SKY_TRY(nan_check(s, L.qrows.as<double>() + at * D, n));
        L.N += n;
        s->n = L.T + L.N;
        s->appended += n;
        return SKY_OK;
    }
    const int64_t n_all = n;
    bool drop_resident = false;
    if (n >= s->window) {   // only the newest `window` tuples of this batch can stay
        ids += n - s->window;
        values += (n - s->window) * D;
        n = s->window;
        drop_resident = true;
    }
    SKY_TRY(ring_reserve(s, n));
    const int64_t at = s->off + s->n;
    HIP_TRY(hipMemcpyAsync(s->ids[s->cur].as<int64_t>() + at, ids, (size_t)n * 8, kind, c->st));
    HIP_TRY(hipMemcpyAsync(s->rows[s->cur].as<double>() + at * D, values, (size_t)n * D * 8, kind, c->st));
    SKY_TRY(nan_check(s, s->rows[s->cur].as<double>() + at * D, n));
    if (drop_resident) {
        s->off = at;
        s->n = 0;
    }
    s->n += n;
    s->appended += n_all;
    if (s->n > s->window) {   // expire the oldest tuples
        s->off += s->n - s->window;
        s->n = s->window;
    }
    return SKY_OK;
    GUARD_END
}

// the landmark query (see the file comment); *n_out = global skyline tuples
int lm_query(sky_stream *s, int64_t *d_ids_out, int32_t *d_origin_out, int64_t cap, int64_t *n_out) {
    sky_ctx *c = s->ctx;
    sky_stream_landmark &L = *s->lm;
    hipStream_t st = c->st;
    const int D = c->D;
    const uint32_t R = (uint32_t)L.R, N = (uint32_t)L.N, T = (uint32_t)L.T;
    SKY_TRY(lm_reserve(s, (int64_t)R + N, (int64_t)T + N));
    // 1. the new rows' partition keys
    if (N) sky::launch_keys(D, L.qrows.as<double>() + (size_t)R * D, N, c->kp(), L.qkey.as<int32_t>() + R, st);
    // 2. the pipeline over [reps ; new rows]
    PipeIn in;
    in.vals = L.qrows.as<double>();
    in.n = R + N;
    in.ids = nullptr;
    in.keys = L.qkey.as<int32_t>();
    in.weights = L.qw.as<int64_t>();
    in.global = true;
    in.K = c->Kq();
    in.row_flags = L.rowf.as<uint8_t>();    // the per-row fates from the run's own count pass
    c->shard_valid = false;
    if (c->profile >= 2) {
        if (!c->pt.ok) c->pt.init();
        c->pt.reset();
    }
    SKY_TRY(pipe_run(*c, c->main, in, c->profile >= 2 ? &c->pt : nullptr));
    store_stats(c, c->main);
    int64_t g = 0;
    for (int64_t x : c->surv) g += x;
    *n_out = g;
    // the per-row fates (bit 0: in L_k, bit 1: in G)
    int64_t sel = 0;
    if (R + N && !c->main.row_flags_done) {   // (the run's count pass wrote them: no pass of its own)
        SKY_TRY(pipe_output(*c, c->main, in, false, nullptr, nullptr, nullptr, 0, &sel, L.rowf.as<uint8_t>()));
    }
    uint32_t *w = L.words.as<uint32_t>();
    const uint32_t TN = T + N;
    // 3. the output in arrival order
    if (TN && (d_ids_out || d_origin_out)) {
        sky::k_ls_select<<<sky::nblk(TN), sky::kThreads, 0, st>>>(T, N, R, L.trep.as<uint32_t>(), L.rowf.as<uint8_t>(),
                                                                  2u, L.flag.as<uint32_t>());
        uint32_t ep = 0;
        SKY_TRY(lm_scan_epoch(s, &ep));
        sky::scan_excl_u32_lb(L.flag.as<uint32_t>(), L.pos.as<uint32_t>(), TN, w, L.lb.as<unsigned long long>(), ep,
                              w + 6, st);
        sky::k_ls_write_out<<<sky::nblk(TN), sky::kThreads, 0, st>>>(
            T, N, R, L.tid.as<int64_t>(), L.trep.as<uint32_t>(), L.qids.as<int64_t>(), L.qkey.as<int32_t>(),
            L.flag.as<uint32_t>(), L.pos.as<uint32_t>(), cap, d_ids_out, d_origin_out);
    }
    // 4. the next state
    const uint32_t hcap = [&] {
        uint32_t h = 1024;
        while (h < 2u * (R + N)) h <<= 1;
        return h;
    }();
    {                                       // the hash table all-ones, the next weights zero: one launch
        sky::FillSet fs;
        fs.add(L.table.p, (size_t)hcap * 8, 0xff);
        fs.add(L.w2.p, (size_t)(R + N) * 8, 0);
        HIP_TRY(fs.launch(st));
    }
    if (R) {
        sky::k_ls_rep_flag<<<sky::nblk(R), sky::kThreads, 0, st>>>(R, L.rowf.as<uint8_t>(), L.rflag.as<uint32_t>());
        uint32_t ep = 0;
        SKY_TRY(lm_scan_epoch(s, &ep));
        sky::scan_excl_u32_lb(L.rflag.as<uint32_t>(), L.rpos.as<uint32_t>(), R, w + 1, L.lb.as<unsigned long long>(), ep,
                              w + 6, st);
        sky::k_ls_rep_keep<<<sky::nblk(R), sky::kThreads, 0, st>>>(
            D, R, L.rflag.as<uint32_t>(), L.rpos.as<uint32_t>(), L.qrows.as<double>(), L.qkey.as<int32_t>(),
            L.qw.as<int64_t>(), L.rows2.as<double>(), L.key2.as<int32_t>(), L.w2.as<int64_t>(),
            L.table.as<unsigned long long>(), hcap - 1);
    } else {
        HIP_TRY(hipMemsetAsync(w + 1, 0, 4, st));
    }
    sky::k_ls_set_ctr<<<1, 64, 0, st>>>(w + 1, w + 2);
    if (N)
        sky::k_ls_new_reps<<<std::min<unsigned>(sky::nblk(N), 1024u), sky::kThreads, 0, st>>>(
            D, N, R, L.rowf.as<uint8_t>(), L.qrows.as<double>(), L.qkey.as<int32_t>(), L.rows2.as<double>(),
            L.key2.as<int32_t>(), L.w2.as<unsigned long long>(), L.table.as<unsigned long long>(), hcap - 1, w + 1,
            w + 2, w + 4, L.newrep.as<uint32_t>());
    if (TN) {
        sky::k_ls_select<<<sky::nblk(TN), sky::kThreads, 0, st>>>(T, N, R, L.trep.as<uint32_t>(), L.rowf.as<uint8_t>(),
                                                                  1u, L.flag.as<uint32_t>());
        uint32_t ep = 0;
        SKY_TRY(lm_scan_epoch(s, &ep));
        sky::scan_excl_u32_lb(L.flag.as<uint32_t>(), L.pos.as<uint32_t>(), TN, w + 3, L.lb.as<unsigned long long>(), ep,
                              w + 6, st);
        sky::k_ls_tuples<<<sky::nblk(TN), sky::kThreads, 0, st>>>(
            T, N, R, L.tid.as<int64_t>(), L.trep.as<uint32_t>(), L.qids.as<int64_t>(), L.rpos.as<uint32_t>(),
            L.newrep.as<uint32_t>(), L.flag.as<uint32_t>(), L.pos.as<uint32_t>(), L.tid2.as<int64_t>(),
            L.trep2.as<uint32_t>());
    } else {
        HIP_TRY(hipMemsetAsync(w + 3, 0, 4, st));
    }
    HIP_TRY(hipGetLastError());
    uint32_t h[8] = {};
    c->host_syncs++;
    HIP_TRY(hipMemcpyAsync(h, w, 32, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (h[6]) {                             // a one-pass scan's look-back ran out of spins: no result
        HIP_TRY(hipMemsetAsync(w + 6, 0, 4, st));
        set_error("a look-back (stream scan) exceeded its spin bound");
        return SKY_E_HIP;
    }
    // swap in the next state: reps (with h[4] holes) [0, h[2]), tuples [0, h[3]), no new rows
    std::swap(L.qrows, L.rows2);
    std::swap(L.qkey, L.key2);
    std::swap(L.qw, L.w2);
    std::swap(L.tid, L.tid2);
    std::swap(L.trep, L.trep2);
    L.R = h[2];
    L.holes = N ? (int64_t)h[4] : 0;        // the race losers of k_ls_new_reps (w[4] is zeroed with w[2])
    L.N = 0;
    L.T = h[3];
    s->n = L.T;
    return SKY_OK;
}

int stream_query(sky_stream *s, int64_t *d_ids_out, int32_t *d_origin_out, int64_t cap, int64_t *n_out) {
    sky_ctx *c = s->ctx;
    if (s->window == 0) {
        SKY_TRY(lm_query(s, d_ids_out, d_origin_out, cap, n_out));
        HIP_TRY(hipGetLastError());
        finish_profile(c);
        return SKY_OK;
    }
    const int D = c->D;
    PipeIn in;
    in.vals = s->rows[s->cur].as<double>() + s->off * D;
    in.ids = s->ids[s->cur].as<int64_t>() + s->off;
    in.n = (uint32_t)s->n;
    in.global = true;
    in.K = c->Kq();
    in.out_ids = d_ids_out;
    in.out_org = d_origin_out;
    in.out_cap = cap;
    c->shard_valid = false;
    if (c->profile >= 2) {
        if (!c->pt.ok) c->pt.init();
        c->pt.reset();
    }
    SKY_TRY(pipe_run(*c, c->main, in, c->profile >= 2 ? &c->pt : nullptr));
    store_stats(c, c->main);
    SKY_TRY(pipe_output(*c, c->main, in, false, d_ids_out, d_origin_out, nullptr, cap, n_out, nullptr));
    HIP_TRY(hipGetLastError());
    finish_profile(c);
    return SKY_OK;
}

// a result copy still in flight (sky_stream_query_async): wait for it on the host
int stream_drain(sky_stream *s, double *copy_ms) {
    if (copy_ms) *copy_ms = 0.0;
    if (!s->copy_pending) return SKY_OK;
    s->copy_pending = false;
    HIP_TRY(hipEventSynchronize(s->ev_done));
    if (copy_ms) {
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, s->ev_ready, s->ev_done));
        *copy_ms = ms;
    }
    return SKY_OK;
}

}  // namespace

sky_stream::~sky_stream() {
    delete lm;
    if (ev_ready) hipEventDestroy(ev_ready);
    if (ev_done) hipEventDestroy(ev_done);
    if (cst) hipStreamDestroy(cst);
}

extern "C" {

int sky_stream_create(sky_ctx *c, int64_t window, sky_stream **out) {
    GUARD_BEGIN
    ARG_CHECK(c && out, "null argument");
    ARG_CHECK(window >= 0 && window < (int64_t)0x3fffffffLL, "window out of range");
    sky_stream *s = new sky_stream();
    s->ctx = c;
    s->window = window;
    if (window == 0) s->lm = new sky_stream_landmark();
    *out = s;
    return SKY_OK;
    GUARD_END
}
int sky_stream_destroy(sky_stream *s) {
    if (!s) return SKY_OK;
    hipSetDevice(s->ctx->dev);
    hipStreamSynchronize(s->ctx->st);
    stream_drain(s, nullptr);
    if (s->nan_host) hipHostFree(s->nan_host);
    delete s;
    return SKY_OK;
}
int sky_stream_append(sky_stream *s, const int64_t *ids, const double *values, int64_t n) {
    return stream_append(s, ids, values, n, hipMemcpyHostToDevice);
}
int sky_stream_append_dev(sky_stream *s, const int64_t *d_ids, const double *d_values, int64_t n) {
    return stream_append(s, d_ids, d_values, n, hipMemcpyDeviceToDevice);
}
int sky_stream_reserve(sky_stream *s, int64_t tuples) {
    GUARD_BEGIN
    ARG_CHECK(s, "null stream");
    ARG_CHECK(tuples >= 0 && tuples < (int64_t)0x3fffffffLL, "tuples out of range");
    sky_ctx *c = s->ctx;
    SKY_TRY(bind(c));
    SKY_TRY(stream_drain(s, nullptr));      // a result copy in flight reads out_ids / out_org
    const size_t m = (size_t)std::max<int64_t>(tuples, 1);
    if (s->window == 0) {
        // rows: at most every appended tuple between two queries plus the reps; tuples: all of them
        SKY_TRY(lm_reserve(s, tuples, tuples));
    } else {
        if (tuples > s->n) SKY_TRY(ring_reserve(s, tuples - s->n));
    }
    SKY_TRY(s->out_ids.ensure(m * 8));
    SKY_TRY(s->out_org.ensure(m * 4));
    SKY_TRY(s->nanflag.ensure(64));
    if (!s->nan_host) HIP_TRY(hipHostMalloc(&s->nan_host, 64, hipHostMallocDefault));
    SKY_TRY(pipe_reserve(*c, c->main, (uint32_t)m));
    HIP_TRY(hipStreamSynchronize(c->st));
    return SKY_OK;
    GUARD_END
}
int sky_stream_size(sky_stream *s, int64_t *resident, int64_t *appended) {
    ARG_CHECK(s, "null stream");
    if (resident) *resident = s->n;
    if (appended) *appended = s->appended;
    return SKY_OK;
}
int sky_stream_vectors(sky_stream *s, int64_t *vectors) {
    ARG_CHECK(s && vectors, "null argument");
    // the rows the next query runs over: the landmark's distinct vectors + the rows appended
    // since (less the inert holes), or the sliding window's tuples
    *vectors = s->window == 0 ? s->lm->R - s->lm->holes + s->lm->N : s->n;
    return SKY_OK;
}
int sky_stream_query_dev(sky_stream *s, int64_t *d_ids_out, int32_t *d_origin_out, int64_t cap, int64_t *n_out) {
    GUARD_BEGIN
    ARG_CHECK(s && n_out, "null argument");
    SKY_TRY(bind(s->ctx));
    SKY_TRY(stream_drain(s, nullptr));
    SKY_TRY(stream_query(s, d_ids_out, d_origin_out, cap, n_out));
    HIP_TRY(hipStreamSynchronize(s->ctx->st));
    if (*n_out > cap && (d_ids_out || d_origin_out)) {
        set_error("output capacity too small");
        return SKY_E_CAPACITY;
    }
    return SKY_OK;
    GUARD_END
}
int sky_stream_query(sky_stream *s, int64_t *ids_out, int32_t *origin_out, int64_t cap, int64_t *n_out) {
    GUARD_BEGIN
    ARG_CHECK(s && n_out, "null argument");
    sky_ctx *c = s->ctx;
    SKY_TRY(bind(c));
    SKY_TRY(stream_drain(s, nullptr));
    const size_t m = (size_t)std::max<int64_t>(s->n, 1);
    SKY_TRY(s->out_ids.ensure(m * 8));
    SKY_TRY(s->out_org.ensure(m * 4));
    int64_t g = 0;
    SKY_TRY(stream_query(s, s->out_ids.as<int64_t>(), s->out_org.as<int32_t>(), (int64_t)m, &g));
    *n_out = g;
    if (g > cap && (ids_out || origin_out)) {
        HIP_TRY(hipStreamSynchronize(c->st));
        set_error("output capacity too small");
        return SKY_E_CAPACITY;
    }
    if (g && ids_out) HIP_TRY(hipMemcpyAsync(ids_out, s->out_ids.p, (size_t)g * 8, hipMemcpyDeviceToHost, c->st));
    if (g && origin_out)
        HIP_TRY(hipMemcpyAsync(origin_out, s->out_org.p, (size_t)g * 4, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    return SKY_OK;
    GUARD_END
}

int sky_stream_query_async(sky_stream *s, int64_t *ids_out, int32_t *origin_out, int64_t cap, int64_t *n_out) {
    GUARD_BEGIN
    ARG_CHECK(s && n_out, "null argument");
    sky_ctx *c = s->ctx;
    SKY_TRY(bind(c));
    SKY_TRY(stream_drain(s, nullptr));      // the last result copy reads the staging buffers
    if (!s->cst) {
        HIP_TRY(hipStreamCreateWithFlags(&s->cst, hipStreamNonBlocking));
        HIP_TRY(hipEventCreate(&s->ev_ready));
        HIP_TRY(hipEventCreate(&s->ev_done));
    }
    const size_t m = (size_t)std::max<int64_t>(s->n, 1);
    SKY_TRY(s->out_ids.ensure(m * 8));
    SKY_TRY(s->out_org.ensure(m * 4));
    int64_t g = 0;
    // the query ends with its own read (the integers, the next state's counts): when it returns,
    // *n_out and sky_global_stats hold the reference's result (FlinkSkyline.java:593-608)
    SKY_TRY(stream_query(s, s->out_ids.as<int64_t>(), s->out_org.as<int32_t>(), (int64_t)m, &g));
    *n_out = g;
    if (g > cap && (ids_out || origin_out)) {
        HIP_TRY(hipStreamSynchronize(c->st));
        set_error("output capacity too small");
        return SKY_E_CAPACITY;
    }
    HIP_TRY(hipEventRecord(s->ev_ready, c->st));
    HIP_TRY(hipStreamWaitEvent(s->cst, s->ev_ready, 0));
    if (g && ids_out) HIP_TRY(hipMemcpyAsync(ids_out, s->out_ids.p, (size_t)g * 8, hipMemcpyDeviceToHost, s->cst));
    if (g && origin_out)
        HIP_TRY(hipMemcpyAsync(origin_out, s->out_org.p, (size_t)g * 4, hipMemcpyDeviceToHost, s->cst));
    HIP_TRY(hipEventRecord(s->ev_done, s->cst));
    s->copy_pending = true;
    return SKY_OK;
    GUARD_END
}

int sky_stream_wait(sky_stream *s, double *copy_ms) {
    GUARD_BEGIN
    ARG_CHECK(s, "null stream");
    SKY_TRY(bind(s->ctx));
    SKY_TRY(stream_drain(s, copy_ms));
    return SKY_OK;
    GUARD_END
}

}  // extern "C"
