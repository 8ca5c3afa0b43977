// k_dom16.hip — the dominance-compare-bound stage for integer-valued streams.
//
// When every candidate value is an integer in [0, 65535] (every reference stream:
// integers in [0, domain], python/unified_producer.py:50-123) a row packs into
// W = ceil(D/8)*4 u32 words of two u16 halves each, and
//     x <= y in every dimension  <=>  OR_w  sat_u16(x_w - y_w)  == 0
// costs W v_pk_sub_u16 (clamp) + an OR tree + one v_cmp per pair: 7 VALU ops for
// 8 dimensions, i.e. more than one compare per VALU lane-op.  The compared rows
// are distinct vectors (representatives), for which "x <= y everywhere, x != y"
// (ServiceTuple.java:67-77) reduces to "x <= y everywhere" for x at another
// position.  x rows are wave-uniform (scalar loads, no LDS), y rows sit in VGPRs
// (PPT per lane), dominated flags accumulate as 64-bit lane masks in SGPRs.
//
// One SFS round over the active segments (sorted by strictly monotone score, so
// a dominator always sits at an earlier position):
//   k_dom16 (tri)   X = the first B candidates of each segment: every y in X vs
//                   the x in X before it           -> dead[y]
//   k_xcompact16    X' = X minus dead: confirmed skyline members -> alive, packed
//                   into xbuf[seg]; every X position is then marked dead
//   k_dom16 (rest)  every remaining y of the segment vs X'       -> dead[y]
//   keep = !dead -> exclusive scan -> k_move16 (next round's layout)
// Work items are (segment, 64*PPT y, <= kDomTx x) tiles, one wave each; a tile
// whose y are all dead skips its remaining x.
#include <cstdlib>
#include "knobs.h"

#include "sky_internal.h"

namespace sky {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t satsub_u16x2(uint32_t x, uint32_t y) {
    return __builtin_bit_cast(uint32_t,
                              __builtin_elementwise_sub_sat(__builtin_bit_cast(u16x2, x), __builtin_bit_cast(u16x2, y)));
}

template <int W>
__device__ __forceinline__ bool le_all16(const uint32_t *x, const uint32_t (&y)[W]) {
    uint32_t r = 0;
#pragma unroll
    for (int w = 0; w < W; w++) r |= satsub_u16x2(x[w], y[w]);
    return r == 0u;
}

// ---- packing ------------------------------------------------------------------
template <int D, int W>
__global__ __launch_bounds__(kThreads) void k_pack16(const float *__restrict__ rows, uint32_t m,
                                                     const uint32_t *__restrict__ idx, uint32_t *__restrict__ out) {
    constexpr int DP = padded_dims<float>(D);
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= m) return;
    const float *r = rows + (size_t)(idx ? idx[j] : j) * DP;
    uint32_t w[W];
#pragma unroll
    for (int q = 0; q < W; q++) {
        const uint32_t lo = 2 * q < D ? (uint32_t)r[2 * q] : 0u;
        const uint32_t hi = 2 * q + 1 < D ? (uint32_t)r[2 * q + 1] : 0u;
        w[q] = lo | (hi << 16);
    }
    uint4 *o = reinterpret_cast<uint4 *>(out + (size_t)j * W);
#pragma unroll
    for (int q = 0; q < W / 4; q++) o[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}

// ---- the pair-test kernel ------------------------------------------------------
// x row q of the scan against every lane's PPT rows; DIAG: only x at an earlier
// position than y (t = position(x) - y0 - 64p; lanes > t)
template <int W, int PPT, bool DIAG>
__device__ __forceinline__ void dom_row(const uint32_t (&x)[W], int32_t t0, const uint32_t (&y)[PPT][W],
                                        uint64_t (&dom)[PPT]) {
#pragma unroll
    for (int p = 0; p < PPT; p++) {
        uint64_t m = __ballot(le_all16<W>(x, y[p]));
        if constexpr (DIAG) {
            const int32_t t = t0 - p * 64;
            m &= t < 0 ? ~0ull : (t >= 63 ? 0ull : (~0ull << (t + 1)));
        }
        dom[p] |= m;
    }
}

// x row vs every lane's PPT rows, VALU only: acc[p] = min over x of OR_w sat(x_w - y_w),
// so y is dominated iff acc[p] == 0 (no VALU -> SGPR -> SALU dependency per pair)
template <int W, int PPT>
__device__ __forceinline__ void dom_row_acc(const uint32_t (&x)[W], const uint32_t (&y)[PPT][W],
                                            uint32_t (&acc)[PPT]) {
#pragma unroll
    for (int p = 0; p < PPT; p++) {
        uint32_t r = 0;
#pragma unroll
        for (int w = 0; w < W; w++) r |= satsub_u16x2(x[w], y[p][w]);
        acc[p] = acc[p] < r ? acc[p] : r;
    }
}

// Scan nx x rows in batches of R, the next batch's scalar loads in flight while the
// current batch is compared (a lone wave otherwise waits a K$/L2 round trip per batch).
template <int W, int PPT, int R, bool DIAG>
__device__ __forceinline__ void dom_scan(const uint32_t *__restrict__ xs, uint32_t nx, int32_t tbase,
                                         const uint32_t (&y)[PPT][W], uint64_t (&dom)[PPT]) {
    uint32_t acc[PPT];
#pragma unroll
    for (int p = 0; p < PPT; p++) acc[p] = 0xffffffffu;
    const uint32_t nb = nx / R;                              // full batches
    uint32_t xn[R][W];
    if (nb) {
#pragma unroll
        for (int q = 0; q < R; q++)
#pragma unroll
            for (int w = 0; w < W; w++) xn[q][w] = xs[(size_t)q * W + w];
    }
    for (uint32_t b = 0; b < nb; b++) {
        uint32_t x[R][W];
#pragma unroll
        for (int q = 0; q < R; q++)
#pragma unroll
            for (int w = 0; w < W; w++) x[q][w] = xn[q][w];
        if (b + 1 < nb) {
#pragma unroll
            for (int q = 0; q < R; q++)
#pragma unroll
                for (int w = 0; w < W; w++) xn[q][w] = xs[(size_t)((b + 1) * R + q) * W + w];
        }
#pragma unroll
        for (int q = 0; q < R; q++) {
            if constexpr (DIAG) dom_row<W, PPT, true>(x[q], tbase + (int32_t)(b * R + q), y, dom);
            else dom_row_acc<W, PPT>(x[q], y, acc);
        }
        if (((b + 1) * R) % 16u == 0u || b + 1 == nb) {
            uint64_t all = ~0ull;
#pragma unroll
            for (int p = 0; p < PPT; p++) {
                if constexpr (!DIAG) dom[p] |= __ballot(acc[p] == 0u);
                all &= dom[p];
            }
            if (all == ~0ull) return;
        }
    }
    for (uint32_t i = nb * R; i < nx; i++) {
        uint32_t x[W];
#pragma unroll
        for (int w = 0; w < W; w++) x[w] = xs[(size_t)i * W + w];
        if constexpr (DIAG) dom_row<W, PPT, true>(x, tbase + (int32_t)i, y, dom);
        else dom_row_acc<W, PPT>(x, y, acc);
    }
    if constexpr (!DIAG) {
#pragma unroll
        for (int p = 0; p < PPT; p++) dom[p] |= __ballot(acc[p] == 0u);
    }
}

// R == 64: the x rows come in vector batches of 64 (lane l loads row b0 + l, the
// next batch in flight while the current one is compared) and are broadcast to
// SGPRs by v_readlane: one L2 round trip per 64 rows instead of per R rows, which
// is what bounds a lone wave's scan (small rounds, few items: latency, not VALU).
template <int W>
__device__ __forceinline__ void load_xrow(const uint32_t *__restrict__ xs, uint32_t row, uint32_t (&x)[W]) {
    const uint4 *src = reinterpret_cast<const uint4 *>(xs + (size_t)row * W);
#pragma unroll
    for (int v = 0; v < W / 4; v++) {
        const uint4 t = src[v];
        x[4 * v] = t.x; x[4 * v + 1] = t.y; x[4 * v + 2] = t.z; x[4 * v + 3] = t.w;
    }
}

template <int W, int PPT, bool DIAG>
__device__ __forceinline__ void dom_scan_v(const uint32_t *__restrict__ xs, uint32_t nx, int32_t tbase,
                                           const uint32_t (&y)[PPT][W], uint64_t (&dom)[PPT]) {
    uint32_t acc[PPT];
#pragma unroll
    for (int p = 0; p < PPT; p++) acc[p] = 0xffffffffu;
    const uint32_t lane = threadIdx.x & 63, last = nx - 1;
    uint32_t xa[W], xb[W];
    load_xrow<W>(xs, min(lane, last), xa);
    for (uint32_t b0 = 0; b0 < nx; b0 += 64) {
        load_xrow<W>(xs, min(b0 + 64 + lane, last), xb);           // unconditional: clamped past the end
        const uint32_t cnt = min(64u, nx - b0);
        for (uint32_t q = 0; q < cnt; q++) {
            uint32_t x[W];
#pragma unroll
            for (int w = 0; w < W; w++) x[w] = __builtin_amdgcn_readlane(xa[w], q);
            if constexpr (DIAG) dom_row<W, PPT, true>(x, tbase + (int32_t)(b0 + q), y, dom);
            else dom_row_acc<W, PPT>(x, y, acc);
            if ((q & 15u) == 15u) {
                uint64_t all = ~0ull;
#pragma unroll
                for (int p = 0; p < PPT; p++) {
                    if constexpr (!DIAG) dom[p] |= __ballot(acc[p] == 0u);
                    all &= dom[p];
                }
                if (all == ~0ull) return;
            }
        }
#pragma unroll
        for (int w = 0; w < W; w++) xa[w] = xb[w];
    }
    if constexpr (!DIAG) {
#pragma unroll
        for (int p = 0; p < PPT; p++) dom[p] |= __ballot(acc[p] == 0u);
    }
}

template <int W, int PPT, int R, bool DIAG>
__global__ __launch_bounds__(256, 8) void k_dom16(const uint32_t *__restrict__ rows, const uint32_t *__restrict__ xbuf,
                                               const uint32_t *__restrict__ xcnt, const DomItem *__restrict__ items,
                                               uint32_t nitems, uint32_t xcap, uint32_t *__restrict__ dead) {
    // one work item per wave (4 per workgroup): waves never synchronise
    const uint32_t wi = blockIdx.x * 4u + (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wi >= nitems) return;
    const DomItem it = items[wi];
    const int lane = threadIdx.x & 63;
    const uint32_t *xs;
    uint32_t nx = it.nx;
    if (it.flags & kDomRest) {
        const uint32_t c = xcnt[it.seg];
        if (it.x0 >= c) return;
        nx = c - it.x0 < nx ? c - it.x0 : nx;
        xs = xbuf + ((size_t)it.seg * xcap + it.x0) * W;
    } else {
        xs = rows + (size_t)it.x0 * W;
    }
    uint32_t y[PPT][W];
    uint64_t dom[PPT];
    uint64_t all = ~0ull;
    // every y row and dead flag loaded unconditionally (index clamped into the tile),
    // so the PPT loads are in flight together instead of one round trip each
    uint32_t dflag[PPT];
#pragma unroll
    for (int p = 0; p < PPT; p++) {
        const uint32_t q = (uint32_t)(p * 64 + lane);
        const uint32_t j = it.y0 + (q < it.ny ? q : it.ny - 1);
        dflag[p] = dead[j];
        load_xrow<W>(rows, j, y[p]);
    }
#pragma unroll
    for (int p = 0; p < PPT; p++) {
        const bool valid = (uint32_t)(p * 64 + lane) < it.ny;
        dom[p] = __ballot(!valid || dflag[p] != 0u);
        all &= dom[p];
        if (!valid) {
#pragma unroll
            for (int w = 0; w < W; w++) y[p][w] = 0xffffffffu;
        }
    }
    if (all == ~0ull) return;
    if constexpr (DIAG) {
        // x before y0: plain rows; x in [y0, y0+ny): masked rows; x after: no dominator
        const int32_t t0 = (int32_t)it.x0 - (int32_t)it.y0;              // < 0: x starts before y0
        const uint32_t nplain = t0 < 0 ? ((uint32_t)(-t0) < nx ? (uint32_t)(-t0) : nx) : 0u;
        const int64_t xend = (int64_t)it.y0 + it.ny - it.x0;            // x index past the last y
        const uint32_t nlim = xend < (int64_t)nx ? (uint32_t)(xend > 0 ? xend : 0) : nx;
        if constexpr (R == 64) {
            if (nplain) dom_scan_v<W, PPT, false>(xs, nplain, 0, y, dom);
            if (nlim > nplain)
                dom_scan_v<W, PPT, true>(xs + (size_t)nplain * W, nlim - nplain, t0 + (int32_t)nplain, y, dom);
        } else {
            if (nplain) dom_scan<W, PPT, R, false>(xs, nplain, 0, y, dom);
            if (nlim > nplain)
                dom_scan<W, PPT, R, true>(xs + (size_t)nplain * W, nlim - nplain, t0 + (int32_t)nplain, y, dom);
        }
    } else if constexpr (R == 64) {
        dom_scan_v<W, PPT, false>(xs, nx, 0, y, dom);
    } else {
        dom_scan<W, PPT, R, false>(xs, nx, 0, y, dom);
    }
#pragma unroll
    for (int p = 0; p < PPT; p++) {
        const uint32_t q = (uint32_t)(p * 64 + lane);
        if (q < it.ny && ((dom[p] >> lane) & 1ull)) dead[it.y0 + q] = 1u;
    }
}

// ---- X' of each active segment ---------------------------------------------------
// One workgroup per active segment slot s: the live positions of X = [b, b+xk) are
// confirmed skyline members -> alive[idx], rows appended (position order) to
// xbuf[s]; xcnt[s] = |X'|; every position of X is then marked dead (it leaves the
// active set).
template <int W>
__global__ __launch_bounds__(kThreads) void k_xcompact16(const uint32_t *__restrict__ rows,
                                                         const uint32_t *__restrict__ idx,
                                                         const SfsSeg *__restrict__ xseg, uint32_t xcap,
                                                         uint32_t *__restrict__ dead, uint32_t *__restrict__ xbuf,
                                                         uint32_t *__restrict__ xcnt, uint8_t *__restrict__ alive) {
    __shared__ uint32_t s_w[kThreads / 64];
    const SfsSeg sg = xseg[blockIdx.x];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    uint32_t run = 0;
    for (uint32_t q0 = 0; q0 < sg.count; q0 += kThreads) {
        const uint32_t q = q0 + threadIdx.x;
        const bool in = q < sg.count;
        const uint32_t pos = sg.begin + q;
        const bool live = in && dead[pos] == 0u;
        const uint64_t b = __ballot(live);
        if (lane == 0) s_w[w] = __popcll(b);
        __syncthreads();
        uint32_t wb = 0, tot = 0;
#pragma unroll
        for (int i = 0; i < kThreads / 64; i++) { wb += i < w ? s_w[i] : 0u; tot += s_w[i]; }
        __syncthreads();
        if (live) {
            const uint32_t slot = run + wb + __popcll(b & lt);
            const uint4 *src = reinterpret_cast<const uint4 *>(rows + (size_t)pos * W);
            uint4 *dst = reinterpret_cast<uint4 *>(xbuf + ((size_t)blockIdx.x * xcap + slot) * W);
#pragma unroll
            for (int v = 0; v < W / 4; v++) dst[v] = src[v];
            alive[idx ? idx[pos] : pos] = 1;
        }
        if (in) dead[pos] = 1u;
        run += tot;
    }
    if (threadIdx.x == 0) xcnt[blockIdx.x] = run;
}

__global__ __launch_bounds__(kThreads) void k_keep16(const uint32_t *__restrict__ dead, uint32_t n,
                                                     uint32_t *__restrict__ keep) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j < n) keep[j] = dead[j] ? 0u : 1u;
}

template <int W>
__global__ __launch_bounds__(kThreads) void k_move16(const uint32_t *__restrict__ keep,
                                                     const uint32_t *__restrict__ scan, uint32_t n,
                                                     const uint32_t *__restrict__ idx, const uint32_t *__restrict__ rows,
                                                     uint32_t *__restrict__ idx_out, uint32_t *__restrict__ rows_out) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= n || !keep[j]) return;
    const uint32_t d = scan[j];
    idx_out[d] = idx ? idx[j] : j;
    const uint4 *src = reinterpret_cast<const uint4 *>(rows + (size_t)j * W);
    uint4 *dst = reinterpret_cast<uint4 *>(rows_out + (size_t)d * W);
#pragma unroll
    for (int v = 0; v < W / 4; v++) dst[v] = src[v];
}

__global__ __launch_bounds__(kThreads) void k_gather_u32(const uint32_t *__restrict__ src,
                                                         const uint32_t *__restrict__ at, uint32_t n,
                                                         uint32_t *__restrict__ out) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j < n) out[j] = src[at[j]];
}

// ---- launchers ---------------------------------------------------------------------
static inline unsigned nb16(size_t n) { return (unsigned)((n + kThreads - 1) / kThreads); }

int dom16_words(int D) { return D <= 8 ? 4 : 8; }

void launch_pack16(int D, const float *rows, uint32_t m, const uint32_t *idx, uint32_t *out, hipStream_t st) {
    if (!m) return;
    if (D <= 8) { SKY_DISPATCH_D(D, (k_pack16<DD, 4><<<nb16(m), kThreads, 0, st>>>(rows, m, idx, out))); }
    else { SKY_DISPATCH_D(D, (k_pack16<DD, 8><<<nb16(m), kThreads, 0, st>>>(rows, m, idx, out))); }
}

// SKY_DOM_PPT in {4, 8} (y rows per lane of the rest tiles; tri tiles use 1), SKY_DOM_R in {2, 4} (x rows per
// scalar-load batch) or 64 (vector batches + v_readlane): tuning knobs, defaults measured on the MI355X
static int env_int(const char *e, int dflt) {
    return e ? atoi(e) : dflt;
}
int dom16_ppt() {
    static int v = [] {
        const int p = env_int(SKY_MEASURE_ENV("SKY_DOM_PPT"), 4);
        return p == 8 ? 8 : 4;
    }();
    return v;
}
uint32_t dom16_tx() {                          // 0: adaptive (sfs_run16)
    const int t = env_int(SKY_MEASURE_ENV("SKY_DOM_TX"), 0);
    return t >= 64 && t <= 4096 ? (uint32_t)t : 0u;
}
static int dom16_r() {
    const int r = env_int(SKY_MEASURE_ENV("SKY_DOM_R"), 4);
    return r == 2 || r == 64 ? r : 4;
}

template <int W, int PPT, int R>
static void dom16_t(bool diag, const uint32_t *rows, const uint32_t *xbuf, const uint32_t *xcnt,
                    const DomItem *items, uint32_t nitems, uint32_t xcap, uint32_t *dead, hipStream_t st) {
    const unsigned g = (nitems + 3) / 4;
    if (diag) k_dom16<W, PPT, R, true><<<g, 256, 0, st>>>(rows, xbuf, xcnt, items, nitems, xcap, dead);
    else k_dom16<W, PPT, R, false><<<g, 256, 0, st>>>(rows, xbuf, xcnt, items, nitems, xcap, dead);
}
template <int W>
static void dom16_w(int ppt, bool diag, const uint32_t *rows, const uint32_t *xbuf, const uint32_t *xcnt,
                    const DomItem *items, uint32_t nitems, uint32_t xcap, uint32_t *dead, hipStream_t st) {
    const int r = dom16_r();
#define DOM16_CASE(P_, R_) \
    if (ppt == P_ && r == R_) { dom16_t<W, P_, R_>(diag, rows, xbuf, xcnt, items, nitems, xcap, dead, st); return; }
    DOM16_CASE(1, 2) DOM16_CASE(1, 4) DOM16_CASE(4, 2) DOM16_CASE(4, 4) DOM16_CASE(8, 2) DOM16_CASE(8, 4)
    DOM16_CASE(1, 64) DOM16_CASE(4, 64) DOM16_CASE(8, 64)
#undef DOM16_CASE
}

void launch_dom16(int W, int ppt, bool diag, const uint32_t *rows, const uint32_t *xbuf, const uint32_t *xcnt,
                  const DomItem *items, uint32_t nitems, uint32_t xcap, uint32_t *dead, hipStream_t st) {
    if (!nitems) return;
    if (W == 4) dom16_w<4>(ppt, diag, rows, xbuf, xcnt, items, nitems, xcap, dead, st);
    else dom16_w<8>(ppt, diag, rows, xbuf, xcnt, items, nitems, xcap, dead, st);
}

void launch_xcompact16(int W, const uint32_t *rows, const uint32_t *idx, const SfsSeg *xseg, uint32_t nslots,
                       uint32_t xcap, uint32_t *dead, uint32_t *xbuf, uint32_t *xcnt, uint8_t *alive, hipStream_t st) {
    if (!nslots) return;
    if (W == 4) k_xcompact16<4><<<nslots, kThreads, 0, st>>>(rows, idx, xseg, xcap, dead, xbuf, xcnt, alive);
    else k_xcompact16<8><<<nslots, kThreads, 0, st>>>(rows, idx, xseg, xcap, dead, xbuf, xcnt, alive);
}

void launch_keep16(const uint32_t *dead, uint32_t n, uint32_t *keep, hipStream_t st) {
    if (n) k_keep16<<<nb16(n), kThreads, 0, st>>>(dead, n, keep);
}

void launch_move16(int W, const uint32_t *keep, const uint32_t *scan, uint32_t n, const uint32_t *idx,
                   const uint32_t *rows, uint32_t *idx_out, uint32_t *rows_out, hipStream_t st) {
    if (!n) return;
    if (W == 4) k_move16<4><<<nb16(n), kThreads, 0, st>>>(keep, scan, n, idx, rows, idx_out, rows_out);
    else k_move16<8><<<nb16(n), kThreads, 0, st>>>(keep, scan, n, idx, rows, idx_out, rows_out);
}

void launch_gather_u32(const uint32_t *src, const uint32_t *at, uint32_t n, uint32_t *out, hipStream_t st) {
    if (n) k_gather_u32<<<nb16(n), kThreads, 0, st>>>(src, at, n, out);
}

}  // namespace sky
