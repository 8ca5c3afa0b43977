// k_sfs.hip — the dominance-compare-bound stage: a blocked, segmented SFS.
//
// Input: the distinct vectors (representatives) of every partition, sorted by
// (partition, monotone score).  A dominator always precedes what it dominates
// in that order (strict score when kFlagScoreTies is clear; equal-score runs are
// checked both ways otherwise), so per round and per partition:
//   k_block_sky    the next B candidates X are staged in LDS; each lane tests its
//                  candidate against the EARLIER ones of X (LDS broadcast reads,
//                  scalar VALU compares, wave-ballot early exit).  Survivors X' are
//                  confirmed skyline members.
//   k_filter_rest  every remaining candidate of the partition is tested against X'
//                  (X' in LDS, PPT candidates per lane in registers).
//   k_act_compact  order-preserving compaction of the survivors for the next round.
// The work is Σ_rounds |R|·|X'| pair tests of D compares each.
#include "sky_internal.h"
#include "sky_tail.h"

namespace sky {

template <typename T>
__device__ __forceinline__ uint32_t key_score(uint64_t k) { return (uint32_t)(k >> 24); }

template <typename T, int D, bool FULL>
__device__ __forceinline__ bool dom_test(const T *x, const T *y) {
    if constexpr (FULL) return dominates_full<D, T>(x, y);
    else return dominates_distinct<D, T>(x, y);
}

template <typename T, int D>
__device__ __forceinline__ void lds_row(const T *s, T (&v)[D]) {
#pragma unroll
    for (int d = 0; d < D; d++) v[d] = s[d];
}

// Round step 1, in parallel over (partition, slice of 256 candidates): the next
// B candidates X of each large partition are tested against their predecessors in
// X, streamed through LDS in tiles of TB rows; survivors are confirmed skyline
// members (alive) and flagged in xkeep for the filter step.
template <typename T, int D, bool FULL, bool TIES>
__global__ __launch_bounds__(kThreads) void k_block_sky(const T *__restrict__ rows, const uint64_t *__restrict__ key,
                                                        const uint32_t *__restrict__ act,
                                                        const SfsSeg *__restrict__ segs,
                                                        const uint32_t *__restrict__ seg_list, int B, int TB,
                                                        uint8_t *__restrict__ alive, uint8_t *__restrict__ xkeep) {
    constexpr int DP = padded_dims<T>(D);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T *s_x = reinterpret_cast<T *>(smem);                               // [TB][DP]
    const uint32_t k = seg_list[blockIdx.x];
    const SfsSeg sg = segs[k];
    const uint32_t xk = sg.count < (uint32_t)B ? sg.count : (uint32_t)B;
    const uint32_t jlo = blockIdx.y * kThreads;
    if (jlo >= xk) return;                                               // block-uniform
    const uint32_t jhi = xk - jlo < (uint32_t)kThreads ? xk : jlo + kThreads;
    const uint32_t j = jlo + threadIdx.x;
    const bool valid = j < jhi;
    T y[D];
    const uint32_t rj = valid ? act[sg.begin + j] : 0u;
#pragma unroll
    for (int d = 0; d < D; d++) y[d] = valid ? rows[(size_t)rj * DP + d] : T(0);
    bool dom = false;
    const uint32_t wlast = jlo + (threadIdx.x | 63u);                  // largest j of this wave
    for (uint32_t c0 = 0; c0 < jhi; c0 += TB) {
        const uint32_t cn = jhi - c0 < (uint32_t)TB ? jhi - c0 : (uint32_t)TB;
        for (uint32_t q = threadIdx.x; q < cn * DP; q += kThreads) {
            const uint32_t row = q / DP, d = q - row * DP;
            s_x[q] = rows[(size_t)act[sg.begin + c0 + row] * DP + d];
        }
        __syncthreads();
        const uint32_t iend = wlast < c0 + cn ? (wlast > c0 ? wlast - c0 : 0u) : cn;
        for (uint32_t i = 0; i < iend; i++) {
            if ((i & 15u) == 0u && __ballot(valid && !dom) == 0ull) break;
            T x[D];
            lds_row<T, D>(s_x + (size_t)i * DP, x);
            dom |= (c0 + i < j) && dom_test<T, D, FULL>(x, y);
        }
        if (!__syncthreads_or(valid && !dom)) break;
    }
    if constexpr (TIES) {
        // equal scores can dominate either way: also test later members of X with the
        // same score and, at the chunk's end, the head of the remaining candidates
        if (valid && !dom) {
            const uint32_t sj = key_score<T>(key[rj]);
            for (uint32_t q = j + 1; q < sg.count && !dom; q++) {
                const uint32_t r = act[sg.begin + q];
                if (key_score<T>(key[r]) != sj) break;
                T x[D];
#pragma unroll
                for (int d = 0; d < D; d++) x[d] = rows[(size_t)r * DP + d];
                dom = dom_test<T, D, true>(x, y);
            }
        }
    }
    if (valid) {
        xkeep[(size_t)k * B + j] = dom ? 0 : 1;
        if (!dom) alive[rj] = 1;
    }
}

// Whole SFS of one small partition in ONE workgroup, no host round trips: the
// partition's representatives are consumed in chunks X of B (sorted order); each
// chunk is tested against the confirmed skyline C so far (streamed through LDS in
// tiles of B) and against its own earlier members; survivors are appended to C
// (a per-partition region of `conf`).  Same result as the round-based path.
template <typename T, int D, bool FULL, bool TIES>
__global__ __launch_bounds__(kThreads) void k_sfs_small(const T *__restrict__ rows, const uint64_t *__restrict__ key,
                                                        const SfsSeg *__restrict__ segs,
                                                        const uint32_t *__restrict__ seg_list, int B,
                                                        uint8_t *__restrict__ alive, T *__restrict__ conf) {
    constexpr int DP = padded_dims<T>(D);
    constexpr int PPT = 2;                                              // B <= 512 = 256 x 2
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T *s_x = reinterpret_cast<T *>(smem);                               // [B][DP]
    T *s_c = s_x + (size_t)B * DP;                                      // [B][DP]
    uint32_t *s_sc = reinterpret_cast<uint32_t *>(s_c + (size_t)B * DP);  // [B]
    uint32_t *s_keep = s_sc + B;                                         // [B]
    __shared__ uint32_t s_w[kThreads / 64];
    const SfsSeg sg = segs[seg_list[blockIdx.x]];
    const uint32_t base = sg.begin, cnt = sg.count;
    T *C = conf + (size_t)base * DP;
    uint32_t nconf = 0;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (uint32_t x0 = 0; x0 < cnt; x0 += B) {
        const uint32_t xk = cnt - x0 < (uint32_t)B ? cnt - x0 : (uint32_t)B;
        const T *src = rows + (size_t)(base + x0) * DP;
        for (uint32_t q = threadIdx.x; q < xk * DP; q += kThreads) s_x[q] = src[q];
        for (uint32_t q = threadIdx.x; q < xk; q += kThreads) s_sc[q] = key_score<T>(key[base + x0 + q]);
        __syncthreads();
        T y[PPT][D];
        bool valid[PPT], dom[PPT];
#pragma unroll
        for (int p = 0; p < PPT; p++) {
            const uint32_t j = threadIdx.x + p * kThreads;
            valid[p] = j < xk;
            dom[p] = false;
#pragma unroll
            for (int d = 0; d < D; d++) y[p][d] = valid[p] ? s_x[(size_t)j * DP + d] : T(0);
        }
        // 1) against the confirmed skyline, tile by tile
        for (uint32_t c0 = 0; c0 < nconf; c0 += B) {
            const uint32_t ck = nconf - c0 < (uint32_t)B ? nconf - c0 : (uint32_t)B;
            for (uint32_t q = threadIdx.x; q < ck * DP; q += kThreads) s_c[q] = C[(size_t)c0 * DP + q];
            __syncthreads();
            bool live = false;
#pragma unroll
            for (int p = 0; p < PPT; p++) live |= valid[p] && !dom[p];
            if (__ballot(live) != 0ull) {
                for (uint32_t i = 0; i < ck; i++) {
                    T x[D];
                    lds_row<T, D>(s_c + (size_t)i * DP, x);
#pragma unroll
                    for (int p = 0; p < PPT; p++) dom[p] |= dom_test<T, D, FULL>(x, y[p]);
                    if ((i & 7u) == 7u) {
                        bool lv = false;
#pragma unroll
                        for (int p = 0; p < PPT; p++) lv |= valid[p] && !dom[p];
                        if (__ballot(lv) == 0ull) break;
                    }
                }
            }
            __syncthreads();
        }
        // 2) against the earlier members of the chunk (and equal-score ones when TIES)
#pragma unroll
        for (int p = 0; p < PPT; p++) {
            const uint32_t j = threadIdx.x + p * kThreads;
            const uint32_t wlast = p * kThreads + (threadIdx.x | 63u);
            const uint32_t iend = xk == 0 ? 0 : (wlast < xk ? wlast : xk - 1);
            bool dm = dom[p];
            for (uint32_t i = 0; i < iend; i++) {
                if ((i & 15u) == 0u && __ballot(valid[p] && !dm) == 0ull) break;
                T x[D];
                lds_row<T, D>(s_x + (size_t)i * DP, x);
                dm |= (i < j) && dom_test<T, D, FULL>(x, y[p]);
            }
            if constexpr (TIES) {
                if (valid[p] && !dm) {
                    const uint32_t sj = s_sc[j];
                    for (uint32_t i = j + 1; i < xk && s_sc[i] == sj && !dm; i++) {
                        T x[D];
                        lds_row<T, D>(s_x + (size_t)i * DP, x);
                        dm = dom_test<T, D, true>(x, y[p]);
                    }
                    for (uint32_t q = x0 + xk; q < cnt && !dm; q++) {
                        if (key_score<T>(key[base + q]) != sj) break;
                        T x[D];
#pragma unroll
                        for (int d = 0; d < D; d++) x[d] = rows[(size_t)(base + q) * DP + d];
                        dm = dom_test<T, D, true>(x, y[p]);
                    }
                }
            }
            if (valid[p]) s_keep[j] = dm ? 0u : 1u;
        }
        __syncthreads();
        // 3) append the chunk's survivors to C, in order
        for (uint32_t j0 = 0; j0 < xk; j0 += kThreads) {
            const uint32_t j = j0 + threadIdx.x;
            const bool keep = j < xk && s_keep[j];
            const uint64_t b = __ballot(keep);
            const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
            if (lane == 0) s_w[w] = __popcll(b);
            __syncthreads();
            uint32_t wb = 0, tot = 0;
            for (int q = 0; q < kThreads / 64; q++) { wb += q < w ? s_w[q] : 0u; tot += s_w[q]; }
            __syncthreads();
            if (keep) {
                const uint32_t pos = nconf + wb + __popcll(b & lt);
#pragma unroll
                for (int d = 0; d < DP; d++) C[(size_t)pos * DP + d] = s_x[(size_t)j * DP + d];
                alive[base + x0 + j] = 1;
            }
            nconf += tot;
        }
        __syncthreads();   // C's new rows (global, written by this workgroup) are read next chunk
    }
}

// Round step 2: every remaining candidate of a large partition is tested against
// the confirmed X' of its partition (kept rows of X packed into LDS tile by tile).
template <typename T, int D, bool FULL, int PPT>
__global__ __launch_bounds__(kThreads) void k_filter_rest(const T *__restrict__ rows, const uint32_t *__restrict__ act,
                                                          const SfsTile *__restrict__ tiles,
                                                          const SfsSeg *__restrict__ segs, int B, int TB,
                                                          const uint8_t *__restrict__ xkeep,
                                                          uint32_t *__restrict__ keep) {
    constexpr int DP = padded_dims<T>(D);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T *s_c = reinterpret_cast<T *>(smem);
    __shared__ uint32_t s_n;
    const SfsTile tl = tiles[blockIdx.x];
    const SfsSeg sg = segs[tl.seg];
    const uint32_t xk = sg.count < (uint32_t)B ? sg.count : (uint32_t)B;
    const uint8_t *xk_flags = xkeep + (size_t)tl.seg * B;
    T y[PPT][D];
    bool valid[PPT], dom[PPT];
#pragma unroll
    for (int p = 0; p < PPT; p++) {
        const uint32_t e = threadIdx.x + p * kThreads;
        valid[p] = e < tl.count;
        dom[p] = false;
        const uint32_t r = valid[p] ? act[tl.start + e] : 0u;
#pragma unroll
        for (int d = 0; d < D; d++) y[p][d] = valid[p] ? rows[(size_t)r * DP + d] : T(0);
    }
    for (uint32_t c0 = 0; c0 < xk; c0 += TB) {
        const uint32_t cn = xk - c0 < (uint32_t)TB ? xk - c0 : (uint32_t)TB;
        if (threadIdx.x == 0) s_n = 0;
        __syncthreads();
        for (uint32_t q = threadIdx.x; q < cn; q += kThreads) {
            if (!xk_flags[c0 + q]) continue;
            const uint32_t pos = atomicAdd(&s_n, 1u);          // order inside X' is irrelevant
            const T *src = rows + (size_t)act[sg.begin + c0 + q] * DP;
#pragma unroll
            for (int d = 0; d < DP; d++) s_c[(size_t)pos * DP + d] = src[d];
        }
        __syncthreads();
        const uint32_t nc = s_n;
        for (uint32_t i = 0; i < nc; i++) {
            T x[D];
            lds_row<T, D>(s_c + (size_t)i * DP, x);
#pragma unroll
            for (int p = 0; p < PPT; p++) dom[p] |= dom_test<T, D, FULL>(x, y[p]);
            if ((i & 7u) == 7u) {
                bool live = false;
#pragma unroll
                for (int p = 0; p < PPT; p++) live |= valid[p] && !dom[p];
                if (__ballot(live) == 0ull) break;
            }
        }
        bool live = false;
#pragma unroll
        for (int p = 0; p < PPT; p++) live |= valid[p] && !dom[p];
        if (!__syncthreads_or(live)) break;
    }
#pragma unroll
    for (int p = 0; p < PPT; p++) {
        const uint32_t e = threadIdx.x + p * kThreads;
        if (valid[p]) keep[tl.out + e] = dom[p] ? 0u : 1u;
    }
}

__global__ __launch_bounds__(kThreads) void k_act_compact(const uint32_t *__restrict__ act_old,
                                                          const uint32_t *__restrict__ keep,
                                                          const uint32_t *__restrict__ keep_scan,
                                                          const SfsTile *__restrict__ tiles,
                                                          uint32_t *__restrict__ act_new,
                                                          uint32_t *__restrict__ segcnt) {
    __shared__ uint32_t s_w[kThreads / 64];
    const SfsTile tl = tiles[blockIdx.x];
    uint32_t c = 0;
    for (uint32_t e = threadIdx.x; e < tl.count; e += kThreads)
        if (keep[tl.out + e]) { act_new[keep_scan[tl.out + e]] = act_old[tl.start + e]; c++; }
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) c += __shfl_xor(c, s, 64);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int i = 0; i < kThreads / 64; i++) t += s_w[i];
        if (t) atomicAdd(&segcnt[tl.seg], t);
    }
}

__global__ __launch_bounds__(kThreads) void k_iota(uint32_t *__restrict__ a, uint32_t n) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j < n) a[j] = j;
}

// Batched fill: the small per-query zero/0xff ranges of one phase in ONE launch
// (each hipMemsetAsync is its own dispatch plus ~5-10 us of CP gap).  blockIdx.y
// picks the range; the range fields are read by compile-time index only (see
// DESIGN §8 on dynamically indexed kernel-argument arrays).
__global__ __launch_bounds__(kThreads) void k_fill_multi(FillRanges f) {
    uint8_t *p = nullptr;
    uint32_t bytes = 0, val = 0;
#pragma unroll
    for (int j = 0; j < kFillMax; j++)
        if ((int)blockIdx.y == j) { p = f.p[j]; bytes = f.bytes[j]; val = f.val[j]; }
    if (!p) return;
    const uint32_t words = bytes >> 2;
    const uint32_t w4 = val * 0x01010101u;
    uint32_t *p4 = reinterpret_cast<uint32_t *>(p);
    for (uint32_t q = blockIdx.x * kThreads + threadIdx.x; q < words; q += gridDim.x * kThreads) p4[q] = w4;
    if (blockIdx.x == 0 && threadIdx.x < (bytes & 3u)) p[words * 4 + threadIdx.x] = (uint8_t)val;
}

void FillSet::add(void *ptr, size_t nbytes, int value) {
    if (!ptr || !nbytes) return;
    if ((uintptr_t)ptr & 3u) {
        plain.push_back({{ptr, nbytes}, value});
        return;
    }
    constexpr size_t kPiece = size_t(1) << 31;   // < 4 GiB per range, 4-aligned pieces
    for (size_t off = 0; off < nbytes; off += kPiece) {
        if (n == kFillMax) {
            full.push_back(static_cast<const FillRanges &>(*this));
            n = 0;
        }
        p[n] = (uint8_t *)ptr + off;
        bytes[n] = (uint32_t)std::min(kPiece, nbytes - off);
        val[n] = (uint32_t)(value & 0xff);
        n++;
    }
}

static void launch_fill_ranges(const FillRanges &f, hipStream_t st) {
    uint32_t mx = 0;
    for (int j = 0; j < f.n; j++) mx = std::max(mx, f.bytes[j]);
    const uint32_t gx = std::max(1u, std::min(256u, (mx / 4 + kThreads * 4 - 1) / (kThreads * 4)));
    k_fill_multi<<<dim3(gx, (unsigned)f.n), kThreads, 0, st>>>(f);
}

bool FillSet::take(FillRanges &out) {
    if (!full.empty() || !plain.empty()) return false;
    out = static_cast<const FillRanges &>(*this);
    n = 0;
    return true;
}

hipError_t FillSet::launch(hipStream_t st) {
    hipError_t e = hipSuccess;
    for (const FillRanges &f : full) launch_fill_ranges(f, st);
    if (n) launch_fill_ranges(*this, st);
    for (auto &q : plain)
        if (hipMemsetAsync(q.first.first, q.second, q.first.second, st) != hipSuccess && e == hipSuccess)
            e = hipGetLastError();
    full.clear();
    plain.clear();
    n = 0;
    const hipError_t l = hipGetLastError();
    return e != hipSuccess ? e : l;
}

// Batched read-back: the small counters one host synchronisation needs, copied by
// ONE launch straight into the pinned (host-mapped) staging buffer instead of one
// copy-engine dispatch per range.  Words only (4-byte aligned ranges).
__global__ __launch_bounds__(kThreads) void k_gather_words(FillRanges g, uint32_t *__restrict__ dst) {
    const uint32_t *src = nullptr;
    uint32_t words = 0, off = 0;
#pragma unroll
    for (int j = 0; j < kFillMax; j++)
        if ((int)blockIdx.x == j) { src = reinterpret_cast<const uint32_t *>(g.p[j]); words = g.bytes[j] >> 2; off = g.val[j] >> 2; }
    if (!src) return;
    for (uint32_t q = threadIdx.x; q < words; q += kThreads) dst[off + q] = src[q];
}

hipError_t launch_gather_words(const FillRanges &g, void *pinned_dst, hipStream_t st) {
    k_gather_words<<<g.n, kThreads, 0, st>>>(g, reinterpret_cast<uint32_t *>(pinned_dst));
    return hipGetLastError();
}

// global merge ordering: (score | rep index) for the alive local representatives
__global__ __launch_bounds__(kThreads) void k_global_keys(const uint64_t *__restrict__ rep_key,
                                                          const uint8_t *__restrict__ alive_l,
                                                          const uint32_t *__restrict__ alive_scan, uint32_t mr,
                                                          uint64_t *__restrict__ gkey, uint32_t *__restrict__ gval,
                                                          unsigned long long *__restrict__ orand) {
    __shared__ unsigned long long s_o[kThreads / 64], s_a[kThreads / 64];
    __shared__ int s_any[kThreads / 64];
    const uint32_t r = blockIdx.x * kThreads + threadIdx.x;
    uint64_t o = 0, an = ~0ull;
    const bool any = __ballot(r < mr && alive_l[r]) != 0ull;
    if (r < mr && alive_l[r]) {
        const uint32_t e = alive_scan[r];
        const uint64_t k = rep_key[r] & 0x00ffffffff000000ull;   // score field only (same layout as rep_key)
        gkey[e] = k;
        gval[e] = r;
        o = k;
        an = k;
    }
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) {
        o |= __shfl_xor(o, s, 64);
        an &= __shfl_xor(an, s, 64);
    }
    // one pair of global atomics per workgroup (per-wave atomics on one address serialise)
    if ((threadIdx.x & 63) == 0) { s_o[threadIdx.x >> 6] = o; s_a[threadIdx.x >> 6] = an; s_any[threadIdx.x >> 6] = any; }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long bo = 0, ba = ~0ull;
        int has = 0;
        for (int q = 0; q < kThreads / 64; q++)
            if (s_any[q]) { bo |= s_o[q]; ba &= s_a[q]; has = 1; }
        if (has) {
            atomicOr(&orand[0], bo);
            atomicAnd(&orand[1], ba);
        }
    }
}

template <typename T, int D>
__global__ __launch_bounds__(kThreads) void k_gather_rows(const T *__restrict__ src, const uint32_t *__restrict__ idx,
                                                          uint32_t m, T *__restrict__ dst) {
    constexpr int DP = padded_dims<T>(D);
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= m) return;
    const T *s = src + (size_t)idx[j] * DP;
    T *o = dst + (size_t)j * DP;
#pragma unroll
    for (int d = 0; d < DP; d++) o[d] = s[d];
}

__global__ __launch_bounds__(kThreads) void k_scatter_alive(const uint32_t *__restrict__ gval,
                                                            const uint8_t *__restrict__ galive, uint32_t mg,
                                                            uint8_t *__restrict__ alive_g) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j < mg) alive_g[gval[j]] = galive[j];
}

// The brute route's per-tile output counts (k_out_hist_count: the duplicate groups whose pruner is
// in G, listed first, plus the tile's candidates in G), their exclusive scan, the stats reduce
// (k_stat_reduce) and the final read's words into host-mapped memory (k_gather_words), in ONE
// 1024-thread workgroup: four dependent launches of 4-6 us each before.  Tiles TT per thread and
// batch, their loads issued together.
constexpr int kTailThreads = 1024;
__global__ __launch_bounds__(kTailThreads) void k_tail_counts(TailArgs a) {
    constexpr int NT = kTailThreads, NW = kTailThreads / 64, TT = 4;
    __shared__ uint16_t s_gq[kHistMaxKM];
    __shared__ uint32_t s_ng, s_w[NW];
    __shared__ unsigned long long s_st[2 * kMaxK];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (wave == 0) {
        uint32_t ng = 0;
        for (int q0 = 0; q0 < a.KM; q0 += 64) {
            const bool g = q0 + lane < a.KM && (a.pruner_fate[q0 + lane] & 2u);
            const uint64_t b = __ballot(g);
            if (g) s_gq[ng + __popcll(b & (lane ? (~0ull >> (64 - lane)) : 0ull))] = (uint16_t)(q0 + lane);
            ng += (uint32_t)__popcll(b);
        }
        if (lane == 0) s_ng = ng;
    }
    // stats: wave w reduces partitions w, w + NW, ... over the shards
    for (int k = wave; k < a.K; k += NW) {
        unsigned long long l = 0, sv = 0;
        for (int sh = lane; sh < kStatShards; sh += 64) {
            l += a.lsz[(size_t)sh * a.K + k];
            sv += a.surv[(size_t)sh * a.K + k];
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            l += __shfl_xor(l, o, 64);
            sv += __shfl_xor(sv, o, 64);
        }
        if (lane == 0) {
            s_st[k] = l;
            s_st[a.K + k] = sv;
            a.statk[k] = l;
            a.statk[a.K + k] = sv;
        }
    }
    __syncthreads();
    const uint32_t ng = s_ng;
    uint32_t base = 0;
    for (uint32_t t0 = 0; t0 < a.ntiles; t0 += TT * NT) {           // block-uniform
        uint32_t c[TT], tot_t = 0;
#pragma unroll
        for (int u = 0; u < TT; u++) {
            const uint32_t t = t0 + (uint32_t)tid * TT + u;          // consecutive tiles per thread
            c[u] = 0;
            if (t < a.ntiles) {
                const uint32_t *h = a.tile_hist + (size_t)t * a.KM;
                for (uint32_t i = 0; i < ng; i++) c[u] += h[s_gq[i]];
                c[u] += a.tile_cand[t];
            }
            tot_t += c[u];
        }
        // block exclusive scan of the per-thread sums
        uint32_t inc = tot_t;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(inc, o, 64);
            if (lane >= o) inc += y;
        }
        if (lane == 63) s_w[wave] = inc;
        __syncthreads();
        uint32_t wb = 0, tot = 0;
#pragma unroll
        for (int i = 0; i < NW; i++) {
            const uint32_t x = s_w[i];
            wb += i < wave ? x : 0u;
            tot += x;
        }
        __syncthreads();
        uint32_t off = base + wb + inc - tot_t;
#pragma unroll
        for (int u = 0; u < TT; u++) {
            const uint32_t t = t0 + (uint32_t)tid * TT + u;
            if (t < a.ntiles) {
                a.out_cnt[t] = c[u];
                a.out_off[t] = off;
            }
            off += c[u];
        }
        base += tot;
    }
    if (tid == 0) a.totals[3] = base;
    __syncthreads();
    if (a.pin) {
        if (tid < 16) a.pin[tid] = tid == 3 ? base : a.totals[tid];
        for (int q = tid; q < a.K; q += NT) {
            a.pin[a.pin_off[0] + 2 * q] = (uint32_t)s_st[q];
            a.pin[a.pin_off[0] + 2 * q + 1] = (uint32_t)(s_st[q] >> 32);
            a.pin[a.pin_off[0] + 2 * (a.K + q)] = (uint32_t)s_st[a.K + q];
            a.pin[a.pin_off[0] + 2 * (a.K + q) + 1] = (uint32_t)(s_st[a.K + q] >> 32);
        }
        for (int q = tid; q < a.Kp; q += NT) {
            a.pin[a.pin_off[1] + q] = a.segalive[q];
            a.pin[a.pin_off[2] + q] = a.segn[q];
        }
        if (tid == 0) a.pin[a.pin_off[3]] = *a.flags;
        for (int q = tid; q < a.KM; q += NT) a.pin[a.pin_off[4] + q] = a.dup_cnt[q];
    }
}

void launch_tail_counts(const TailArgs &a, hipStream_t st) {
    k_tail_counts<<<1, kTailThreads, 0, st>>>(a);
}

// sum the [shard][K] stat accumulators into [K] (one workgroup per key)
__global__ __launch_bounds__(kThreads) void k_stat_reduce(const unsigned long long *__restrict__ lsz,
                                                          const unsigned long long *__restrict__ surv, int K,
                                                          unsigned long long *__restrict__ out) {
    __shared__ unsigned long long s_l[kThreads / 64], s_s[kThreads / 64];
    const int k = blockIdx.x;
    unsigned long long l = 0, sv = 0;
    for (int sh = threadIdx.x; sh < kStatShards; sh += kThreads) {
        l += lsz[(size_t)sh * K + k];
        sv += surv[(size_t)sh * K + k];
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        l += __shfl_xor(l, o, 64);
        sv += __shfl_xor(sv, o, 64);
    }
    if ((threadIdx.x & 63) == 0) { s_l[threadIdx.x >> 6] = l; s_s[threadIdx.x >> 6] = sv; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int q = 1; q < kThreads / 64; q++) { l = s_l[0] += s_l[q]; sv = s_s[0] += s_s[q]; }
        out[k] = s_l[0];
        out[K + k] = s_s[0];
    }
}

void launch_stat_reduce(const unsigned long long *lsz, const unsigned long long *surv, int K, unsigned long long *out,
                        hipStream_t st) {
    if (K > 0) k_stat_reduce<<<K, kThreads, 0, st>>>(lsz, surv, K, out);
}

__global__ __launch_bounds__(kThreads) void k_u8_to_u32(const uint8_t *__restrict__ in, uint32_t n,
                                                        uint32_t *__restrict__ out) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j < n) out[j] = in[j] ? 1u : 0u;
}

// distinct local-skyline vectors per partition (for the algorithmic work count W)
__global__ __launch_bounds__(kThreads) void k_seg_alive(const uint64_t *__restrict__ rep_key,
                                                        const uint8_t *__restrict__ alive, uint32_t mr,
                                                        uint32_t *__restrict__ cnt) {
    __shared__ uint32_t s_c[kMaxK];
    for (int q = threadIdx.x; q < kMaxK; q += kThreads) s_c[q] = 0;
    __syncthreads();
    for (uint32_t r = blockIdx.x * kThreads + threadIdx.x; r < mr; r += gridDim.x * kThreads) {
        const bool a = alive[r] != 0;
        const uint32_t k = a ? (uint32_t)(rep_key[r] >> 56) : 0u;
        // reps are sorted by partition: a wave is nearly always one partition
        const uint64_t am = __ballot(a);
        if (!am) continue;
        const uint32_t k0 = __shfl(k, __ffsll((unsigned long long)am) - 1, 64);
        if (__ballot(a && k != k0) == 0ull) {
            if ((threadIdx.x & 63) == __ffsll((unsigned long long)am) - 1) atomicAdd(&s_c[k0], (uint32_t)__popcll(am));
        } else if (a) {
            atomicAdd(&s_c[k], 1u);
        }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < kMaxK; q += kThreads)
        if (s_c[q]) atomicAdd(&cnt[q], s_c[q]);
}

void launch_seg_alive(const uint64_t *rep_key, const uint8_t *alive, uint32_t mr, uint32_t *cnt, hipStream_t st) {
    if (!mr) return;
    unsigned g = (mr + kThreads - 1) / kThreads;
    if (g > 1024) g = 1024;
    k_seg_alive<<<g, kThreads, 0, st>>>(rep_key, alive, mr, cnt);
}

// Both skyline levels of a SMALL candidate-slot set without sort, duplicate collapse, rounds
// or host round trips: slot y is in L_k iff no slot of its partition dominates it, and in G
// iff no slot at all dominates it (a dominator outside the union of the L_k is itself
// dominated by a member of it: transitivity).  Full dominance test in f64 (duplicates stay:
// equal vectors never dominate each other, so they share their fate).  A slot with a larger
// f32 score is skipped (the clamped f64 sum rounded to f32 is monotone under dominance).
//   k_brute_pairs   grid (y blocks of 64 = one wave, x chunks of 64 rows in LDS): the
//                   wave's lanes test their y against the chunk; hits are OR-ed into
//                   domf[y] (bit0: same partition, bit1: any)
//   k_brute_finish  alive_l / alive_g from domf, identity slot -> rep map, per-partition
//                   slot and alive counts
constexpr int kBruteY = 64, kBruteX = 64;
// T: the compare type (f32 when every candidate value is exactly an f32, else f64); the slot
// rows in HBM are f64 either way
template <typename T, int D>
__global__ __launch_bounds__(kBruteY) void k_brute_pairs(const double *__restrict__ rows,
                                                         const uint64_t *__restrict__ key, uint32_t mr,
                                                         const uint32_t *__restrict__ d_mr,
                                                         uint32_t *__restrict__ domf) {
    constexpr int DP = padded_dims<double>(D);
    if (d_mr) mr = min(mr, *d_mr);             // device-sized launch: mr is the bound
    if (blockIdx.x * kBruteY >= mr || blockIdx.y * kBruteX >= mr) return;
    __shared__ T s_x[kBruteX * D];
    __shared__ uint32_t s_k[kBruteX];                         // f32 order key of the score
    __shared__ uint32_t s_p[kBruteX];                         // partition
    const uint32_t y0 = blockIdx.x * kBruteY, x0 = blockIdx.y * kBruteX;
    const uint32_t cn = mr - x0 < (uint32_t)kBruteX ? mr - x0 : (uint32_t)kBruteX;
    for (uint32_t q = threadIdx.x; q < cn * D; q += kBruteY) {
        const uint32_t r = q / D, d = q - r * D;
        s_x[q] = (T)rows[(size_t)(x0 + r) * DP + d];
    }
    for (uint32_t q = threadIdx.x; q < cn; q += kBruteY) {
        const uint64_t kx = key[x0 + q];
        s_k[q] = (uint32_t)(kx >> 24);                        // score bits 55..24
        s_p[q] = (uint32_t)(kx >> 56);
    }
    const uint32_t j = y0 + threadIdx.x;
    const bool valid = j < mr;
    T y[D];
#pragma unroll
    for (int d = 0; d < D; d++) y[d] = valid ? (T)rows[(size_t)j * DP + d] : T(0);
    const uint64_t ky = valid ? key[j] : 0ull;
    const uint32_t py = (uint32_t)(ky >> 56), sy = valid ? (uint32_t)(ky >> 24) : 0u;
    __syncthreads();
    uint32_t f = 0;
#pragma unroll 4
    for (uint32_t i = 0; i < cn; i++) {
        const bool cand = s_k[i] <= sy;                       // a larger score cannot dominate
        const bool dom = cand && dominates_full<D, T>(s_x + (size_t)i * D, y);
        f |= dom ? (s_p[i] == py ? 3u : 2u) : 0u;
    }
    if (valid && f) atomicOr(&domf[j], f);
}

// The same two levels for integer rows (every candidate value an integer in [0, 65535]):
// rows pack into W u32 words of two u16 halves, and for integers
//     x dominates y  <=>  x <= y everywhere and sum(x) < sum(y)
// (x <= y with x != y makes the sum strictly smaller; equal vectors have equal sums), i.e.
//     OR_w sat_u16(x_w - y_w)  |  sat_u32(sum(x) + 1 - sum(y))  == 0.
// A dense all-pairs tile: a workgroup holds 256 YL y (YL per lane) and stages X x rows in LDS
// once, ordered by partition (a counting sort of the chunk), so that every x row costs the
// compare words and ONE running minimum per y: per partition run the lane keeps min_x(word); at
// the run's end the any-partition minimum takes it, and the same-partition minimum too where the
// run's partition is the y's.  8D: 4 v_pk_sub_u16 (clamp) + 1 saturating u32 subtract + 2 v_or3 +
// 1 v_min per pair test (8 compares), no per-pair VALU -> SGPR mask traffic; every x row read
// from LDS serves both of a lane's y (half the LDS reads per pair test of one y per lane).
// Tile shape by size: YL y per lane and X rows per chunk.  Large sets (the 64k dense line): two y
// per lane, 512-row chunks; the query's slot sets (C4: 7.9k slots) keep one y per lane and 128-row
// chunks, so that the grid still holds ~2k workgroups (16 x 16 of the large shape was one wave
// per SIMD: 41 us against 24 us for C4's slots)
constexpr int kB16T = 256;

typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t sat_sub_u16x2(uint32_t x, uint32_t y) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(__builtin_bit_cast(u16x2_t, x),
                                                                      __builtin_bit_cast(u16x2_t, y)));
}

template <int D, int W>
__device__ __forceinline__ uint32_t pack_row16(const double *r, uint32_t (&w)[W]) {
    uint32_t s = 0;
#pragma unroll
    for (int q = 0; q < W; q++) {
        const uint32_t lo = 2 * q < D ? (uint32_t)r[2 * q] : 0u;
        const uint32_t hi = 2 * q + 1 < D ? (uint32_t)r[2 * q + 1] : 0u;
        w[q] = lo | (hi << 16);
        s += lo + hi;
    }
    return s;
}

template <int W>
__device__ __forceinline__ uint32_t dom16_word(const uint4 (&xw)[W / 4], uint32_t xs, const uint32_t (&y)[W],
                                               uint32_t sy) {
    uint32_t r = __builtin_elementwise_sub_sat(xs, sy);
#pragma unroll
    for (int q = 0; q < W / 4; q++)
        r |= sat_sub_u16x2(xw[q].x, y[4 * q]) | sat_sub_u16x2(xw[q].y, y[4 * q + 1]) |
             sat_sub_u16x2(xw[q].z, y[4 * q + 2]) | sat_sub_u16x2(xw[q].w, y[4 * q + 3]);
    return r;
}

template <int D, int W, int YL, int X>
__global__ __launch_bounds__(kB16T) void k_brute16_pairs(const double *__restrict__ rows,
                                                         const uint64_t *__restrict__ key, uint32_t mr,
                                                         const uint32_t *__restrict__ d_mr,
                                                         uint32_t *__restrict__ domf) {
    constexpr int DP = padded_dims<double>(D);
    constexpr int RPT = (X + kB16T - 1) / kB16T;                // x rows staged per thread (at most)
    constexpr int YB = kB16T * YL;                              // y per workgroup
    if (d_mr) mr = min(mr, *d_mr);
    if (blockIdx.x * YB >= mr || blockIdx.y * X >= mr) return;
    __shared__ uint4 s_x[X][W / 4];
    __shared__ uint32_t s_s[X];                                 // sum + 1 of each staged row
    __shared__ uint32_t s_h[kMaxK];                             // rows per partition -> run start
    __shared__ uint32_t s_rb[kMaxK + 1], s_rp[kMaxK];            // runs: start, partition
    __shared__ uint32_t s_w[kB16T / 64];
    static_assert(kMaxK == kB16T, "the partition scan takes one partition per thread");
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t y0 = blockIdx.x * YB, x0 = blockIdx.y * X;
    const uint32_t cn = mr - x0 < (uint32_t)X ? mr - x0 : (uint32_t)X;
    for (int q = tid; q < kMaxK; q += kB16T) s_h[q] = 0;
    // this lane's y's
    uint32_t y[YL][W], sy[YL], py[YL];
#pragma unroll
    for (int v = 0; v < YL; v++) {
        const uint32_t j = y0 + v * kB16T + tid;
        sy[v] = 0;
        py[v] = 0xffffffffu;
        if (j < mr) {
            sy[v] = pack_row16<D, W>(rows + (size_t)j * DP, y[v]);
            py[v] = (uint32_t)(key[j] >> 56);
        } else {
#pragma unroll
            for (int q = 0; q < W; q++) y[v][q] = 0u;
        }
    }
    // the chunk's rows, ranked within their partition
    uint32_t xw[RPT][W], xs[RPT], xp[RPT], xr[RPT];
#pragma unroll
    for (int u = 0; u < RPT; u++) {
        const uint32_t r = u * kB16T + tid;
        xp[u] = 0xffffffffu;
        if (r < cn) {                                           // (cn <= X)
            xs[u] = pack_row16<D, W>(rows + (size_t)(x0 + r) * DP, xw[u]) + 1u;
            xp[u] = (uint32_t)(key[x0 + r] >> 56);
        }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < RPT; u++)
        if (xp[u] != 0xffffffffu) xr[u] = atomicAdd(&s_h[xp[u]], 1u);
    __syncthreads();
    // exclusive scan of the partition counts (one per thread) and the run list
    {
        const uint32_t c = s_h[tid];
        uint32_t inc = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(inc, o, 64);
            if (lane >= o) inc += t;
        }
        const uint64_t nz = __ballot(c != 0u);
        if (lane == 63) s_w[wave] = inc | ((uint32_t)__popcll(nz) << 16);
        __syncthreads();
        uint32_t base = 0, rbase = 0, tot_r = 0;
#pragma unroll
        for (int w = 0; w < kB16T / 64; w++) {
            const uint32_t v = s_w[w];
            if (w < wave) { base += v & 0xffffu; rbase += v >> 16; }
            tot_r += v >> 16;
        }
        const uint32_t start = base + inc - c;
        __syncthreads();
        s_h[tid] = start;
        if (c) {
            const uint32_t ri = rbase + (uint32_t)__popcll(nz & ((1ull << lane) - 1ull));
            s_rb[ri] = start;
            s_rp[ri] = (uint32_t)tid;
        }
        if (tid == 0) s_rb[tot_r] = cn;                         // the end of the last run
        if (tid == 0) s_w[0] = tot_r;
    }
    __syncthreads();
    const uint32_t nruns = __builtin_amdgcn_readfirstlane((int)s_w[0]);
#pragma unroll
    for (int u = 0; u < RPT; u++) {
        if (xp[u] == 0xffffffffu) continue;
        const uint32_t pos = s_h[xp[u]] + xr[u];
#pragma unroll
        for (int q = 0; q < W / 4; q++) s_x[pos][q] = make_uint4(xw[u][4 * q], xw[u][4 * q + 1], xw[u][4 * q + 2], xw[u][4 * q + 3]);
        s_s[pos] = xs[u];
    }
    __syncthreads();
    uint32_t acc_a[YL], acc_s[YL];
#pragma unroll
    for (int v = 0; v < YL; v++) acc_a[v] = acc_s[v] = 0xffffffffu;
    for (uint32_t rr = 0; rr < nruns; rr++) {
        const uint32_t b = __builtin_amdgcn_readfirstlane((int)s_rb[rr]);
        const uint32_t e = __builtin_amdgcn_readfirstlane((int)s_rb[rr + 1]);
        const uint32_t px = __builtin_amdgcn_readfirstlane((int)s_rp[rr]);
        constexpr int U = 4;                                    // rows in flight
        uint32_t acc_u[YL][U];
#pragma unroll
        for (int v = 0; v < YL; v++)
#pragma unroll
            for (int u = 0; u < U; u++) acc_u[v][u] = 0xffffffffu;
        uint32_t i = b;
        for (; i + U <= e; i += U) {
            uint4 xa[U][W / 4];
            uint32_t sa[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
#pragma unroll
                for (int q = 0; q < W / 4; q++) xa[u][q] = s_x[i + u][q];
                sa[u] = s_s[i + u];
            }
#pragma unroll
            for (int v = 0; v < YL; v++)
#pragma unroll
                for (int u = 0; u < U; u++) acc_u[v][u] = min(acc_u[v][u], dom16_word<W>(xa[u], sa[u], y[v], sy[v]));
        }
        for (; i < e; i++) {
            uint4 xa[W / 4];
#pragma unroll
            for (int q = 0; q < W / 4; q++) xa[q] = s_x[i][q];
            const uint32_t sa = s_s[i];
#pragma unroll
            for (int v = 0; v < YL; v++) acc_u[v][0] = min(acc_u[v][0], dom16_word<W>(xa, sa, y[v], sy[v]));
        }
#pragma unroll
        for (int v = 0; v < YL; v++) {
            const uint32_t acc = min(min(acc_u[v][0], acc_u[v][1]), min(acc_u[v][2], acc_u[v][3]));
            acc_a[v] = min(acc_a[v], acc);
            if (px == py[v]) acc_s[v] = min(acc_s[v], acc);
        }
    }
#pragma unroll
    for (int v = 0; v < YL; v++) {
        const uint32_t j = y0 + v * kB16T + tid;
        const uint32_t f = (acc_s[v] == 0u ? 3u : 0u) | (acc_a[v] == 0u ? 2u : 0u);
        if (j < mr && f) atomicOr(&domf[j], f);
    }
}

__global__ __launch_bounds__(kThreads) void k_brute_finish(const uint64_t *__restrict__ key, uint32_t mr,
                                                           const uint32_t *__restrict__ d_mr, int gmerge,
                                                           const uint32_t *__restrict__ domf,
                                                           uint8_t *__restrict__ alive_l, uint8_t *__restrict__ alive_g,
                                                           uint32_t *__restrict__ segalive,
                                                           uint32_t *__restrict__ segn, uint32_t *__restrict__ slot_rep) {
    __shared__ uint32_t s_n[kMaxK], s_a[kMaxK];
    for (int q = threadIdx.x; q < kMaxK; q += kThreads) { s_n[q] = 0; s_a[q] = 0; }
    if (d_mr) mr = min(mr, *d_mr);
    __syncthreads();
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j < mr) {
        const uint32_t f = domf[j];
        const bool in_l = !(f & 1u);
        const uint32_t k = (uint32_t)(key[j] >> 56);
        alive_l[j] = in_l ? 1 : 0;
        alive_g[j] = (gmerge ? !(f & 2u) : in_l) ? 1 : 0;
        slot_rep[j] = j;                                      // every slot is its own representative
        atomicAdd(&s_n[k], 1u);                               // per-block counts, then one global add
        if (in_l) atomicAdd(&s_a[k], 1u);
    }
    __syncthreads();
    for (int q = threadIdx.x; q < kMaxK; q += kThreads) {
        if (s_n[q]) atomicAdd(&segn[q], s_n[q]);
        if (s_a[q]) atomicAdd(&segalive[q], s_a[q]);
    }
}

void launch_brute_pairs(int D, bool f32, bool u16, const void *rows, const uint64_t *key, uint32_t mr, uint32_t *domf,
                        hipStream_t st, const uint32_t *d_mr) {
    if (!mr) return;
    const dim3 g((mr + kBruteY - 1) / kBruteY, (mr + kBruteX - 1) / kBruteX);
    if (u16) {
        // the large shape once it still fills the chip with >= 4096 workgroups (mr >= ~46k)
        const bool big = (uint64_t)((mr + 511) / 512) * ((mr + 511) / 512) >= 4096;
#define SKY_B16(YL, X)                                                                                       \
    do {                                                                                                     \
        const dim3 g16((mr + kB16T * YL - 1) / (kB16T * YL), (mr + X - 1) / X);                              \
        if (D <= 8) { SKY_DISPATCH_D(D, (k_brute16_pairs<DD, 4, YL, X><<<g16, kB16T, 0, st>>>((const double *)rows, key, mr, d_mr, domf))); } \
        else { SKY_DISPATCH_D(D, (k_brute16_pairs<DD, 8, YL, X><<<g16, kB16T, 0, st>>>((const double *)rows, key, mr, d_mr, domf))); }     \
    } while (0)
        if (big) SKY_B16(2, 512);
        else SKY_B16(1, 128);
#undef SKY_B16
    } else if (f32) {
        SKY_DISPATCH_D(D, (k_brute_pairs<float, DD><<<g, kBruteY, 0, st>>>((const double *)rows, key, mr, d_mr, domf)));
    } else {
        SKY_DISPATCH_D(D, (k_brute_pairs<double, DD><<<g, kBruteY, 0, st>>>((const double *)rows, key, mr, d_mr, domf)));
    }
}

void launch_brute_fates(int D, bool f32, bool u16, const void *rows, const uint64_t *key, uint32_t mr, bool gmerge,
                        uint32_t *domf, uint8_t *alive_l, uint8_t *alive_g, uint32_t *segalive, uint32_t *segn,
                        uint32_t *slot_rep, hipStream_t st, const uint32_t *d_mr) {
    if (!mr) return;
    launch_brute_pairs(D, f32, u16, rows, key, mr, domf, st, d_mr);
    k_brute_finish<<<(mr + kThreads - 1) / kThreads, kThreads, 0, st>>>(key, mr, d_mr, gmerge ? 1 : 0, domf, alive_l,
                                                                         alive_g, segalive, segn, slot_rep);
}

// ---- launchers ------------------------------------------------------------------
static inline unsigned nb(size_t n) { return (unsigned)((n + kThreads - 1) / kThreads); }

template <typename T, int D>
static void block_sky_t(bool full, bool ties, int B, int TB, const void *rows, const uint64_t *key, const uint32_t *act,
                        const SfsSeg *segs, const uint32_t *seg_list, uint32_t nseg_work, uint8_t *alive,
                        uint8_t *xkeep, hipStream_t st) {
    constexpr int DP = padded_dims<T>(D);
    const size_t lds = (size_t)TB * DP * sizeof(T);
    const dim3 grid(nseg_work, (B + kThreads - 1) / kThreads);
    const T *r = (const T *)rows;
    if (full) {
        if (ties) k_block_sky<T, D, true, true><<<grid, kThreads, lds, st>>>(r, key, act, segs, seg_list, B, TB, alive, xkeep);
        else k_block_sky<T, D, true, false><<<grid, kThreads, lds, st>>>(r, key, act, segs, seg_list, B, TB, alive, xkeep);
    } else {
        if (ties) k_block_sky<T, D, false, true><<<grid, kThreads, lds, st>>>(r, key, act, segs, seg_list, B, TB, alive, xkeep);
        else k_block_sky<T, D, false, false><<<grid, kThreads, lds, st>>>(r, key, act, segs, seg_list, B, TB, alive, xkeep);
    }
}

void launch_block_sky(int D, bool f64, bool full, bool ties, int B, int TB, const void *rows, const uint64_t *key,
                      const uint32_t *act, const SfsSeg *segs, const uint32_t *seg_list, uint32_t nseg_work,
                      uint8_t *alive, uint8_t *xkeep, hipStream_t st) {
    if (!nseg_work) return;
    if (f64) { SKY_DISPATCH_D(D, (block_sky_t<double, DD>(full, ties, B, TB, rows, key, act, segs, seg_list, nseg_work, alive, xkeep, st))); }
    else { SKY_DISPATCH_D(D, (block_sky_t<float, DD>(full, ties, B, TB, rows, key, act, segs, seg_list, nseg_work, alive, xkeep, st))); }
}

template <typename T, int D>
static void sfs_small_t(bool full, bool ties, int B, const void *rows, const uint64_t *key, const SfsSeg *segs,
                        const uint32_t *seg_list, uint32_t nwork, uint8_t *alive, void *conf, hipStream_t st) {
    constexpr int DP = padded_dims<T>(D);
    const size_t lds = 2 * (size_t)B * DP * sizeof(T) + 2 * (size_t)B * sizeof(uint32_t);
    const T *r = (const T *)rows;
    T *c = (T *)conf;
    if (full) {
        if (ties) k_sfs_small<T, D, true, true><<<nwork, kThreads, lds, st>>>(r, key, segs, seg_list, B, alive, c);
        else k_sfs_small<T, D, true, false><<<nwork, kThreads, lds, st>>>(r, key, segs, seg_list, B, alive, c);
    } else {
        if (ties) k_sfs_small<T, D, false, true><<<nwork, kThreads, lds, st>>>(r, key, segs, seg_list, B, alive, c);
        else k_sfs_small<T, D, false, false><<<nwork, kThreads, lds, st>>>(r, key, segs, seg_list, B, alive, c);
    }
}

void launch_sfs_small(int D, bool f64, bool full, bool ties, int B, const void *rows, const uint64_t *key,
                      const SfsSeg *segs, const uint32_t *seg_list, uint32_t nwork, uint8_t *alive, void *conf,
                      hipStream_t st) {
    if (!nwork) return;
    if (f64) { SKY_DISPATCH_D(D, (sfs_small_t<double, DD>(full, ties, B, rows, key, segs, seg_list, nwork, alive, conf, st))); }
    else { SKY_DISPATCH_D(D, (sfs_small_t<float, DD>(full, ties, B, rows, key, segs, seg_list, nwork, alive, conf, st))); }
}

constexpr int kPPT = 4;

template <typename T, int D>
static void filter_rest_t(bool full, int B, int TB, const void *rows, const uint32_t *act, const SfsTile *tiles,
                          uint32_t ntiles, const SfsSeg *segs, const uint8_t *xkeep, uint32_t *keep, hipStream_t st) {
    constexpr int DP = padded_dims<T>(D);
    const size_t lds = (size_t)TB * DP * sizeof(T);
    if (full)
        k_filter_rest<T, D, true, kPPT><<<ntiles, kThreads, lds, st>>>((const T *)rows, act, tiles, segs, B, TB, xkeep, keep);
    else
        k_filter_rest<T, D, false, kPPT><<<ntiles, kThreads, lds, st>>>((const T *)rows, act, tiles, segs, B, TB, xkeep, keep);
}

void launch_filter_rest(int D, bool f64, bool full, int B, int TB, const void *rows, const uint32_t *act,
                        const SfsTile *tiles, uint32_t ntiles, const SfsSeg *segs, const uint8_t *xkeep,
                        uint32_t *keep, hipStream_t st) {
    if (!ntiles) return;
    if (f64) { SKY_DISPATCH_D(D, (filter_rest_t<double, DD>(full, B, TB, rows, act, tiles, ntiles, segs, xkeep, keep, st))); }
    else { SKY_DISPATCH_D(D, (filter_rest_t<float, DD>(full, B, TB, rows, act, tiles, ntiles, segs, xkeep, keep, st))); }
}

void launch_act_compact(const uint32_t *act_old, const uint32_t *keep, const uint32_t *keep_scan,
                        const SfsTile *tiles, uint32_t ntiles, uint32_t *act_new, uint32_t *segcnt, hipStream_t st) {
    if (ntiles) k_act_compact<<<ntiles, kThreads, 0, st>>>(act_old, keep, keep_scan, tiles, act_new, segcnt);
}

void launch_iota(uint32_t *a, uint32_t n, hipStream_t st) {
    if (n) k_iota<<<nb(n), kThreads, 0, st>>>(a, n);
}

// *flag |= 1 if any of the `count` doubles is NaN (the stream append's admission check)
__global__ __launch_bounds__(kThreads) void k_nan_any(const double *__restrict__ v, size_t count,
                                                      uint32_t *__restrict__ flag) {
    bool nan = false;
    for (size_t q = (size_t)blockIdx.x * kThreads + threadIdx.x; q < count; q += (size_t)gridDim.x * kThreads)
        nan |= v[q] != v[q];
    if (__ballot(nan) != 0ull && (threadIdx.x & 63) == 0) atomicOr(flag, 1u);
}

void launch_nan_any(const double *v, size_t count, uint32_t *flag, hipStream_t st) {
    if (!count) return;
    const size_t blocks = std::min<size_t>(2048, (count + kThreads - 1) / kThreads);
    k_nan_any<<<(unsigned)blocks, kThreads, 0, st>>>(v, count, flag);
}

void launch_global_keys(const uint64_t *rep_key, const uint8_t *alive_l, const uint32_t *alive_scan, uint32_t mr,
                        uint64_t *gkey, uint32_t *gval, unsigned long long *orand, hipStream_t st) {
    if (mr) k_global_keys<<<nb(mr), kThreads, 0, st>>>(rep_key, alive_l, alive_scan, mr, gkey, gval, orand);
}

void launch_gather_rows(int D, bool f64, const void *src, const uint32_t *idx, uint32_t m, void *dst,
                        hipStream_t st) {
    if (!m) return;
    if (f64) { SKY_DISPATCH_D(D, (k_gather_rows<double, DD><<<nb(m), kThreads, 0, st>>>((const double *)src, idx, m, (double *)dst))); }
    else { SKY_DISPATCH_D(D, (k_gather_rows<float, DD><<<nb(m), kThreads, 0, st>>>((const float *)src, idx, m, (float *)dst))); }
}

void launch_scatter_alive(const uint32_t *gval, const uint8_t *galive, uint32_t mg, uint8_t *alive_g,
                          hipStream_t st) {
    if (mg) k_scatter_alive<<<nb(mg), kThreads, 0, st>>>(gval, galive, mg, alive_g);
}

void launch_flag_u8_to_u32(const uint8_t *in, uint32_t n, uint32_t *out, hipStream_t st) {
    if (n) k_u8_to_u32<<<nb(n), kThreads, 0, st>>>(in, n, out);
}

}  // namespace sky
