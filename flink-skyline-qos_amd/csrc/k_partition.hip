// k_partition.hip — the HBM-streaming stages of the skyline path on gfx950.
//
//   k_keys           getKey for every tuple (FlinkSkyline.java:707-712 / 774-789 / 827-875)
//   k_sample         strided sample: key + f64 monotone score
//   k_select_pruners per partition, up to M mutually non-dominated sample tuples, smallest
//                    score first (pruners never change the result: a tuple they dominate is
//                    outside its partition's skyline; a tuple EQUAL to one shares its fate)
//   k_filter         one pass over the f64 rows: key, pruner test, status word, per-tile
//                    candidate counts (wave-ballot + LDS), NaN / f32-exactness flags
//   k_compact<T>     order-preserving compaction of the candidates into AoS rows of T
//                    (f32 when every candidate value is exactly an f32, else f64) with a
//                    64-bit sort key (partition | score | vector hash)
//   k_gather_runs / k_run_first / k_rep_of / k_build_reps
//                    exact-duplicate collapse after the sort: one representative per
//                    distinct vector of a partition
//   k_out_count / k_out_write
//                    per tuple: is it in its local / the global skyline? -> stats
//                    (|L_k|, survivors_k) and the stream-ordered output ids
#include <algorithm>
#include "knobs.h"
#include <cstdlib>

#include "sky_internal.h"

namespace sky {

template <int D>
__device__ __forceinline__ void load_row(const double *__restrict__ p, double (&v)[D]) {
    if constexpr (D % 2 == 0) {
        const double2 *q = reinterpret_cast<const double2 *>(p);
#pragma unroll
        for (int d = 0; d < D / 2; d++) {
            double2 x = q[d];
            v[2 * d] = x.x;
            v[2 * d + 1] = x.y;
        }
    } else {
#pragma unroll
        for (int d = 0; d < D; d++) v[d] = p[d];
    }
}

template <typename T, int D>
__device__ __forceinline__ void store_row(T *__restrict__ p, const T (&v)[D]) {
    constexpr int DP = padded_dims<T>(D);
    T w[DP];
#pragma unroll
    for (int d = 0; d < DP; d++) w[d] = d < D ? v[d] : T(0);
    if constexpr (sizeof(T) == 4) {
        float4 *q = reinterpret_cast<float4 *>(p);
#pragma unroll
        for (int d = 0; d < DP / 4; d++) q[d] = make_float4(w[4 * d], w[4 * d + 1], w[4 * d + 2], w[4 * d + 3]);
    } else {
        double2 *q = reinterpret_cast<double2 *>(p);
#pragma unroll
        for (int d = 0; d < DP / 2; d++) q[d] = make_double2(w[2 * d], w[2 * d + 1]);
    }
}

template <typename T, int D>
__device__ __forceinline__ void load_trow(const T *__restrict__ p, T (&v)[D]) {
    constexpr int DP = padded_dims<T>(D);
    if constexpr (sizeof(T) == 4) {
        const float4 *q = reinterpret_cast<const float4 *>(p);
#pragma unroll
        for (int d = 0; d < DP / 4; d++) {
            float4 x = q[d];
            if (4 * d + 0 < D) v[4 * d + 0] = x.x;
            if (4 * d + 1 < D) v[4 * d + 1] = x.y;
            if (4 * d + 2 < D) v[4 * d + 2] = x.z;
            if (4 * d + 3 < D) v[4 * d + 3] = x.w;
        }
    } else {
        const double2 *q = reinterpret_cast<const double2 *>(p);
#pragma unroll
        for (int d = 0; d < DP / 2; d++) {
            double2 x = q[d];
            if (2 * d + 0 < D) v[2 * d + 0] = x.x;
            if (2 * d + 1 < D) v[2 * d + 1] = x.y;
        }
    }
}

// number of set bits of the wave mask m below this lane (v_mbcnt, no lane mask register)
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// exclusive rank of `flag` in (round, thread) order within the block; `base` carries
// the running count across rounds.  All threads of the block must call it.
__device__ __forceinline__ uint32_t block_rank(bool flag, uint32_t *s_w, uint32_t &base) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t b = __ballot(flag);
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    const uint32_t pre = __popcll(b & lt);
    if (lane == 0) s_w[w] = __popcll(b);
    __syncthreads();
    uint32_t wb = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kThreads / 64; i++) {
        const uint32_t c = s_w[i];
        wb += i < w ? c : 0u;
        tot += c;
    }
    __syncthreads();
    const uint32_t r = base + wb + pre;
    base += tot;
    return r;
}

__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t *s_w) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) v += __shfl_xor(v, s, 64);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = v;
    __syncthreads();
    uint32_t t = 0;
#pragma unroll
    for (int i = 0; i < kThreads / 64; i++) t += s_w[i];
    __syncthreads();
    return t;
}

// ---------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(kThreads) void k_keys(const double *__restrict__ vals, uint32_t n, KeyParams kp,
                                                   int32_t *__restrict__ keys) {
    for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < n; i += gridDim.x * kThreads) {
        double v[D];
        load_row<D>(vals + (size_t)i * D, v);
        const int32_t kk = partition_key<D>(v, kp);
        keys[i] = kk == kKeyFiltered ? -1 : kk;   // API: -1 = removed by the grid filter
    }
}

// ---- pruners ------------------------------------------------------------------
// A pruner of partition k is a tuple of k; any tuple of k it dominates is outside
// L_k, and a tuple EQUAL to it shares its fate, so the choice only affects speed.
// Pruner j of k is the sample tuple of k minimising the positive-weight linear
// criterion c_j (j = 0: the plain sum, i.e. the SFS score; j >= 1: the sum with
// dimension (j-1) mod D weighted 4x, pulling the winner towards another corner of
// the front): a minimiser of a positive-weight sum is never
// dominated within the sample, so the winners are (up to f32 rounding of c_j,
// checked exactly in k_pick_pruners) skyline points of the sample.  One parallel
// pass: per-(k, j) packed (order-key(c_j) << 32 | sample id) minima, LDS atomics
// per workgroup, one global atomicMin per workgroup and slot.
template <int D>
__global__ __launch_bounds__(kThreads) void k_sample_min(const double *__restrict__ vals, uint32_t n, uint32_t S,
                                                         KeyParams kp, const int32_t *__restrict__ given_keys,
                                                         int single, int Kp, int M,
                                                         unsigned long long *__restrict__ gmin, uint32_t tag,
                                                         FillRanges pre) {
    __shared__ unsigned long long s_min[2048];
    const int KM = Kp * M;
    fill_ranges_grid(pre);                   // the query's fills (read by the later kernels only)
    const unsigned long long tg = (unsigned long long)tag << 48;
    for (int q = threadIdx.x; q < KM; q += kThreads) s_min[q] = ~0ull;
    __syncthreads();
    // grid-stride over the sample (few workgroups: each adds its KM minima to the same KM
    // global words, so 256 workgroups serialised 256 atomics per word at L2)
#pragma unroll 4
    for (uint32_t s = blockIdx.x * kThreads + threadIdx.x; s < S; s += gridDim.x * kThreads) {
        const uint32_t i = (uint32_t)(((uint64_t)s * n) / S);
        double v[D];
        load_row<D>(vals + (size_t)i * D, v);
        bool nan = false;
#pragma unroll
        for (int d = 0; d < D; d++) nan |= v[d] != v[d];
        const int32_t k = single ? 0 : given_keys ? given_keys[i] : (nan ? -1 : partition_key<D>(v, kp));
        if (!nan && k >= 0 && k < Kp) {
            float f[D];
            float sum = 0.0f;
#pragma unroll
            for (int d = 0; d < D; d++) { f[d] = (float)v[d]; sum += f[d]; }
#pragma unroll
            for (int j = 0; j < 8; j++) {
                if (j >= M) break;
                const float c = j == 0 ? sum : sum + 3.0f * f[(j - 1) % D];
                if (c != c) continue;
                atomicMin(&s_min[k * M + j], tg | ((unsigned long long)f32_order_key(c) << 16) | s);
            }
        }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < KM; q += kThreads)
        if (s_min[q] != ~0ull && s_min[q] < __hip_atomic_load(&gmin[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            atomicMin(&gmin[q], s_min[q]);
}

// One workgroup per partition: the (<= M) winners are deduplicated (equal rows keep
// the first) and every winner another winner dominates is dropped (exact f64 test),
// so the pruners of k are distinct and mutually non-dominated.  Order: criterion j.
template <int D>
__global__ __launch_bounds__(64) void k_pick_pruners(const double *__restrict__ vals, uint32_t n, uint32_t S,
                                                     const unsigned long long *__restrict__ gmin, int M,
                                                     double *__restrict__ pruners, int32_t *__restrict__ npr,
                                                     uint32_t tag) {
    __shared__ double s_c[64][D];
    __shared__ int s_ok[64];
    const int k = blockIdx.x, j = threadIdx.x;
    const unsigned long long w = j < M ? gmin[k * M + j] : ~0ull;
    const bool has = (uint32_t)(w >> 48) == tag;       // (a word of an earlier query: empty)
    if (has) {
        const uint32_t s = (uint32_t)(w & 0xffffu);
        const uint32_t i = (uint32_t)(((uint64_t)s * n) / S);
#pragma unroll
        for (int d = 0; d < D; d++) s_c[j][d] = vals[(size_t)i * D + d];
    }
    s_ok[j] = has ? 1 : 0;
    __syncthreads();
    bool ok = has;
    if (ok) {
        for (int q = 0; q < M && ok; q++) {
            if (q == j || !s_ok[q]) continue;
            bool le = true, lt = false, eq = true;
#pragma unroll
            for (int d = 0; d < D; d++) {
                le &= s_c[q][d] <= s_c[j][d];
                lt |= s_c[q][d] < s_c[j][d];
                eq &= s_c[q][d] == s_c[j][d];
            }
            if ((le && lt) || (eq && q < j)) ok = false;
        }
    }
    const uint64_t b = __ballot(ok);
    if (ok) {
        const int pos = __popcll(b & (j == 0 ? 0ull : (~0ull >> (64 - j))));
#pragma unroll
        for (int d = 0; d < D; d++) pruners[((size_t)k * M + pos) * D + d] = s_c[j][d];
    }
    if (j == 0) npr[k] = __popcll(b);
}

// score = f64 sum of the (exact) T values in dimension order, each clamped to
// [-1e300, 1e300] so that +inf and -inf never meet (the clamp is monotone, so the
// score stays a linear extension of dominance).  A tie-free key needs no clamp, an
// exact sum and an exact f32 of it -> otherwise flag kFlagScoreTies.
template <typename T, int D>
__device__ __forceinline__ uint64_t make_sortkey(const T (&tv)[D], uint32_t part, uint32_t &lflags) {
    double s = 0.0;
    bool inexact = false;
#pragma unroll
    for (int d = 0; d < D; d++) {
        const double raw = (double)tv[d];
        const double x = raw > 1e300 ? 1e300 : (raw < -1e300 ? -1e300 : raw);
        inexact |= x != raw;
        const double sn = s + x;
        const double bb = sn - s;
        const double err = (s - (sn - bb)) + (x - bb);
        inexact |= err != 0.0;
        s = sn;
    }
    const float f = (float)s;
    inexact |= (double)f != s;
    if (inexact) lflags |= kFlagScoreTies;
    bool u16 = true;
#pragma unroll
    for (int d = 0; d < D; d++) {
        const double x = (double)tv[d];
        // -0.0 is excluded: packed it becomes +0 and would merge with a +0.0 twin of another
        // partition (MR-Angle keys read the sign bit), which the distinct-row tests assume away
        u16 &= (x >= 0.0) && (x <= 65535.0) && (x == floor(x)) &&
               (__double_as_longlong(x) != (long long)0x8000000000000000ull);
    }
    if (!u16) lflags |= kFlagNotU16;
    uint32_t h = 0x9e3779b9u;
#pragma unroll
    for (int d = 0; d < D; d++) {
        uint64_t bits;
        if constexpr (sizeof(T) == 4) bits = __float_as_uint(tv[d] == T(0) ? T(0) : tv[d]);
        else bits = (uint64_t)__double_as_longlong(tv[d] == T(0) ? T(0) : tv[d]);
        h = mix32(h ^ (uint32_t)bits ^ (uint32_t)(bits >> 32) * 0x85ebca6bu);
    }
    // 16 hash bits: equal vectors stay adjacent; a collision only lengthens one
    // equal-key run, which k_rep_of resolves by exact row compares
    return ((uint64_t)part << 56) | ((uint64_t)f32_order_key(f) << 24) | (uint64_t)(h & 0xffffu);
}

// A candidate joins the slot list (wave-aggregated append, unordered): f64 row,
// sort key (partition | score | hash) and source index.  OR / AND of the keys
// accumulate in o / an.
template <int D>
__device__ __forceinline__ void append_candidate(const FilterArgs &a, bool cand, const double (&v)[D], int32_t k,
                                                 uint32_t i, uint32_t &lflags, uint64_t &o, uint64_t &an) {
    const uint64_t cm = __ballot(cand);
    if (!cm) return;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((unsigned long long)cm) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(a.m_total, (uint32_t)__popcll(cm));
    base = __shfl(base, leader, 64);
    if (!cand) return;
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    const uint32_t slot = base + (uint32_t)__popcll(cm & lt);
    if (slot >= a.slot_cap) return;          // counted; the host re-runs with more slots
    constexpr int DP = padded_dims<double>(D);
    store_row<double, D>(a.crow + (size_t)slot * DP, v);
    const uint64_t key = make_sortkey<double, D>(v, (uint32_t)k, lflags);
    a.sortkey[slot] = key;
    a.slot_src[slot] = i;
    o |= key;
    an &= key;
}

// LDS image of the pruner table.  8D rows are 64 bytes; with partitions M rows
// apart every partition's row j starts on the same banks, so a wave whose lanes
// hold up to 16 partitions reads them 16-way conflicted.  For D == 8 each
// partition gets 64 bytes of padding (partition k -> 64-byte slot k % 4 of a
// 256-byte bank row) and its rows' 16-byte chunks are XOR-permuted by (k / 4) % 4:
// the 16 partitions of a ds_read_b128 lane group then hit 16 distinct bank quads.
template <int D>
__host__ __device__ constexpr int pr_stride(int M) { return M * D + (D == 8 ? 8 : 0); }   // doubles per partition
template <int D>
__device__ __forceinline__ int pr_off(int k, int j, int d) {   // within partition k's rows
    if constexpr (D == 8) return j * D + ((((d >> 1) ^ ((k >> 2) & 3)) << 1) | (d & 1));
    else return j * D + d;
}
template <int D>
constexpr size_t pruner_lds_bytes(int Kp, int M) {
    return (size_t)Kp * pr_stride<D>(M) * sizeof(double) + (size_t)Kp * M * 4;
}

// Classify one tuple of partition k: dropped (dominated by a pruner of k), exact
// duplicate of pruner j (code 1+j, counted by count_dups), or candidate.  Pruners
// are tested in f64.
template <int D>
__device__ __forceinline__ uint16_t classify(const double (&v)[D], int32_t k, const double *s_pr, const int32_t *s_npr,
                                             int M, uint32_t &lflags) {
    uint16_t code = kCodeCandidate;
    const int np = s_npr[k];
    const double *pr = s_pr + k * pr_stride<D>(M);
    // one compare per dimension and pruner: the first pruner with all(p <= v) decides, as a
    // duplicate if all(p == v) (tested for that pruner only), else dropped (p <= v and
    // p != v is dominance).  A NaN value fails every compare: the tuple comes out a
    // candidate, and the caller looks for NaN there.
    for (int j = 0; j < np; j++) {
        bool le = true;
#pragma unroll
        for (int d = 0; d < D; d++) le &= pr[pr_off<D>(k, j, d)] <= v[d];
        if (le) {
            bool eq = true;
#pragma unroll
            for (int d = 0; d < D; d++) eq &= pr[pr_off<D>(k, j, d)] == v[d];
            code = eq ? (uint16_t)(1 + j) : kCodeDropped;
            break;
        }
    }
    if (code == kCodeCandidate) {
#pragma unroll
        for (int d = 0; d < D; d++)
            if ((double)(float)v[d] != v[d]) lflags |= kFlagNotF32;
    }
    return code;
}

// Per-(partition, pruner) duplicate counts: the wave's first duplicate's (k, j)
// with ONE LDS atomic for all lanes sharing it (duplicates of one pruner usually
// fill whole waves; per-lane atomics on one address serialise), the others per
// lane.  All lanes call it.
__device__ __forceinline__ void count_dups(uint16_t code, int32_t k, int M, uint32_t *s_dup) {
    const bool dup = code != kCodeCandidate && code != kCodeDropped;
    const uint64_t m = __ballot(dup);
    if (!m) return;                                                  // wave-uniform
    const uint32_t kj = (uint32_t)k * M + code - 1;
    const int leader = __ffsll((unsigned long long)m) - 1;
    const uint32_t kj0 = __shfl(kj, leader, 64);
    const bool same = dup && kj == kj0;
    const uint64_t sm = __ballot(same);
    if ((threadIdx.x & 63) == leader) atomicAdd(&s_dup[kj0], (uint32_t)__popcll(sm));
    if (dup && !same) atomicAdd(&s_dup[kj], 1u);
}

template <int D>
__device__ __forceinline__ void load_pruners_lds(const FilterArgs &a, double *s_pr, int32_t *s_npr, uint32_t *s_dup,
                                                 int ndup_arrays = 1) {
    const int nprw = a.Kp * a.M;
    const int MD = a.M * D;
    if (a.pick_gmin) {
        // k_pick_pruners per workgroup: one wave per partition, lane j = criterion j's sample
        // winner; duplicates keep the first, winners another winner dominates are dropped
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        for (int k = wave; k < a.Kp; k += kThreads / 64) {
            const unsigned long long w = lane < a.M ? a.pick_gmin[k * a.M + lane] : ~0ull;
            const bool has = (uint32_t)(w >> 48) == a.pick_tag;
            double c[D];
            if (has) {
                const uint32_t i = (uint32_t)(((uint64_t)(uint32_t)(w & 0xffffu) * a.n) / a.pick_S);
#pragma unroll
                for (int d = 0; d < D; d++) c[d] = a.vals[(size_t)i * D + d];
            } else {
#pragma unroll
                for (int d = 0; d < D; d++) c[d] = 0.0;
            }
            const uint64_t hm = __ballot(has);
            bool ok = has;
            for (int q = 0; q < a.M; q++) {
                bool le = true, lt = false, eq = true;
#pragma unroll
                for (int d = 0; d < D; d++) {
                    const double x = __shfl(c[d], q, 64);
                    le &= x <= c[d];
                    lt |= x < c[d];
                    eq &= x == c[d];
                }
                if (q != lane && ((hm >> q) & 1ull) && ((le && lt) || (eq && q < lane))) ok = false;
            }
            const uint64_t b = __ballot(ok);
            if (ok) {
                const int pos = (int)lanes_below(b);
#pragma unroll
                for (int d = 0; d < D; d++) {
                    s_pr[k * pr_stride<D>(a.M) + pr_off<D>(k, pos, d)] = c[d];
                    if (blockIdx.x == 0) a.pruners_w[((size_t)k * a.M + pos) * D + d] = c[d];
                }
            }
            if (lane == 0) {
                s_npr[k] = __popcll(b);
                if (blockIdx.x == 0) a.npr_w[k] = __popcll(b);
            }
        }
        for (int q = threadIdx.x; q < nprw * ndup_arrays; q += kThreads) s_dup[q] = 0;
        __syncthreads();
        return;
    }
    for (int q = threadIdx.x; q < nprw * D; q += kThreads) {
        const int k = q / MD, r = q - k * MD;
        s_pr[k * pr_stride<D>(a.M) + pr_off<D>(k, r / D, r % D)] = a.pruners[q];
    }
    for (int q = threadIdx.x; q < a.Kp; q += kThreads) s_npr[q] = a.npr[q];
    for (int q = threadIdx.x; q < nprw * ndup_arrays; q += kThreads) s_dup[q] = 0;
    __syncthreads();
}

// The HBM stream.  MR-Angle keys the fast path cannot certify are appended to a
// deferred list and finished by k_filter_deferred, so this kernel carries no
// exact-fdlibm code (no call, no scratch, fewer VGPRs).
//
// Memory-pipeline rules this loop is built around (gfx950):
//  * the row of item r+1 is in flight while item r is classified, and NOTHING else
//    issued in the loop is a vector-memory op that a later wait must cover, except
//    the status store of item r-1, issued together with that prefetch (vmcnt counts
//    loads and stores together, in issue order: a store issued after the prefetch
//    would make every wait for the row also wait for the store's acknowledgement);
//  * every load is unconditional (row index clamped into [0, n)), so the prefetch
//    registers never merge with a not-loaded path (no copies that wait for them);
//  * waves_per_eu(6) caps the allocation at 80 VGPRs (72 in practice: 7 waves per
//    SIMD), +5 % over the 81-VGPR default allocation (5 waves).  Row loads as whole 1 KB pieces transposed
//    through LDS (full lines per instruction) measured 1.5 % SLOWER, at the lower
//    occupancy their LDS image allows: the row-per-lane loads are not the limit.
// Candidates (partition << 16 | offset) fill each wave's LDS list from the front,
// deferred offsets from the back; the tile reserves its slots with one atomic.
#ifndef SKY_FILTER_FT
#define SKY_FILTER_FT 1           // output tiles per k_filter iteration (A/B builds)
#endif
constexpr int kFilterFT = SKY_FILTER_FT;
#ifndef SKY_FILTER_PF2
#define SKY_FILTER_PF2 0          // 1: two rows in flight per lane (A/B builds)
#endif
#ifndef SKY_FILTER_WPE
#define SKY_FILTER_WPE 6          // waves per SIMD the register budget is sized for: 6 (80 VGPRs) -3.5 % vs 7, 8 +2 %
#endif
template <int D, bool GIVEN>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(D <= 8 ? SKY_FILTER_WPE : 1))) void k_filter(FilterArgs a) {
    // one iteration = a span of kFilterFT output tiles (kFilterFT * 2048 tuples): one candidate
    // reservation, one histogram flush and three barriers per span
    constexpr int FT = kFilterFT;
    constexpr int kSpan = FT * kTile;
    constexpr int kSpanItems = FT * kItems;                      // items per thread per span
    constexpr int kList = kSpanItems * 64;                       // list entries per wave
    extern __shared__ __attribute__((aligned(16))) double s_pr[];   // pruner image (pr_stride), then [FT][Kp*M] u32 dup counts
    uint32_t *s_dup = reinterpret_cast<uint32_t *>(s_pr + (size_t)a.Kp * pr_stride<D>(a.M));
    __shared__ int32_t s_npr[kMaxK];
    __shared__ uint32_t s_list[kSpan];
    __shared__ uint32_t s_wc[kThreads / 64], s_wd[kThreads / 64], s_base, s_dbase;
    load_pruners_lds<D>(a, s_pr, s_npr, s_dup, FT);
    uint32_t lflags = 0;
    uint64_t o = 0, an = ~0ull;                                  // OR / AND of the appended sort keys
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t *wlist = s_list + __builtin_amdgcn_readfirstlane(wave) * kList;
    const uint32_t nl = a.n - 1;
    const uint32_t ntiles = (a.n + kTile - 1) / kTile;
    const uint32_t nspans = (a.n + kSpan - 1) / kSpan;
    const int KM = a.Kp * a.M;
    // status planes (a.planes): per (item, wave) of a tile one 64-bit B word (the tuple is a
    // duplicate of the designated group a.dom_kj) and one E word (its status word is stored);
    // every other tuple is dropped and stores nothing
    const bool planes = a.planes != nullptr;
    // the designated group's status word (never equal to a stored word when there is none)
    const uint32_t sg = a.dom_kj >= 0 ? ((uint32_t)(a.dom_kj / a.M) << 8) | (uint32_t)(1 + a.dom_kj % a.M) : 0x10000u;
    double vn[D];                                                // the row of item r+1, in flight
    int32_t kn = 0;
#ifdef SKY_MEASURE
    uint32_t n_stored = 0;                                       // status words stored (planes on)
#endif
#define SKY_FILTER_FETCH_TO(I, VN, KN)                                                     \
    do {                                                                                   \
        const uint32_t i_ = min((uint32_t)(I), nl);                                        \
        load_row<D>(a.vals + (size_t)i_ * D, VN);                                          \
        if constexpr (GIVEN) KN = a.given_keys[i_];                                        \
    } while (0)
#if SKY_FILTER_PF2
    double vn2[D];                                               // the row of item r+2, in flight
    int32_t kn2 = 0;
#define SKY_FILTER_FETCH(I)                                                                \
    do {                                                                                   \
        SKY_FILTER_FETCH_TO(I, vn, kn);                                                    \
        SKY_FILTER_FETCH_TO((I) + kThreads, vn2, kn2);                                     \
    } while (0)
#else
#define SKY_FILTER_FETCH(I) SKY_FILTER_FETCH_TO(I, vn, kn)
#endif
    // a.tpb tiles per workgroup, interleaved over the grid (tile = t * grid + block): the
    // pruner image is loaded once per workgroup, not once per 2048 tuples
    SKY_FILTER_FETCH(blockIdx.x * kSpan + threadIdx.x);
#pragma unroll 1
    for (uint32_t span = blockIdx.x; span < nspans; span += gridDim.x) {
    uint32_t wcnt = 0, dcnt = 0;
    const uint32_t base = span * kSpan;
    uint16_t st_prev = 0;
#pragma unroll 1
    for (int r = 0; r < kSpanItems; r++) {
        const uint32_t i = base + r * kThreads + threadIdx.x;
        const bool valid = i < a.n;
        double v[D];
#pragma unroll
        for (int d = 0; d < D; d++) v[d] = vn[d];
        const int32_t kg = kn;
        if (r > 0 && !(a.dbg & 2)) {                                    // item r-1, beside the prefetch
            const bool vp = i - kThreads < a.n;
            if (!planes) {
                if (vp) a.status[i - kThreads] = st_prev;
            } else {
                // planes from the stored word alone (no extra live registers in the loop)
                const bool dg = vp && (uint32_t)st_prev == sg, ex = vp && (st_prev & 0xffu) != kCodeDropped && !dg;
                const uint64_t bm = __ballot(dg), em = __ballot(ex);
                if (ex) a.status[i - kThreads] = st_prev;
#ifdef SKY_MEASURE
                n_stored += (uint32_t)__popcll(em);
#endif
                if (lane == 0)
                    reinterpret_cast<ulonglong2 *>(a.planes)[((size_t)span * FT + (r - 1) / kItems) * 32 +
                                                             ((r - 1) % kItems) * (kThreads / 64) + wave] =
                        make_ulonglong2(bm, em);
            }
        }
#if SKY_FILTER_PF2
#pragma unroll
        for (int d = 0; d < D; d++) vn[d] = vn2[d];
        kn = kn2;
        SKY_FILTER_FETCH_TO(r + 2 < kSpanItems ? i + 2 * kThreads : i, vn2, kn2);
#else
        SKY_FILTER_FETCH(r + 1 < kSpanItems ? i + kThreads : i);       // past the span: a cache hit
#endif
        if (a.dbg & 3) {             // measurement only (SKY_FILTER_DBG=1): the stream without the work
            double acc = 0;
#pragma unroll
            for (int d = 0; d < D; d++) acc += v[d];
            st_prev = acc == 1234.5 ? 1 : 0;
            continue;
        }
        int32_t k = GIVEN ? kg : a.single ? 0 : partition_key_fast<D>(v, a.kp);
        // NaN fails the MR-Angle fast path and every pruner compare: it is looked for only
        // where a tuple comes out undecided, out of the queried keys or a candidate
        const bool undecided = !GIVEN && !a.single && k == kAngleUndecided;
        const bool nan = undecided && any_nan<D>(v);
        const bool defer = valid && undecided && !nan;
        const uint64_t dm = __ballot(defer);
        if (defer) wlist[kList - 1 - (dcnt + lanes_below(dm))] = i - base;
        dcnt += (uint32_t)__popcll(dm);
        bool cand = false;
        // deferred: kCodeDeferred, rewritten by k_filter_deferred (a stored word under planes)
        uint16_t st = defer ? kCodeDeferred : (uint16_t)0;
        if (valid && !defer) {
            uint16_t code = kCodeCandidate;
            if (nan) { lflags |= kFlagNaN; code = kCodeDropped; k = 0; }
            else if (k < 0 || k >= a.Kp) {
                if (any_nan<D>(v)) lflags |= kFlagNaN;
                code = kCodeDropped;
                k = 0;
            } else {
                code = classify<D>(v, k, s_pr, s_npr, a.M, lflags);
                if (code == kCodeCandidate && any_nan<D>(v)) { lflags |= kFlagNaN; code = kCodeDropped; k = 0; }
            }
            cand = code == kCodeCandidate;
            st = (uint16_t)(((uint32_t)k << 8) | code);
        }
        count_dups((uint16_t)(defer ? 0u : (st & 0xffu)), (int32_t)(st >> 8), a.M,
                   s_dup + (FT > 1 ? (r / kItems) * KM : 0));
        const uint64_t cm = __ballot(cand);
        if (cand) wlist[wcnt + lanes_below(cm)] = ((uint32_t)k << 16) | (i - base);
        wcnt += (uint32_t)__popcll(cm);
        st_prev = st;
    }
    if (!(a.dbg & 2)) {
        const uint32_t il = base + (kSpanItems - 1) * kThreads + threadIdx.x;
        const bool vp = il < a.n;
        if (!planes) {
            if (vp) a.status[il] = st_prev;
        } else {
            const bool dg = vp && (uint32_t)st_prev == sg, ex = vp && (st_prev & 0xffu) != kCodeDropped && !dg;
            const uint64_t bm = __ballot(dg), em = __ballot(ex);
            if (ex) a.status[il] = st_prev;
#ifdef SKY_MEASURE
            n_stored += (uint32_t)__popcll(em);
#endif
            if (lane == 0)
                reinterpret_cast<ulonglong2 *>(a.planes)[((size_t)span * FT + FT - 1) * 32 +
                                                         (kItems - 1) * (kThreads / 64) + wave] =
                    make_ulonglong2(bm, em);
        }
    }
    // the tile's candidates: ONE slot reservation per tile, then rows re-read (cache
    // hot) and appended with their sort keys
    if (lane == 0) { s_wc[wave] = wcnt; s_wd[wave] = dcnt; }
    __syncthreads();
    uint32_t woff[kThreads / 64 + 1], doff[kThreads / 64 + 1];
    woff[0] = 0;
    doff[0] = 0;
#pragma unroll
    for (int q = 0; q < kThreads / 64; q++) {
        woff[q + 1] = woff[q] + s_wc[q];
        doff[q + 1] = doff[q] + s_wd[q];
    }
    const uint32_t total = woff[kThreads / 64], dtotal = doff[kThreads / 64];
    // the tile's duplicate counts: into the per-tile histogram (the output count reads it
    // instead of the status words) and the per-(partition, pruner) totals
    for (int fq = threadIdx.x; fq < FT * KM; fq += kThreads) {
        const int f = FT > 1 ? fq / KM : 0, q = fq - f * KM;
        const uint32_t c = s_dup[fq];
        const uint32_t tile = span * FT + f;
        if (a.tile_hist && tile < ntiles) a.tile_hist[(size_t)tile * KM + q] = c;
        if (c) {
            if (!(a.dbg & 4)) atomicAdd(&a.dup_cnt[q], c);      // (SKY_FILTER_DBG & 4: no global atomics)
            s_dup[fq] = 0;
        }
    }
    if (threadIdx.x == 0) s_base = total && !(a.dbg & 4) ? atomicAdd(a.m_total, total) : 0u;
    if (threadIdx.x == 64 && dtotal) s_dbase = atomicAdd(a.defer_cnt, dtotal);
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < dtotal; q += kThreads) {
        int w = 0;
#pragma unroll
        for (int t = 1; t < kThreads / 64; t++) w += q >= doff[t] ? 1 : 0;
        a.defer_list[s_dbase + q] = base + s_list[w * kList + kList - 1 - (q - doff[w])];
    }
    for (uint32_t q = threadIdx.x; q < total; q += kThreads) {
        int w = 0;
#pragma unroll
        for (int t = 1; t < kThreads / 64; t++) w += q >= woff[t] ? 1 : 0;
        const uint32_t e = s_list[w * kList + (q - woff[w])];
        const uint32_t i = base + (e & 0xffffu);
        const uint32_t k = e >> 16;
        double v[D];
        load_row<D>(a.vals + (size_t)i * D, v);
        const uint32_t slot = s_base + q;
        if (slot >= a.slot_cap) continue;      // counted; the host re-runs with more slots
        constexpr int DP = padded_dims<double>(D);
        store_row<double, D>(a.crow + (size_t)slot * DP, v);
        const uint64_t key = make_sortkey<double, D>(v, k, lflags);
        a.sortkey[slot] = key;
        a.slot_src[slot] = i;
        o |= key;
        an &= key;
    }
    // the next tile's first row, in flight over the barrier (not over the candidate appends
    // above: the row registers live across them spilled to scratch, and every scratch
    // reload's vmcnt wait then also waited for the prefetch)
    SKY_FILTER_FETCH((span + gridDim.x) * kSpan + threadIdx.x);
    __syncthreads();                           // s_list / s_wc reused by the next span
    }
#undef SKY_FILTER_FETCH
#undef SKY_FILTER_FETCH_TO
    // OR / AND of the appended sort keys (they size the radix sort): one atomic pair per wave
    // that appended any, at the end (no per-tile barrier, table or reduce kernel)
#pragma unroll
    for (int sh = 32; sh >= 1; sh >>= 1) {
        o |= __shfl_xor(o, sh, 64);
        an &= __shfl_xor(an, sh, 64);
    }
    if (lane == 0 && o != 0ull) {
        atomicOr(a.orand, (unsigned long long)o);
        atomicAnd(a.orand + 1, (unsigned long long)an);
    }
    if (lflags) atomicOr(a.flags, lflags);
#ifdef SKY_MEASURE
    if (lane == 0 && n_stored) atomicAdd(a.flags + 8, n_stored);   // measurement builds: flags[8]
#endif
}

// The deferred MR-Angle tuples: exact fdlibm key, then the same classification;
// per-tile candidate counts are added atomically (before the scan).
template <int D>
__global__ __launch_bounds__(kThreads) void k_filter_deferred(FilterArgs a) {
    extern __shared__ __attribute__((aligned(16))) double s_pr[];
    uint32_t *s_dup = reinterpret_cast<uint32_t *>(s_pr + (size_t)a.Kp * pr_stride<D>(a.M));
    __shared__ int32_t s_npr[kMaxK];
    load_pruners_lds<D>(a, s_pr, s_npr, s_dup);
    const uint32_t cnt = *a.defer_cnt;
    uint32_t lflags = 0;
    uint64_t o = 0, an = ~0ull;
    const uint32_t span = (cnt + gridDim.x * kThreads - 1) / (gridDim.x * kThreads) * (gridDim.x * kThreads);
    for (uint32_t q = blockIdx.x * kThreads + threadIdx.x; q < span; q += gridDim.x * kThreads) {
        const bool valid = q < cnt;                       // every lane runs the wave-wide append
        const uint32_t i = valid ? a.defer_list[q] : 0u;
        double v[D];
        int32_t k = 0;
        bool cand = false;
        uint16_t code = kCodeDropped;
        if (valid) {
            load_row<D>(a.vals + (size_t)i * D, v);
            k = angle_key_exact<D>(v, a.kp.P);
            if (k < 0 || k >= a.Kp) { code = kCodeDropped; k = 0; }
            else code = classify<D>(v, k, s_pr, s_npr, a.M, lflags);
            cand = code == kCodeCandidate;
            a.status[i] = (uint16_t)(((uint32_t)k << 8) | code);
        } else {
#pragma unroll
            for (int d = 0; d < D; d++) v[d] = 0.0;
        }
        count_dups(code, k, a.M, s_dup);
        if (a.tile_hist && valid && code != kCodeCandidate && code != kCodeDropped)
            atomicAdd(&a.tile_hist[(size_t)(i / kTile) * (a.Kp * a.M) + (uint32_t)k * a.M + code - 1], 1u);
        append_candidate<D>(a, cand, v, k, i, lflags, o, an);
    }
#pragma unroll
    for (int sh = 32; sh >= 1; sh >>= 1) {
        o |= __shfl_xor(o, sh, 64);
        an &= __shfl_xor(an, sh, 64);
    }
    if ((threadIdx.x & 63) == 0 && o != 0ull) {
        atomicOr(a.orand, (unsigned long long)o);
        atomicAnd(a.orand + 1, (unsigned long long)an);
    }
    __syncthreads();
    for (int q = threadIdx.x; q < a.Kp * a.M; q += kThreads)
        if (s_dup[q]) atomicAdd(&a.dup_cnt[q], s_dup[q]);
    if (lflags) atomicOr(a.flags, lflags);
}

// Blocked tile layout for the status-word passes: thread t of tile b owns the
// kItems CONSECUTIVE tuples b*kTile + t*kItems ...; its 8 status words are one
// 16-byte load, and index order inside the tile is (thread, item) order, so one
// block-wide exclusive scan per tile gives order-preserving ranks.
__device__ __forceinline__ void load_status8(const uint16_t *__restrict__ status, uint32_t n, uint32_t i0,
                                             uint16_t (&st)[kItems]) {
    // the status array is allocated to whole tiles (engine.hip), so one clamped
    // 16-byte load always stays inside it: no partial-tile branch, whose merge
    // would make the loads of consecutive tiles wait for each other
    const uint32_t ic = min(i0, (n + kTile - 1) / kTile * kTile - kItems);
    const uint4 q = *reinterpret_cast<const uint4 *>(status + ic);
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int k = 0; k < 4; k++) {
        st[2 * k] = i0 + 2 * k < n ? (uint16_t)(w[k] & 0xffffu) : (uint16_t)0;
        st[2 * k + 1] = i0 + 2 * k + 1 < n ? (uint16_t)(w[k] >> 16) : (uint16_t)0;
    }
}

__device__ __forceinline__ uint32_t block_scan_excl(uint32_t v, uint32_t *s_w, uint32_t &total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    uint32_t wb = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kThreads / 64; i++) {
        const uint32_t c = s_w[i];
        wb += i < w ? c : 0u;
        tot += c;
    }
    __syncthreads();
    total = tot;
    return wb + inc - v;
}



// One workgroup: every pruner that some tuple duplicates becomes one more candidate
// slot (m + e) carrying that duplicate group; builds entries[e] = k*M+j and
// pruner_slot[k*M+j] on the device (no host round trip).
template <typename T, int D>
__device__ __forceinline__ uint64_t emit_pruner(const double *pr, uint32_t part, T *rows_t, uint32_t slot,
                                                uint64_t *sortkey, uint32_t &lflags) {
    constexpr int DP = padded_dims<T>(D);
    T tv[D];
#pragma unroll
    for (int d = 0; d < D; d++) {
        tv[d] = (T)pr[d];
        // a duplicated pruner is a slot like any candidate: its values decide the row type too
        if ((double)(float)pr[d] != pr[d]) lflags |= kFlagNotF32;
    }
    store_row<T, D>(rows_t + (size_t)slot * DP, tv);
    const uint64_t key = make_sortkey<T, D>(tv, part, lflags);
    sortkey[slot] = key;
    return key;
}

template <int D>
__global__ __launch_bounds__(kThreads) void k_append_pruners(AppendArgs a) {
    __shared__ uint32_t s_w[kThreads / 64];
    const uint32_t m = *a.m_total;
    const int KM = a.Kp * a.M;
    uint32_t run = 0, lflags = 0;
    uint64_t o = 0, an = ~0ull;
    for (int q0 = 0; q0 < KM; q0 += kThreads) {
        const int q = q0 + threadIdx.x;
        const bool has = q < KM && a.dup_cnt[q] > 0;
        uint32_t tot;
        const uint32_t e = run + block_scan_excl(has ? 1u : 0u, s_w, tot);
        if (has) {
            const uint32_t slot = m + e;
            a.entries[e] = q;
            a.pruner_slot[q] = (int32_t)slot;
            if (slot < a.slot_cap) {             // past it: the host re-runs with more slots
                a.slot_src[slot] = 0x80000000u | e;
                const double *pr = a.pruners + (size_t)q * D;
                const uint64_t key = emit_pruner<double, D>(pr, q / a.M, (double *)a.rows, slot, a.sortkey, lflags);
                o |= key;
                an &= key;
            }
        } else if (q < KM) {
            a.pruner_slot[q] = -1;
        }
        run += tot;
    }
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) {
        o |= __shfl_xor(o, s, 64);
        an &= __shfl_xor(an, s, 64);
    }
    if ((threadIdx.x & 63) == 0 && run) {
        atomicOr(&a.orand[0], (unsigned long long)o);
        atomicAnd(&a.orand[1], (unsigned long long)an);
    }
    if (lflags) atomicOr(a.flags, lflags);
    if (threadIdx.x == 0) {
        *a.nps_total = run;
        if (a.mt_total) *a.mt_total = min(m + run, a.slot_cap);   // slots written (device-sized launches)
    }
}

// ---- candidate prefilter: second-level pruners drawn from the candidates ------------
// The first-level pruners come from a 65536-tuple sample (<= 8 per partition, they live in
// k_filter's LDS).  The candidates that survive them are far closer to each partition's
// skyline, so per partition up to M2 (<= 64) candidates minimising positive-weight linear
// criteria (never dominated among the candidates: skyline points, up to the f32 rounding of
// the criterion, re-checked exactly below) prune every other candidate of that partition by
// one brute-force pass (|candidates| x M2 pair tests) before the sort.  A candidate they
// dominate is outside L_k; equal vectors are never dropped.  Exactness: dominance in f64.
// Criterion j: a positive-weight sum.  Base weights spread the winners along the front
// (j % 16 == 0: the plain sum; 1..D: one dimension weighted 4x, pulling towards a corner;
// above: pairs), plus a small deterministic perturbation (< 1e-4 per weight) that breaks the
// ties of integer-valued data by a fixed secondary order instead of by the (unordered) slot
// order; criteria j and j + 16 share the base and differ in the tie-break.
__device__ __forceinline__ float cand_eps(int j, int d) {
    uint32_t h = (uint32_t)((j + 1) * 0x9E3779B1u) ^ (uint32_t)((d + 1) * 0x85EBCA77u);
    h ^= h >> 15;
    h *= 0x2C1B3C6Du;
    h ^= h >> 12;
    return (float)(h >> 8) * (1e-4f / 16777216.0f);
}
__device__ __forceinline__ float cand_weight(int j, int d, int D) {
    const int b = j & 15;
    int da = -1, db = -1;
    if (b >= 1 && b <= D) da = b - 1;
    else if (b > D) { da = (b - 1) % D; db = (b - 1 + 1 + (b - 1) / D) % D; }
    return 1.0f + (d == da ? 3.0f : 0.0f) + (d == db ? 3.0f : 0.0f) + cand_eps(j, d);
}

// The weights are row-independent: computed once per workgroup into LDS (read back as
// broadcasts), and a slot only issues the LDS atomicMin when it beats the value it reads
// (the minima settle after a few rows, so most slots issue none)
template <int D>
__global__ __launch_bounds__(kThreads) void k_cand_min(const double *__restrict__ rows, const uint64_t *__restrict__ key,
                                                       uint32_t mt, const uint32_t *__restrict__ d_mt, int Kp,
                                                       int M2, unsigned long long *__restrict__ gmin) {
    constexpr int DP = padded_dims<double>(D);
    if (d_mt) mt = min(mt, *d_mt);             // device-sized launch: mt is the bound
    __shared__ unsigned long long s_min[2048];
    __shared__ float s_w[64][D];
    const int KM = Kp * M2;
    for (int q = threadIdx.x; q < KM; q += kThreads) s_min[q] = ~0ull;
    for (int q = threadIdx.x; q < M2 * D; q += kThreads) s_w[q / D][q % D] = cand_weight(q / D, q % D, D);
    __syncthreads();
    // two rows per thread and iteration, both loads issued before either is used
    const uint32_t stride = gridDim.x * kThreads;
    for (uint32_t j0 = blockIdx.x * kThreads + threadIdx.x; j0 < mt; j0 += 2 * stride) {
        double v[2][D];
        int k[2];
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const uint32_t jc = min(j0 + u * stride, mt - 1u);
            k[u] = (int)(key[jc] >> 56);
            load_trow<double, D>(rows + (size_t)jc * DP, v[u]);
        }
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const uint32_t j = j0 + u * stride;
            if (j >= mt) break;
            float f[D];
#pragma unroll
            for (int d = 0; d < D; d++) f[d] = (float)v[u][d];
            for (int c = 0; c < M2; c++) {
                float cv = 0.0f;
#pragma unroll
                for (int d = 0; d < D; d++) cv += s_w[c][d] * f[d];
                if (cv != cv) continue;
                const unsigned long long e = ((unsigned long long)f32_order_key(cv) << 32) | j;
                unsigned long long *m = &s_min[k[u] * M2 + c];
                if (e < *m) atomicMin(m, e);
            }
        }
    }
    __syncthreads();
    // the global minima: every workgroup's value for one address serialises at L2, so a
    // workgroup only adds its own when it beats what is already there
    for (int q = threadIdx.x; q < KM; q += kThreads)
        if (s_min[q] != ~0ull && s_min[q] < __hip_atomic_load(&gmin[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            atomicMin(&gmin[q], s_min[q]);
}

// one 64-lane workgroup per partition: winners deduplicated and mutually non-dominated
template <int D>
__global__ __launch_bounds__(64) void k_cand_pick(const double *__restrict__ rows,
                                                  const unsigned long long *__restrict__ gmin, int M2,
                                                  double *__restrict__ pr2, int32_t *__restrict__ npr2) {
    constexpr int DP = padded_dims<double>(D);
    __shared__ double s_c[64][D];
    __shared__ int s_ok[64];
    const int k = blockIdx.x, j = threadIdx.x;
    const unsigned long long w = j < M2 ? gmin[k * M2 + j] : ~0ull;
    const bool has = w != ~0ull;
    if (has) {
        const uint32_t slot = (uint32_t)(w & 0xffffffffu);
#pragma unroll
        for (int d = 0; d < D; d++) s_c[j][d] = rows[(size_t)slot * DP + d];
    }
    s_ok[j] = has ? 1 : 0;
    __syncthreads();
    bool ok = has;
    for (int q = 0; q < M2 && ok; q++) {
        if (q == j || !s_ok[q]) continue;
        bool le = true, lt = false, eq = true;
#pragma unroll
        for (int d = 0; d < D; d++) {
            le &= s_c[q][d] <= s_c[j][d];
            lt |= s_c[q][d] < s_c[j][d];
            eq &= s_c[q][d] == s_c[j][d];
        }
        if ((le && lt) || (eq && q < j)) ok = false;
    }
    const uint64_t b = __ballot(ok);
    if (ok) {
        const int pos = __popcll(b & (j == 0 ? 0ull : (~0ull >> (64 - j))));
#pragma unroll
        for (int d = 0; d < D; d++) pr2[((size_t)k * M2 + pos) * D + d] = s_c[j][d];
    }
    if (j == 0) npr2[k] = __popcll(b);
}

// live[j] = candidate j is not dominated by a second-level pruner of its partition.  The pruners
// (Kp x M2 rows, <= 2048) are staged in LDS once per workgroup: each lane's partition picks its
// own rows, so global reads would be per-lane gathers (one 8-byte load per pruner and dimension)
template <int D, bool STAGED>
__global__ __launch_bounds__(kThreads) void k_cand_filter(const double *__restrict__ rows,
                                                          const uint64_t *__restrict__ key, uint32_t mt,
                                                          const uint32_t *__restrict__ d_mt, int Kp, int M2,
                                                          const double *__restrict__ pr2,
                                                          const int32_t *__restrict__ npr2,
                                                          uint32_t *__restrict__ live) {
    constexpr int DP = padded_dims<double>(D);
    extern __shared__ __attribute__((aligned(16))) double s_pr2[];   // [Kp * M2][D]
    __shared__ int32_t s_np[kMaxK];
    if (d_mt) mt = min(mt, *d_mt);
    const uint32_t j0 = blockIdx.x * kThreads;
    if (j0 >= mt) return;                          // block-uniform
    if constexpr (STAGED)
        for (int q = threadIdx.x; q < Kp * M2 * D; q += kThreads) s_pr2[q] = pr2[q];
    for (int q = threadIdx.x; q < Kp; q += kThreads) s_np[q] = npr2[q];
    __syncthreads();
    const uint32_t j = j0 + threadIdx.x;
    if (j >= mt) return;
    const int k = (int)(key[j] >> 56);
    double v[D];
    load_trow<double, D>(rows + (size_t)j * DP, v);
    const int np = s_np[k];
    const double *pr = (STAGED ? s_pr2 : pr2) + (size_t)k * M2 * D;
    bool dom = false;
    for (int q = 0; q < np; q++) {
        bool le = true, lt = false;
#pragma unroll
        for (int d = 0; d < D; d++) {
            const double x = pr[q * D + d];
            le &= x <= v[d];
            lt |= x < v[d];
        }
        dom |= le & lt;
    }
    live[j] = dom ? 0u : 1u;
}

// decoupled look-back words: flag (aggregate / inclusive prefix) | count
constexpr unsigned long long kLbAgg = 1ull << 62, kLbInc = 2ull << 62, kLbCount = (1ull << 62) - 1;

// The prefilter's pick, live test, scan and compaction in ONE launch (was: k_cand_pick,
// k_cand_filter, one to three scan kernels, k_cand_compact -- four to six dependent launches of
// 3-6 us each).  Every workgroup redoes the pick (k_cand_pick: one wave per partition, lane =
// criterion winner, shuffles) into LDS; one slot per thread; the tile's exclusive prefix comes
// from a decoupled look-back over the earlier tiles (tiles numbered in start order by a ticket, so a
// tile only waits for tiles already running; bounded spin -> kFlagRadixSpin), which keeps the
// compaction in slot order exactly as the scan + k_cand_compact did.  The appended pruner slots'
// indices are remapped from their entries (a dropped one: -1).
// PICKED (CandArgs::picked, large slot counts): k_cand_pick ran once before and its pr2 / npr2 are
// staged instead, one slot per thread -- at C4's 241k slots the per-workgroup pick over 236
// workgroups of four slots per thread (one per CU) was slower than the launch chain it replaced
template <int D, int FI, bool PICKED>
__global__ __launch_bounds__(kThreads) void k_cand_fused(CandArgs a) {
    constexpr int DP = padded_dims<double>(D);
    constexpr int kCandFI = FI;
    extern __shared__ __attribute__((aligned(16))) double s_pr2[];   // [Kp][M2 * D + 1]
    __shared__ int32_t s_np[kMaxK];
    __shared__ uint32_t s_w[kThreads / 64];
    __shared__ uint32_t s_tile;
    __shared__ unsigned long long s_prefix;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int M2 = a.M2, PS = a.M2 * D + 1;
    // tiles in blockIdx order, as k_out_hist_scan: each XCD dispatches its workgroups in order, so a
    // tile only waits for tiles dispatched before it.  (A ticket -- an atomic per workgroup on one
    // address, serialised at one L2 channel ahead of every workgroup's loads -- cost C4's 943-tile
    // pass 11 us of its 29.)
    if (threadIdx.x == 0) s_tile = blockIdx.x;
    const uint32_t mt = a.d_mt ? min(a.mt, *a.d_mt) : a.mt;
    if constexpr (PICKED) {
        for (int q = threadIdx.x; q < a.Kp * M2 * D; q += kThreads) {
            const int k = q / (M2 * D), r = q - k * (M2 * D);
            s_pr2[k * PS + r] = a.pr2[q];
        }
        for (int k = threadIdx.x; k < a.Kp; k += kThreads) s_np[k] = a.npr2[k];
    }
    for (int k = wave; k < (PICKED ? 0 : a.Kp); k += kThreads / 64) {
        const unsigned long long w = lane < M2 ? a.cmin[k * M2 + lane] : ~0ull;
        const bool has = w != ~0ull;
        double c[D];
        if (has) {
            load_trow<double, D>(a.rows + (size_t)(uint32_t)(w & 0xffffffffu) * DP, c);
        } else {
#pragma unroll
            for (int d = 0; d < D; d++) c[d] = 0.0;
        }
        const uint64_t hm = __ballot(has);
        bool ok = has;
        for (int q = 0; q < M2; q++) {
            bool le = true, lt = false, eq = true;
#pragma unroll
            for (int d = 0; d < D; d++) {
                const double x = __shfl(c[d], q, 64);
                le &= x <= c[d];
                lt |= x < c[d];
                eq &= x == c[d];
            }
            if (q != lane && ((hm >> q) & 1ull) && ((le && lt) || (eq && q < lane))) ok = false;
        }
        const uint64_t b = __ballot(ok);
        if (ok) {
            const int pos = (int)lanes_below(b);
#pragma unroll
            for (int d = 0; d < D; d++) s_pr2[k * PS + pos * D + d] = c[d];
        }
        if (lane == 0) s_np[k] = __popcll(b);
    }
    __syncthreads();
    const uint32_t tile = s_tile;
    // the invariant k_cand_compact keeps: a pruner slot at or past mt (slots truncated) is no slot
    // of this round's index space.  Race-free: no tile rewrites an entry whose slot is >= mt, and
    // an entry below mt stays below it when remapped
    if (tile == 0)
        for (int q = threadIdx.x; q < a.KM; q += kThreads) {
            const int32_t ps = a.pruner_slot[q];
            if (ps >= 0 && (uint32_t)ps >= mt) a.pruner_slot[q] = -1;
        }
    // kCandFI consecutive slots per thread (the tile's order = slot order): the pick above is
    // paid once per kCandFI * kThreads slots
    const uint32_t j0 = (tile * kThreads + threadIdx.x) * kCandFI;
    bool liv[kCandFI];
    double v[kCandFI][D];
    uint64_t kv[kCandFI];
    uint32_t sv[kCandFI];
#pragma unroll
    for (int u = 0; u < kCandFI; u++) {
        const uint32_t jc = min(j0 + u, mt > 0 ? mt - 1u : 0u);
        kv[u] = a.key[jc];
        sv[u] = a.src[jc];
        load_trow<double, D>(a.rows + (size_t)jc * DP, v[u]);
    }
    uint32_t cnt = 0;
#pragma unroll
    for (int u = 0; u < kCandFI; u++) {
        liv[u] = false;
        if (j0 + u < mt) {
            const int k = (int)(kv[u] >> 56);
            const double *pr = s_pr2 + (size_t)k * PS;
            const int np = s_np[k];
            bool dom = false;
            for (int q = 0; q < np; q++) {
                bool le = true, lt = false;
#pragma unroll
                for (int d = 0; d < D; d++) {
                    const double x = pr[q * D + d];
                    le &= x <= v[u][d];
                    lt |= x < v[u][d];
                }
                dom |= le & lt;
            }
            liv[u] = !dom;
            cnt += liv[u] ? 1u : 0u;
        }
    }
    uint32_t bt;
    const uint32_t pl = block_scan_excl(cnt, s_w, bt);
    if (threadIdx.x < 64) {
        unsigned long long excl = 0;
        if (lane == 0)
            __hip_atomic_store(a.lb + tile, (tile == 0 ? kLbInc : kLbAgg) | bt, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        if (tile > 0) {
            int64_t end = (int64_t)tile - 1;
            uint32_t spins = 0;
            for (;;) {
                const int64_t idx = end - lane;
                const unsigned long long svv = idx >= 0 ? __hip_atomic_load(a.lb + idx, __ATOMIC_RELAXED,
                                                                            __HIP_MEMORY_SCOPE_AGENT)
                                                        : kLbInc;
                const unsigned long long f = svv & ~kLbCount;
                const uint64_t inc = __ballot(f == kLbInc), zero = __ballot(f == 0ull);
                const int first = inc ? __ffsll((unsigned long long)inc) - 1 : 64;
                const uint64_t upto = first >= 63 ? ~0ull : ((2ull << first) - 1ull);
                if (zero & upto) {
                    if (++spins > (1u << 22)) {
                        if (lane == 0) atomicOr(a.err, kFlagRadixSpin);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                unsigned long long c = lane <= first ? (svv & kLbCount) : 0ull;
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
                excl += c;
                if (first < 64) break;
                end -= 64;
            }
            if (lane == 0)
                __hip_atomic_store(a.lb + tile, kLbInc | (excl + bt), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) {
            s_prefix = excl;
            if (tile == gridDim.x - 1) *a.d_live = (uint32_t)(excl + bt);
        }
    }
    __syncthreads();
    uint32_t pos = (uint32_t)s_prefix + pl;
#pragma unroll
    for (int u = 0; u < kCandFI; u++) {
        if (liv[u]) {
            store_row<double, D>(a.rows2 + (size_t)pos * DP, v[u]);
            a.key2[pos] = kv[u];
            a.src2[pos] = sv[u];
        }
        if (j0 + u < mt && (sv[u] & 0x80000000u))
            a.pruner_slot[a.entries[sv[u] & 0x7fffffffu]] = liv[u] ? (int32_t)pos : -1;
        pos += liv[u] ? 1u : 0u;
    }
}

// order-preserving compaction of the live slots (rows, keys, sources); the appended
// pruner slots' indices are remapped (a dropped one: its duplicate group's fate is 0)
template <int D>
__global__ __launch_bounds__(kThreads) void k_cand_compact(uint32_t mt, const uint32_t *__restrict__ d_mt,
                                                           const uint32_t *__restrict__ live,
                                                           const uint32_t *__restrict__ pos,
                                                           const double *__restrict__ rows,
                                                           const uint64_t *__restrict__ key,
                                                           const uint32_t *__restrict__ src, double *__restrict__ rows2,
                                                           uint64_t *__restrict__ key2, uint32_t *__restrict__ src2,
                                                           int32_t *__restrict__ pruner_slot, int KM) {
    constexpr int DP = padded_dims<double>(D);     // even: rows move as 16-byte pieces
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (d_mt) mt = min(mt, *d_mt);
    if (j < mt && live[j]) {
        const uint32_t o = pos[j];
        const double2 *s2 = reinterpret_cast<const double2 *>(rows + (size_t)j * DP);
        double2 *d2 = reinterpret_cast<double2 *>(rows2 + (size_t)o * DP);
        double2 t[DP / 2];
#pragma unroll
        for (int q = 0; q < DP / 2; q++) t[q] = s2[q];
#pragma unroll
        for (int q = 0; q < DP / 2; q++) d2[q] = t[q];
        key2[o] = key[j];
        src2[o] = src[j];
    }
    if (j < (uint32_t)KM) {
        const int32_t ps = pruner_slot[j];
        if (ps >= 0) pruner_slot[j] = (uint32_t)ps < mt && live[ps] ? (int32_t)pos[ps] : -1;
    }
}

// ---- duplicate collapse after the sort --------------------------------------
template <typename T, int D>
__global__ __launch_bounds__(kThreads) void k_gather_runs(RepArgs a) {
    constexpr int DP = padded_dims<T>(D);
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= a.mt) return;
    // slot rows are f64 (written by the filter before the row type was known)
    const double *src = reinterpret_cast<const double *>(a.rows) + (size_t)a.perm[j] * padded_dims<double>(D);
    T *dst = reinterpret_cast<T *>(a.rows_sorted) + (size_t)j * DP;
    double dv[D];
    load_trow<double, D>(src, dv);
    T v[D];
#pragma unroll
    for (int d = 0; d < D; d++) v[d] = (T)dv[d];
    store_row<T, D>(dst, v);
    a.runflag[j] = (j == 0 || a.skey[j] != a.skey[j - 1]) ? 1u : 0u;
}

__global__ __launch_bounds__(kThreads) void k_run_first(RepArgs a) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= a.mt) return;
    if (a.runflag[j]) a.run_first[a.runscan[j]] = j;
}

template <typename T, int D>
__global__ __launch_bounds__(kThreads) void k_rep_of(RepArgs a) {
    constexpr int DP = padded_dims<T>(D);
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= a.mt) return;
    const T *rs = reinterpret_cast<const T *>(a.rows_sorted);
    T v[D];
    load_trow<T, D>(rs + (size_t)j * DP, v);
    const uint32_t s0 = a.run_first[a.runscan[j] + a.runflag[j] - 1];
    uint32_t q = s0;
    for (; q < j; q++) {
        T u[D];
        load_trow<T, D>(rs + (size_t)q * DP, u);
        if (rows_equal<D, T>(u, v)) break;
    }
    a.repof[j] = q;
    a.repflag[j] = q == j ? 1u : 0u;
}

template <typename T, int D>
__global__ __launch_bounds__(kThreads) void k_build_reps(RepArgs a) {
    constexpr int DP = padded_dims<T>(D);
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= a.mt) return;
    const uint32_t r = a.repscan[a.repof[j]];
    a.rep_of_sorted[j] = r;
    a.slot_rep[a.perm[j]] = r;
    if (a.repflag[j]) {
        T v[D];
        load_trow<T, D>(reinterpret_cast<const T *>(a.rows_sorted) + (size_t)j * DP, v);
        store_row<T, D>(reinterpret_cast<T *>(a.rep_rows) + (size_t)r * DP, v);
        a.rep_key[r] = a.skey[j];
    }
}

__global__ __launch_bounds__(kThreads) void k_seg_bounds(const uint64_t *__restrict__ rep_key,
                                                         const uint32_t *__restrict__ d_mr,
                                                         uint32_t *__restrict__ seg_begin,
                                                         uint32_t *__restrict__ seg_end) {
    const uint32_t r = blockIdx.x * kThreads + threadIdx.x;
    const uint32_t mr = *d_mr;
    if (r >= mr) return;
    const uint32_t p = (uint32_t)(rep_key[r] >> 56);
    if (r == 0 || (uint32_t)(rep_key[r - 1] >> 56) != p) seg_begin[p] = r;
    if (r == mr - 1 || (uint32_t)(rep_key[r + 1] >> 56) != p) seg_end[p] = r + 1;
}

__global__ __launch_bounds__(kThreads) void k_rep_mult(uint32_t mt, const uint32_t *__restrict__ perm,
                                                       const uint32_t *__restrict__ slot_src,
                                                       const uint32_t *__restrict__ rep_of_sorted,
                                                       const int64_t *__restrict__ given_w,
                                                       const uint32_t *__restrict__ dup_cnt,
                                                       const int32_t *__restrict__ pr_entries,
                                                       unsigned long long *__restrict__ mult) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= mt) return;
    const uint32_t src = slot_src[perm[j]];
    unsigned long long w;
    if (src & 0x80000000u) w = dup_cnt[pr_entries[src & 0x7fffffffu]];
    else w = given_w ? (unsigned long long)given_w[src] : 1ull;
    atomicAdd(&mult[rep_of_sorted[j]], w);
}

// ---- output: per tuple local / global membership ------------------------------
// fate = inL | inG << 1.  A candidate's fate is written into its own status word
// (code kCodeFate0 + fate, from its slot's representative), a duplicate group's per
// (partition, pruner) into pruner_fate, so the per-tuple passes read the status
// word and at most one LDS byte: no dependent global lookups.
//
// Stats (|L_k|, survivors_k) for unit weights and computed origins: every stream
// tuple in L_k is a candidate (one slot, weight 1) or a duplicate of a pruner
// (weight dup_cnt), so they are summed over slots here instead of over tuples.
__device__ __forceinline__ uint32_t fate_from_domf(const FateArgs &a, uint32_t r) {
    const uint32_t df = a.domf[r];
    const bool in_l = !(df & 1u), in_g = a.gmerge ? !(df & 2u) : in_l;
    return (in_l ? 1u : 0u) | (in_g ? 2u : 0u);
}

__global__ __launch_bounds__(kThreads) void k_fate_tables(FateArgs a) {
    __shared__ unsigned long long s_l[kMaxK], s_s[kMaxK];
    __shared__ uint32_t s_n[kMaxK], s_a[kMaxK];
    const bool stats = a.lsz != nullptr, fin = a.domf != nullptr;
    if (stats || fin) {
        if (stats)
            for (int q = threadIdx.x; q < a.K; q += kThreads) { s_l[q] = 0; s_s[q] = 0; }
        if (fin)
            for (int q = threadIdx.x; q < kMaxK; q += kThreads) { s_n[q] = 0; s_a[q] = 0; }
        __syncthreads();
    }
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    const uint32_t mtd = a.d_mt ? min(a.mt, *a.d_mt) : a.mt;   // device-sized: a.mt is the bound
    uint32_t cand_tile = 0xffffffffu;          // a candidate in G: its stream tile (output counts)
    int k = -1;
    unsigned long long w = 0;
    uint32_t f = 0;
    if (j < a.mt) {
        if (fin && j < mtd) {                          // k_brute_finish's outputs for slot j
            const uint32_t fj = fate_from_domf(a, j);
            const uint32_t kk = (uint32_t)(a.key[j] >> 56);
            a.alive_l_w[j] = (uint8_t)(fj & 1u);
            a.alive_g_w[j] = (uint8_t)(fj >> 1);
            a.slot_rep_w[j] = j;
            atomicAdd(&s_n[kk], 1u);
            if (fj & 1u) atomicAdd(&s_a[kk], 1u);
        }
        const uint32_t src = j < mtd ? a.slot_src[j] : 0x80000000u;
        if (!(src & 0x80000000u)) {                    // (appended pruner slots: below)
            if (fin) {
                f = fate_from_domf(a, j);
            } else {
                const uint32_t r = a.slot_rep[j];
                f = (a.alive_l[r] ? 1u : 0u) | (a.alive_g[r] ? 2u : 0u);
            }
            const uint16_t s0 = a.status[src];
            a.status[src] = (uint16_t)((s0 & 0xff00u) | (kCodeFate0 + f));
            cand_tile = (f & 2u) ? src / kTile : 0xffffffffu;
            k = s0 >> 8;
            w = 1;
        }
    } else if (j - a.mt < (uint32_t)a.KM) {
        const uint32_t q = j - a.mt;
        const int32_t ps = a.pruner_slot[q];
        if (ps >= 0 && (uint32_t)ps < mtd) {
            if (fin) {
                f = fate_from_domf(a, (uint32_t)ps);
            } else {
                const uint32_t r = a.slot_rep[ps];
                f = (a.alive_l[r] ? 1u : 0u) | (a.alive_g[r] ? 2u : 0u);
            }
            k = (int)(q / (uint32_t)a.M);
            w = stats ? a.dup_cnt[q] : 0u;
        }
        a.pruner_fate[q] = (uint8_t)f;
    }
    if (a.tile_cand) {
        // one atomic per distinct tile in the wave (slots are in stream-tile order, so a wave
        // spans one or two tiles; per-lane atomics on one counter serialised: 0.8 ms at 1M slots)
        uint64_t pend = __ballot(cand_tile != 0xffffffffu);
        while (pend) {
            const int leader = __ffsll((unsigned long long)pend) - 1;
            const uint32_t t0 = __shfl(cand_tile, leader, 64);
            const uint64_t same = __ballot(cand_tile == t0);
            if ((int)(threadIdx.x & 63) == leader) atomicAdd(&a.tile_cand[t0], (uint32_t)__popcll(same));
            pend &= ~same;
        }
    }
    if (stats && k >= 0 && (f & 1u)) {
        atomicAdd(&s_l[k], w);
        if (f & 2u) atomicAdd(&s_s[k], w);
    }
    if (stats || fin) __syncthreads();
    if (stats) {
        const size_t sh = (size_t)(blockIdx.x % kStatShards) * a.K;
        for (int q = threadIdx.x; q < a.K; q += kThreads) {
            if (s_l[q]) atomicAdd(&a.lsz[sh + q], s_l[q]);
            if (s_s[q]) atomicAdd(&a.surv[sh + q], s_s[q]);
        }
    }
    if (fin)
        for (int q = threadIdx.x; q < kMaxK; q += kThreads) {
            if (s_n[q]) atomicAdd(&a.segn[q], s_n[q]);
            if (s_a[q]) atomicAdd(&a.segalive[q], s_a[q]);
        }
}

// fate of one tuple from its status word (candidates: after k_fate_tables), branch
// free: one unconditional LDS byte read (index 0 when unused)
__device__ __forceinline__ uint32_t tuple_fate(uint16_t st, const uint8_t *s_pf, int M) {
    const uint32_t code = st & 0xffu;
    const bool dup = code != kCodeDropped && code < kCodeFate0;
    const uint32_t pf = s_pf[dup ? (uint32_t)(st >> 8) * (uint32_t)M + code - 1u : 0u];
    const uint32_t cf = code >= kCodeFate0 && code != kCodeCandidate ? code - kCodeFate0 : 0u;
    return dup ? pf : cf;
}

// Count from the filter's per-tile duplicate histograms (unit weights, stats summed over
// slots, global level selected): a tile's selected tuples = its duplicates of surviving
// pruner groups + its surviving candidates (counted by k_fate_tables).  One wave per tile
// reads KM words instead of the tile's 2048 status words.
__global__ __launch_bounds__(kThreads) void k_out_hist_count(const uint32_t *__restrict__ hist,
                                                             const uint32_t *__restrict__ tile_cand,
                                                             const uint8_t *__restrict__ pruner_fate, int KM,
                                                             uint32_t ntiles, uint32_t *__restrict__ out_cnt) {
    __shared__ uint8_t s_pf[kHistMaxKM];
    for (int q = threadIdx.x; q < KM; q += kThreads) s_pf[q] = pruner_fate[q];
    __syncthreads();
    const uint32_t tile = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    if (tile >= ntiles) return;
    const int lane = threadIdx.x & 63;
    const uint32_t *h = hist + (size_t)tile * KM;
    uint32_t c = 0;
    for (int q = lane; q < KM; q += 64) c += (s_pf[q] & 2u) ? h[q] : 0u;
#pragma unroll
    for (int sh = 32; sh >= 1; sh >>= 1) c += __shfl_xor(c, sh, 64);
    if (lane == 0) out_cnt[tile] = c + tile_cand[tile];
}

// The same per-tile counts AND their exclusive scan in ONE launch (k_out_hist_count + the
// three-kernel scan before: four dependent launches): a workgroup takes 256 consecutive tiles
// (one per thread; the duplicate groups whose pruner is in G listed once in LDS, usually a
// handful), scans them in the block and takes its prefix from a decoupled look-back over the
// earlier workgroups (blockIdx order: every earlier workgroup was dispatched first).  The
// look-back words carry the launch's epoch in their high half, so the words of an earlier
// launch never read as this launch's (no zeroing launch): bits 63..34 epoch, 33..32 state
// (1 aggregate, 2 inclusive prefix), 31..0 count.  A spin past its bound -> kFlagRadixSpin.
__global__ __launch_bounds__(kThreads) void k_out_hist_scan(const uint32_t *__restrict__ hist,
                                                            const uint32_t *__restrict__ tile_cand,
                                                            const uint8_t *__restrict__ pruner_fate, int KM,
                                                            uint32_t ntiles, uint32_t *__restrict__ out_cnt,
                                                            uint32_t *__restrict__ out_off, uint32_t *__restrict__ d_total,
                                                            unsigned long long *__restrict__ lb, uint32_t epoch,
                                                            uint32_t *__restrict__ err) {
    __shared__ uint8_t s_gq[kHistMaxKM];
    __shared__ uint32_t s_ng, s_w[kThreads / 64];
    __shared__ uint32_t s_prefix;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (wave == 0) {
        uint32_t ng = 0;
        for (int q0 = 0; q0 < KM; q0 += 64) {
            const bool g = q0 + lane < KM && (pruner_fate[q0 + lane] & 2u);
            const uint64_t b = __ballot(g);
            if (g) s_gq[ng + lanes_below(b)] = (uint8_t)(q0 + lane);
            ng += (uint32_t)__popcll(b);
        }
        if (lane == 0) s_ng = ng;
    }
    const uint32_t t = blockIdx.x * kThreads + threadIdx.x;
    const uint32_t tc = t < ntiles ? tile_cand[t] : 0u;
    __syncthreads();
    const uint32_t ng = s_ng;
    uint32_t c = tc;
    if (t < ntiles) {
        const uint32_t *h = hist + (size_t)t * KM;
        for (uint32_t i = 0; i < ng; i++) c += h[s_gq[i]];
    }
    uint32_t bt;
    const uint32_t pl = block_scan_excl(c, s_w, bt);
    const unsigned long long tag = (unsigned long long)epoch << 34;
    const unsigned long long kAgg = 1ull << 32, kInc = 2ull << 32, kState = 3ull << 32;
    if (wave == 0) {
        uint32_t excl = 0;
        const uint32_t b = blockIdx.x;
        if (lane == 0)
            __hip_atomic_store(lb + b, tag | (b == 0 ? kInc : kAgg) | bt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (b > 0) {
            int64_t end = (int64_t)b - 1;
            uint32_t spins = 0;
            for (;;) {
                const int64_t idx = end - lane;
                const unsigned long long w = idx >= 0 ? __hip_atomic_load(lb + idx, __ATOMIC_RELAXED,
                                                                          __HIP_MEMORY_SCOPE_AGENT)
                                                      : (tag | kInc);
                const bool cur = (w >> 34) == (unsigned long long)epoch;
                const unsigned long long st = cur ? (w & kState) : 0ull;
                const uint64_t inc = __ballot(st == kInc), none = __ballot(st == 0ull);
                const int first = inc ? __ffsll((unsigned long long)inc) - 1 : 64;
                const uint64_t upto = first >= 63 ? ~0ull : ((2ull << first) - 1ull);
                if (none & upto) {
                    if (++spins > (1u << 22)) {
                        if (lane == 0) atomicOr(err, kFlagRadixSpin);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                uint32_t v = lane <= first ? (uint32_t)w : 0u;
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
                excl += v;
                if (first < 64) break;
                end -= 64;
            }
            if (lane == 0)
                __hip_atomic_store(lb + b, tag | kInc | (unsigned long long)(excl + bt), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) {
            s_prefix = excl;
            if (b == gridDim.x - 1) *d_total = excl + bt;
        }
    }
    __syncthreads();
    if (t < ntiles) {
        out_cnt[t] = c;
        out_off[t] = s_prefix + pl;
    }
}

// Count pass: kOutTPB tiles per workgroup, every tile's status words loaded up front
// (the pass is latency-bound per workgroup otherwise); per-tile selected counts by
// ballot + popcount.  Stats (|L_k|, survivors_k): unit weights by wave ballots per
// origin (see below); given weights (GW) per thread over all its tuples, one wave
// add when the threads agree on the origin; flushed once per workgroup into
// per-shard accumulators.  GO / GW: given origins / weights.
template <bool GO, bool GW, int kOutTPB>
__global__ __launch_bounds__(kThreads) void k_out_count(OutArgs a) {
    __shared__ unsigned long long s_lsz[kMaxK];
    __shared__ unsigned long long s_surv[kMaxK];
    __shared__ uint8_t s_pf[2048];
    __shared__ uint32_t s_tw[kOutTPB][kThreads / 64];
    const bool stats = a.lsz != nullptr;
    const uint32_t ntiles = (a.n + kTile - 1) / kTile;
    const uint32_t t0 = blockIdx.x * kOutTPB;
    const uint32_t nl = a.n - 1;
    // the status words first, then the small tables: all in flight together (one
    // round trip per workgroup, not one for the tables and another for the stream)
    uint16_t st[kOutTPB][kItems];
#pragma unroll
    for (int t = 0; t < kOutTPB; t++) {
        const uint32_t i0 = (t0 + t) * kTile + threadIdx.x * kItems;
        load_status8(a.status, a.n, i0, st[t]);                     // past the last tile: all masked
    }
    if (stats)
        for (int q = threadIdx.x; q < a.K; q += kThreads) { s_lsz[q] = 0; s_surv[q] = 0; }
    for (int q = threadIdx.x; q < a.KM; q += kThreads) s_pf[q] = a.pruner_fate[q];
    __syncthreads();                                   // s_pf ready
    const int shift = a.select_local ? 0 : 1;
    const int lane = threadIdx.x & 63;
    // !GW (unit weights): wave-wide counts by ballot + popcount (SALU, no cross-lane
    // shuffles): the wave's selected tuples of its first origin o0 are counted
    // together, tuples of any other origin by per-lane LDS atomics
    int o0 = -1;                                       // wave-uniform
    unsigned long long cl = 0, cg = 0;                 // wave-uniform counts for o0
    // GW: per-thread (origin, weights) accumulation, reduced below
    int o1 = -1;
    bool mixed = false;
    unsigned long long wl = 0, wg = 0;
#pragma unroll
    for (int t = 0; t < kOutTPB; t++) {
        const uint32_t i0 = (t0 + t) * kTile + threadIdx.x * kItems;
        uint32_t fate[kItems];
        uint32_t nsel = 0;                             // wave-uniform
#pragma unroll
        for (int k = 0; k < kItems; k++) {
            fate[k] = tuple_fate(st[t][k], s_pf, a.M);             // past n: status 0, fate 0
            nsel += (uint32_t)__popcll(__ballot((fate[k] >> shift) & 1u));
        }
        if (lane == 0) s_tw[t][threadIdx.x >> 6] = nsel;
        if (a.row_flags) {
#pragma unroll
            for (int k = 0; k < kItems; k++)
                if (i0 + k < a.n) a.row_flags[i0 + k] = (uint8_t)fate[k];
        }
        if (stats) {
#pragma unroll
            for (int k = 0; k < kItems; k++) {
                const bool sel = fate[k] & 1u;
                const int o = GO ? a.given_origin[min(i0 + k, nl)] : (int)(st[t][k] >> 8);
                if constexpr (!GW) {
                    const uint64_t bl = __ballot(sel);
                    if (bl) {                                          // wave-uniform
                        if (o0 < 0) o0 = __builtin_amdgcn_readlane(o, __ffsll((unsigned long long)bl) - 1);
                        const uint64_t bad = __ballot(sel && o != o0);
                        cl += (unsigned long long)__popcll(bl & ~bad);
                        cg += (unsigned long long)__popcll(__ballot(sel && (fate[k] & 2u)) & ~bad);
                        if (bad && sel && o != o0) {
                            atomicAdd(&s_lsz[o], 1ull);
                            if (fate[k] & 2u) atomicAdd(&s_surv[o], 1ull);
                        }
                    }
                } else {
                    const unsigned long long w = (unsigned long long)a.given_w[min(i0 + k, nl)];
                    o1 = sel && o1 < 0 ? o : o1;
                    mixed |= sel && o != o1;
                    wl += sel ? w : 0ull;
                    wg += sel && (fate[k] & 2u) ? w : 0ull;
                }
            }
        }
    }
    if (stats && !GW) {
        if (lane == 0 && o0 >= 0) {
            atomicAdd(&s_lsz[o0], cl);
            if (cg) atomicAdd(&s_surv[o0], cg);
        }
    }
    if (stats && GW) {
        if (mixed) {                                   // this thread saw two origins: per tuple
#pragma unroll 1
            for (int t = 0; t < kOutTPB; t++) {
                const uint32_t i0 = (t0 + t) * kTile + threadIdx.x * kItems;
                for (int k = 0; k < kItems; k++) {
                    const uint32_t f = tuple_fate(st[t][k], s_pf, a.M);
                    if (!(f & 1u)) continue;
                    const int o = GO ? a.given_origin[i0 + k] : (int)(st[t][k] >> 8);
                    const unsigned long long w = (unsigned long long)a.given_w[i0 + k];
                    atomicAdd(&s_lsz[o], w);
                    if (f & 2u) atomicAdd(&s_surv[o], w);
                }
            }
        }
        const bool has = o1 >= 0 && !mixed;
        unsigned long long rl = has ? wl : 0ull, rg = has ? wg : 0ull;
        const uint64_t act = __ballot(has);
        if (act) {                                     // wave-uniform
            const int oa0 = __shfl(o1, __ffsll((unsigned long long)act) - 1, 64);
            if (__ballot(has && o1 != oa0) == 0ull) {
#pragma unroll
                for (int sh = 32; sh >= 1; sh >>= 1) {
                    rl += __shfl_xor(rl, sh, 64);
                    rg += __shfl_xor(rg, sh, 64);
                }
                if (lane == 0) {
                    atomicAdd(&s_lsz[oa0], rl);
                    if (rg) atomicAdd(&s_surv[oa0], rg);
                }
            } else if (has) {
                atomicAdd(&s_lsz[o1], rl);
                if (rg) atomicAdd(&s_surv[o1], rg);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x < kOutTPB && t0 + threadIdx.x < ntiles) {
        uint32_t c = 0;
#pragma unroll
        for (int w = 0; w < kThreads / 64; w++) c += s_tw[threadIdx.x][w];
        a.out_cnt[t0 + threadIdx.x] = c;
    }
    if (stats) {
        // sharded accumulators: one global address per (shard, origin), reduced on device
        const size_t sh = (size_t)(blockIdx.x % kStatShards) * a.K;
        for (int q = threadIdx.x; q < a.K; q += kThreads) {
            if (s_lsz[q]) atomicAdd(&a.lsz[sh + q], s_lsz[q]);
            if (s_surv[q]) atomicAdd(&a.surv[sh + q], s_surv[q]);
        }
    }
}

// Write pass: item k of thread t is tuple tile*2048 + k*256 + t, so every status / id load
// of a wave is lane-contiguous (coalesced 128 / 512-byte requests; the thread-contiguous
// layout of the count pass made the id loads 64-byte strided).  Index order within the tile
// is (k, wave, lane): a selected tuple's output position is the count of the (k, wave)
// groups before it (32 per tile, scanned in LDS) plus its rank in its wave's ballot.
// The write pass's epilogue workgroups (OutArgs::ep_pin): workgroup e < K sums stat key e over the
// shards (k_stat_reduce), workgroup K copies the final read's other words (k_gather_words); every
// word they read was final before this launch, and the write pass changes none of them
__device__ __forceinline__ void out_epilogue(const OutArgs &a, uint32_t e) {
    __shared__ unsigned long long s_l[kThreads / 64], s_s[kThreads / 64];
    const int K = a.K;
    if (e < (uint32_t)K) {
        unsigned long long l = 0, sv = 0;
        for (int sh = threadIdx.x; sh < kStatShards; sh += kThreads) {
            l += a.ep_lsz[(size_t)sh * K + e];
            sv += a.ep_surv[(size_t)sh * K + e];
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            l += __shfl_xor(l, o, 64);
            sv += __shfl_xor(sv, o, 64);
        }
        if ((threadIdx.x & 63) == 0) { s_l[threadIdx.x >> 6] = l; s_s[threadIdx.x >> 6] = sv; }
        __syncthreads();
        if (threadIdx.x == 0) {
            l = 0;
            sv = 0;
            for (int q = 0; q < kThreads / 64; q++) { l += s_l[q]; sv += s_s[q]; }
            a.ep_statk[e] = l;
            a.ep_statk[K + e] = sv;
            unsigned long long *pk = reinterpret_cast<unsigned long long *>(a.ep_pin + a.ep_off[0]);
            pk[e] = l;
            pk[K + e] = sv;
        }
        return;
    }
    for (int q = threadIdx.x; q < 16; q += kThreads) a.ep_pin[q] = a.ep_totals[q];
    for (int q = threadIdx.x; q < a.ep_Kp; q += kThreads) {
        a.ep_pin[a.ep_off[1] + q] = a.ep_segalive[q];
        a.ep_pin[a.ep_off[2] + q] = a.ep_segn[q];
    }
    if (threadIdx.x == 0) a.ep_pin[a.ep_off[3]] = a.ep_flags[0];
    for (int q = threadIdx.x; q < a.KM; q += kThreads) a.ep_pin[a.ep_off[4] + q] = a.ep_dup[q];
}

// SPARSE (OutArgs::sparse_ids: the last run selected < 1/32 of its tuples): the ids are loaded
// after the selection, only by the selected lanes (C2 selects 0.13 %: the dense form read every id)
template <bool SPARSE>
__global__ __launch_bounds__(kThreads) void k_out_write(OutArgs a) {
    // after a one-workgroup tail that missed (or tripped its guard) no fate / offset is valid:
    // the caller's buffers are left untouched (the host re-runs the query or returns the error)
    if (a.skip_flags && (*a.skip_flags & (kFlagTinyMiss | kFlagTinyOob))) return;
    {
        const uint32_t ntile = (a.n + kTile - 1) / kTile;
        if (blockIdx.x >= ntile) {                     // (block-uniform) the final read's words
            out_epilogue(a, blockIdx.x - ntile);
            return;
        }
    }
    __shared__ uint8_t s_pf[2048];
    __shared__ uint32_t s_cnt[kItems * (kThreads / 64)];
    __shared__ uint32_t s_tot;
    __shared__ int64_t s_oid[kTile];
    __shared__ int32_t s_oorg[kTile];
    const uint32_t tile = blockIdx.x;
    const uint32_t i0 = tile * kTile + threadIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t nl = a.n - 1;
    // status, ids and the pruner-fate table in flight together; indices clamped into [0, n)
    // (tuples past n are never selected: masked below)
    uint16_t st[kItems];
    int64_t idv[kItems];
    // the id loads first: the status words are widened / packed as soon as they arrive, and
    // vmcnt waits in issue order, so ids issued after them would wait behind that
    if constexpr (!SPARSE) {
        if (a.ids) {
#pragma unroll
            for (int k = 0; k < kItems; k++) idv[k] = a.ids[min(i0 + k * kThreads, nl)];
        } else {
#pragma unroll
            for (int k = 0; k < kItems; k++) idv[k] = (int64_t)(i0 + k * kThreads);
        }
    }
    // status planes: the (item, wave) words are wave-uniform (scalar loads); a status word is
    // loaded only where the E bit says the filter stored one, the B bit stands for the
    // designated duplicate group's status
    uint64_t pb[kItems], pe[kItems];
    if (a.planes) {
        const ulonglong2 *pw = reinterpret_cast<const ulonglong2 *>(a.planes) + (size_t)tile * 32 +
                               __builtin_amdgcn_readfirstlane(wave);
#pragma unroll
        for (int k = 0; k < kItems; k++) {
            const ulonglong2 w = pw[k * (kThreads / 64)];
            pb[k] = w.x;
            pe[k] = w.y;
        }
        const uint16_t sg = (uint16_t)(a.dom_kj >= 0 ? ((a.dom_kj / a.M) << 8) | (1 + a.dom_kj % a.M) : 0);
        // a wave's 64 status words are loaded only if the filter stored one of them (pe is
        // wave-uniform: a scalar branch, and the load itself unconditional per lane — a per-lane
        // conditional load made the compiler wait on each one)
        uint16_t raw[kItems];
#pragma unroll
        for (int k = 0; k < kItems; k++) raw[k] = pe[k] ? a.status[min(i0 + k * kThreads, nl)] : (uint16_t)0;
#pragma unroll
        for (int k = 0; k < kItems; k++) {
            const bool e = (pe[k] >> lane) & 1ull;
            st[k] = e ? raw[k] : (((pb[k] >> lane) & 1ull) ? sg : (uint16_t)0);
        }
    } else {
#pragma unroll
        for (int k = 0; k < kItems; k++) st[k] = a.status[min(i0 + k * kThreads, nl)];
    }
    for (int q = threadIdx.x; q < a.KM; q += kThreads) s_pf[q] = a.pruner_fate[q];
    __syncthreads();                                   // s_pf ready
    const int shift = a.select_local ? 0 : 1;
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    uint64_t msk[kItems];
#pragma unroll
    for (int k = 0; k < kItems; k++) {
        const bool in = i0 + k * kThreads < a.n;
        const uint32_t f = in ? tuple_fate(st[k], s_pf, a.M) : 0u;
        msk[k] = __ballot((f >> shift) & 1u);
        if (lane == 0) s_cnt[k * (kThreads / 64) + wave] = (uint32_t)__popcll(msk[k]);
    }
    if constexpr (SPARSE) {
#pragma unroll
        for (int k = 0; k < kItems; k++) {
            const uint32_t i = i0 + k * kThreads;             // (selected: i < n)
            idv[k] = (msk[k] >> lane) & 1ull ? (a.ids ? a.ids[i] : (int64_t)i) : 0;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {                            // exclusive offsets of the 32 (k, wave) groups
        uint32_t run = 0;
        for (int q = 0; q < kItems * (kThreads / 64); q++) {
            const uint32_t c = s_cnt[q];
            s_cnt[q] = run;
            run += c;
        }
        s_tot = run;
    }
    __syncthreads();
    const uint32_t base = a.out_off[tile];
#pragma unroll
    for (int k = 0; k < kItems; k++) {
        if (!((msk[k] >> lane) & 1ull)) continue;
        const uint32_t pl = s_cnt[k * (kThreads / 64) + wave] + (uint32_t)__popcll(msk[k] & lt);
        const uint32_t i = i0 + k * kThreads;
        s_oid[pl] = idv[k];
        s_oorg[pl] = a.given_origin ? a.given_origin[i] : (int32_t)(st[k] >> 8);
        if (a.rows_out && (int64_t)base + pl < a.out_cap)
            for (int d = 0; d < a.D; d++) a.rows_out[(size_t)(base + pl) * a.D + d] = a.vals[(size_t)i * a.D + d];
    }
    __syncthreads();
    const uint32_t total = s_tot;
    for (uint32_t q = threadIdx.x; q < total; q += kThreads) {
        if ((int64_t)base + q >= a.out_cap) break;
        if (a.ids_out) a.ids_out[base + q] = s_oid[q];
        if (a.origin_out) a.origin_out[base + q] = s_oorg[q];
    }
}

// Single-pass output (unit weights, stats already summed over slots): per tile, the
// selected tuples' ranks by a block scan, the tile's exclusive prefix by a decoupled
// look-back over the earlier tiles' published counts (tiles numbered in start order by a
// ticket: a tile only waits for tiles already running; bounded spin -> error flag), then
// the ids / origins staged in LDS and written coalesced.  Replaces count pass + scan +
// host read + write pass; positions >= cap are not written (the caller reports
// SKY_E_CAPACITY from the total).
__global__ __launch_bounds__(kThreads) void k_out_fused(OutArgs a, unsigned long long *__restrict__ lb,
                                                        uint32_t *__restrict__ ticket, uint32_t *__restrict__ d_total,
                                                        uint32_t *__restrict__ err, int64_t cap) {
    __shared__ uint8_t s_pf[2048];
    __shared__ uint32_t s_w[kThreads / 64];
    __shared__ int64_t s_oid[kTile];
    __shared__ int32_t s_oorg[kTile];
    __shared__ uint32_t s_tile;
    __shared__ unsigned long long s_prefix;
    if (threadIdx.x == 0) s_tile = atomicAdd(ticket, 1u);
    for (int q = threadIdx.x; q < a.KM; q += kThreads) s_pf[q] = a.pruner_fate[q];
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint32_t ntiles = (a.n + kTile - 1) / kTile;
    const uint32_t i0 = tile * kTile + threadIdx.x * kItems;
    uint16_t st[kItems];
    load_status8(a.status, a.n, i0, st);
    int64_t idv[kItems];
    if (a.ids) {
#pragma unroll
        for (int k = 0; k < kItems; k++) idv[k] = a.ids[min(i0 + k, a.n - 1)];
    } else {
#pragma unroll
        for (int k = 0; k < kItems; k++) idv[k] = (int64_t)(i0 + k);
    }
    const int shift = a.select_local ? 0 : 1;
    uint8_t fate[kItems];
    uint32_t nsel = 0;
#pragma unroll
    for (int k = 0; k < kItems; k++) {
        fate[k] = (uint8_t)tuple_fate(st[k], s_pf, a.M);
        nsel += (fate[k] >> shift) & 1u;
    }
    uint32_t bt;
    uint32_t pl = block_scan_excl(nsel, s_w, bt);
    if (threadIdx.x < 64) {
        // wave-parallel look-back: 64 predecessors per step, nearest inclusive prefix by ballot
        const int lane = threadIdx.x;
        unsigned long long excl = 0;
        if (lane == 0)
            __hip_atomic_store(lb + tile, (tile == 0 ? kLbInc : kLbAgg) | bt, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        if (tile > 0) {
            int64_t end = (int64_t)tile - 1;
            uint32_t spins = 0;
            for (;;) {
                const int64_t idx = end - lane;
                const unsigned long long sv = idx >= 0 ? __hip_atomic_load(lb + idx, __ATOMIC_RELAXED,
                                                                           __HIP_MEMORY_SCOPE_AGENT)
                                                       : kLbInc;                 // before tile 0: prefix 0
                const unsigned long long f = sv & ~kLbCount;
                const uint64_t inc = __ballot(f == kLbInc), zero = __ballot(f == 0ull);
                const int first = inc ? __ffsll((unsigned long long)inc) - 1 : 64;
                const uint64_t upto = first >= 63 ? ~0ull : ((2ull << first) - 1ull);
                if (zero & upto) {                                   // a predecessor not yet published
                    if (++spins > (1u << 22)) {
                        if (lane == 0) atomicOr(err, kFlagRadixSpin);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                unsigned long long c = lane <= first ? (sv & kLbCount) : 0ull;
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
                excl += c;
                if (first < 64) break;
                end -= 64;
            }
            if (lane == 0)
                __hip_atomic_store(lb + tile, kLbInc | (excl + bt), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) {
            s_prefix = excl;
            if (tile == ntiles - 1) *d_total = (uint32_t)(excl + bt);
        }
    }
#pragma unroll
    for (int k = 0; k < kItems; k++) {
        if (!((fate[k] >> shift) & 1)) continue;
        s_oid[pl] = idv[k];
        s_oorg[pl] = a.given_origin ? a.given_origin[i0 + k] : (int32_t)(st[k] >> 8);
        pl++;
    }
    __syncthreads();
    const int64_t base = (int64_t)s_prefix;
    for (uint32_t q = threadIdx.x; q < bt; q += kThreads) {
        const int64_t dst = base + q;
        if (dst >= cap) break;
        if (a.ids_out) a.ids_out[dst] = s_oid[q];
        if (a.origin_out) a.origin_out[dst] = s_oorg[q];
    }
}

// ---- host launchers -----------------------------------------------------------
static inline unsigned nblk(size_t n, int per) { return (unsigned)((n + per - 1) / per); }

void launch_keys(int D, const double *vals, uint32_t n, const KeyParams &kp, int32_t *keys, hipStream_t st) {
    unsigned g = nblk(n, kThreads);
    if (g > 4096) g = 4096;
    if (g == 0) return;
    SKY_DISPATCH_D(D, (k_keys<DD><<<g, kThreads, 0, st>>>(vals, n, kp, keys)));
}

void launch_select_pruners(int D, const double *vals, uint32_t n, uint32_t S, const KeyParams &kp,
                           const int32_t *given_keys, int single, int Kp, int M, unsigned long long *gmin,
                           double *pruners, int32_t *npr, hipStream_t st, bool pick, uint32_t tag,
                           const FillRanges *pre) {
    if (S == 0) return;                               // (S <= 65536: 16-bit sample ids)
    static const unsigned sgrid = [] {        // SKY_SAMPLE_WG: workgroups of the sample pass (A/B knob)
        const char *e = SKY_MEASURE_ENV("SKY_SAMPLE_WG");
        return e ? (unsigned)std::max(1, atoi(e)) : 256u;   // 32: +20 us, 64: +2 us (latency-bound per row)
    }();
    const unsigned g = std::min<unsigned>(nblk(S, kThreads), sgrid);
    const FillRanges none{};
    const FillRanges &f = pre ? *pre : none;
    SKY_DISPATCH_D(D, (k_sample_min<DD><<<g, kThreads, 0, st>>>(vals, n, S, kp, given_keys, single, Kp, M, gmin, tag, f)));
    if (pick) SKY_DISPATCH_D(D, (k_pick_pruners<DD><<<Kp, 64, 0, st>>>(vals, n, S, gmin, M, pruners, npr, tag)));
}

void launch_filter(int D, const FilterArgs &a, hipStream_t st) {
    const size_t lds = (D == 8 ? pruner_lds_bytes<8>(a.Kp, a.M) : (size_t)a.Kp * a.M * D * sizeof(double) + (size_t)a.Kp * a.M * 4) +
                       (size_t)(kFilterFT - 1) * a.Kp * a.M * 4;   // one duplicate-count array per output tile of a span
    static const int tpb_env = [] {            // tiles per workgroup (SKY_FILTER_TPB, A/B knob)
        const char *e = SKY_MEASURE_ENV("SKY_FILTER_TPB");
        return e ? std::max(1, std::min(atoi(e), 64)) : 0;
    }();
    // 8D (C4): 4 tiles -4 % filter time vs 1 (2: -3 %, 8: -3 %); up to 4D (C3's 50M): 8 tiles -2.5 % vs 4
    const unsigned tpb = tpb_env ? (unsigned)tpb_env : (D <= 4 ? 8u : 4u);
    const unsigned spans = nblk(a.n, kTile * kFilterFT);
    static const unsigned minwg = [] {         // SKY_FILTER_MINWG: the grid's floor (A/B knob; 512 / 256
        const char *e = SKY_MEASURE_ENV("SKY_FILTER_MINWG");   // measured no faster at C2-C4 sizes)
        return e ? (unsigned)std::max(1, atoi(e)) : 1024u;
    }();
    // several tiles per workgroup only while the grid still holds >= 1024 workgroups (4 per CU): a
    // 1M-tuple query (C1, a C5 trigger) has 489 tiles, which at 4 per workgroup left half the CUs idle
    const unsigned tpe = std::max(1u, std::min(tpb, spans / minwg));
    const unsigned g = (spans + tpe - 1) / tpe;
    if (!g) return;
    if (a.given_keys) { SKY_DISPATCH_D(D, (k_filter<DD, true><<<g, kThreads, lds, st>>>(a))); }
    else { SKY_DISPATCH_D(D, (k_filter<DD, false><<<g, kThreads, lds, st>>>(a))); }
}

void launch_filter_deferred(int D, const FilterArgs &a, hipStream_t st) {
    const size_t lds = D == 8 ? pruner_lds_bytes<8>(a.Kp, a.M) : (size_t)a.Kp * a.M * D * sizeof(double) + (size_t)a.Kp * a.M * 4;
    static const unsigned dgrid = [] {        // SKY_DEFER_WG: workgroups of the deferred-key pass (A/B knob)
        const char *e = SKY_MEASURE_ENV("SKY_DEFER_WG");
        return e ? (unsigned)std::max(1, atoi(e)) : 256u;
    }();
    SKY_DISPATCH_D(D, (k_filter_deferred<DD><<<dgrid, kThreads, lds, st>>>(a)));
}


// ---- the small planned route's tail in one workgroup (sky_internal.h TinyArgs) -------------
// Phase for phase the kernels it replaces, restated over one workgroup: k_append_pruners,
// per prefilter round k_cand_min / k_cand_pick / k_cand_filter / the scan / k_cand_compact,
// the brute pair pass + k_brute_finish (exact f64 dominance tests instead of the packed / f32
// compare types: the same answer for every row type), k_fate_tables (slot stats), and
// k_out_hist_count + the tile scan + k_stat_reduce.  Data that the next phase reads stays in LDS
// (minima, second-level pruners, the final slots, fates, tile counts, stats); the slot arrays
// the output pass and the host read are written as those kernels write them.
__device__ __forceinline__ uint32_t tiny_scan_excl(uint32_t v, uint32_t *s_w, uint32_t &total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    uint32_t wb = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kTinyThreads / 64; i++) {
        const uint32_t c = s_w[i];
        wb += i < w ? c : 0u;
        tot += c;
    }
    __syncthreads();
    total = tot;
    return wb + inc - v;
}


#ifdef SKY_MEASURE
#define TINY_OK(i, c, bit)                                                                          \
    ((uint64_t)(i) < (uint64_t)(c) ? true                                                         \
                                   : ((lflags |= kFlagTinyOob), (a.chk ? (atomicOr(a.chk, 1u << (bit)), false) : false)))
#define TINY_CLK(i) \
    if (a.clk && threadIdx.x == 0) a.clk[i] = __builtin_amdgcn_s_memrealtime()
#else
// product build: the same capacity check on every global index the tail computes; an index out
// of range skips its access and raises kFlagTinyOob (the run fails with SKY_E_HIP, no fault)
#define TINY_OK(i, c, bit) ((uint64_t)(i) < (uint64_t)(c) ? true : ((lflags |= kFlagTinyOob), false))
#define TINY_CLK(i)
#endif

template <int D>
__global__ __launch_bounds__(kTinyThreads) void k_tiny_tail(TinyArgs a) {
    constexpr int DP = padded_dims<double>(D);
    extern __shared__ __attribute__((aligned(16))) unsigned char s_arena[];
    __shared__ uint32_t s_w[kTinyThreads / 64];
    __shared__ int32_t s_np[kMaxK];
    __shared__ uint32_t s_fl, t_tot[16], f_start;
    // the pruner slot table, the entry -> pruner map and the duplicate counts stay in LDS for the
    // whole tail (no dependent global round trips for them: one workgroup is latency-bound)
    __shared__ int32_t s_ps[kHistMaxKM], s_ps2[kHistMaxKM];
    __shared__ uint16_t s_ent[kHistMaxKM];
    __shared__ uint32_t s_dupc[kHistMaxKM];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) s_fl = 0u;
    constexpr int NT = kTinyThreads, NW = kTinyThreads / 64;
    const AppendArgs &ap = a.ap;
    const int Kp = ap.Kp, M = ap.M, KM = Kp * M;
    constexpr int TU = 16 / DP > 0 ? 16 / DP : 1;                 // slot rows per thread and batch
    uint32_t lflags = 0;
    TINY_CLK(0);
    // round 0's criterion minima (k_cand_min over the whole GPU), fetched with the first round trip
    constexpr int MS0 = kTinyM2 + 1;
    const bool cm0_pre = a.cmin0 && Kp * MS0 <= NT;
    const unsigned long long cm0 = cm0_pre && tid < Kp * MS0 && tid % MS0 < kTinyM2
                                       ? a.cmin0[(tid / MS0) * kTinyM2 + tid % MS0] : ~0ull;

    // ---- 1. one slot per duplicated pruner (k_append_pruners)
    const uint32_t m = *ap.m_total;
    // thread 0 mirrors the totals words and the flags word for the final read: the earlier kernels'
    // values read here, in the first round trip, this kernel's own kept as it writes them
    if (tid < 16) t_tot[tid] = a.totals[tid];
    if (tid == 16) f_start = *ap.flags;
    uint32_t run = 0;
    uint64_t o = 0, an = ~0ull;
    for (int q0 = 0; q0 < KM; q0 += NT) {
        const int q = q0 + tid;
        const uint32_t dc = q < KM ? ap.dup_cnt[q] : 0u;
        double prow[D];                          // the pruner's row, loaded with its count
        load_row<D>(ap.pruners + (size_t)min(q, KM - 1) * D, prow);
        const bool has = dc > 0;
        if (q < KM) s_dupc[q] = dc;
        uint32_t tot;
        const uint32_t e = run + tiny_scan_excl(has ? 1u : 0u, s_w, tot);
        if (has) {
            const uint32_t slot = m + e;
            if (TINY_OK(e, a.cap[7], 0)) ap.entries[e] = q;
            s_ent[e] = (uint16_t)q;
            s_ps[q] = (int32_t)slot;
            if (slot < ap.slot_cap && TINY_OK(slot, a.cap[0], 0)) {
                ap.slot_src[slot] = 0x80000000u | e;
                const uint64_t key = emit_pruner<double, D>(prow, q / M, (double *)ap.rows, slot, ap.sortkey, lflags);
                o |= key;
                an &= key;
            }
        } else if (q < KM) {
            s_ps[q] = -1;
        }
        run += tot;
    }
#pragma unroll
    for (int sh = 32; sh >= 1; sh >>= 1) {
        o |= __shfl_xor(o, sh, 64);
        an &= __shfl_xor(an, sh, 64);
    }
    if (lane == 0 && run) {
        atomicOr(&ap.orand[0], (unsigned long long)o);
        atomicAnd(&ap.orand[1], (unsigned long long)an);
    }
    uint32_t cnt = min(m + run, ap.slot_cap);            // slots written (the launches' device count)
    if (tid == 0) {
        *ap.nps_total = run;
        a.totals[10] = cnt;
        t_tot[5] = run;
        t_tot[10] = cnt;
    }
    __syncthreads();
    TINY_CLK(1);

    // ---- 2. the prefilter rounds
    const double *rows = reinterpret_cast<const double *>(ap.rows);
    const uint64_t *keys = ap.sortkey;
    const uint32_t *src = ap.slot_src;
    constexpr int M2 = kTinyM2;                                    // (tiny_fits: a.M2 == kTinyM2)
    [[maybe_unused]] uint32_t rcap = a.cap[0];                                     // (SKY_TINY_CHK) the current slot arrays
    // a plan without prefilter rounds gets one here when its slots are more than a few: in LDS it
    // costs a few microseconds and keeps the brute pass below (exact either way) small
    const int rounds = a.rounds ? a.rounds : (cnt > kTinyForce ? 1 : 0);
    for (int r = 0; r < rounds; r++) {
        const uint32_t wcap = r == 0 ? a.cap[2] : (r == 1 ? a.cap[3] : a.cap[4]);
        const uint32_t mt = min(a.bound[r], cnt);
        // per-partition strides padded by one element: lanes of different partitions read
        // different banks (unpadded, every partition's row started on the same bank)
        const int MS = M2 + 1, PS = M2 * D + 1;
        // one minima copy per wave when they fit (LDS atomics then contend within a wave only),
        // merged into copy 0 after the pass
        const int ncopy = (size_t)NW * Kp * MS * 8 + (size_t)Kp * PS * 8 + M2 * D * 4 + 64 <= kTinyArena ? NW : 1;
        unsigned long long *s_min = reinterpret_cast<unsigned long long *>(s_arena);        // [ncopy][Kp][MS]
        float *s_wt = reinterpret_cast<float *>(s_min + ncopy * Kp * MS);                   // [M2][D]
        double *s_pr = reinterpret_cast<double *>(s_wt + ((M2 * D + 3) & ~3));             // [Kp][PS]
        unsigned long long *s_minw = s_min + (ncopy > 1 ? wave * Kp * MS : 0);
        if (r == 0 && cm0_pre) {                 // the minima prefetched above: no pass, no merge
            for (int q = tid; q < Kp * MS; q += NT) s_min[q] = cm0;
            __syncthreads();
        } else {
        for (int q = tid; q < ncopy * Kp * MS; q += NT) s_min[q] = ~0ull;
        for (int q = tid; q < M2 * D; q += NT) s_wt[q] = cand_weight(q / D, q % D, D);
        __syncthreads();
        // k_cand_min: per (partition, criterion) the minimising slot; TU rows per thread and batch,
        // their loads issued before the first is used.  Round 0 of a planned route with rounds takes
        // the minima k_cand_min computed over the candidate slots on the whole GPU (a.cmin0): on one
        // CU this pass cost 15-27 us at C1's 10k slots (loads ~7, criteria ~7, atomics ~6, measured)
        const uint32_t ns = (r == 0 && a.cmin0) ? 0u : mt;
        auto slot_of = [&](uint32_t i) -> uint32_t { return i; };
        auto cand_min_rows = [&](uint32_t j0, uint32_t stride) {
            double v[TU][D];
            int kk[TU];
#pragma unroll
            for (int u = 0; u < TU; u++) {               // (row addresses independent of the keys)
                const uint32_t jc = slot_of(min(j0 + u * stride, ns - 1u));
                const bool okc = TINY_OK(jc, rcap, 1);
                const uint32_t jr = okc ? jc : 0u;
                kk[u] = okc ? (int)(reinterpret_cast<const uint32_t *>(keys)[2 * (size_t)jr + 1] >> 24) : -1;
                load_trow<double, D>(rows + (size_t)jr * DP, v[u]);
            }
#pragma unroll
            for (int u = 0; u < TU; u++) {
                if (j0 + u * stride >= ns || !TINY_OK(kk[u], Kp, 12) || kk[u] < 0) continue;
                const uint32_t j = slot_of(j0 + u * stride);
#ifdef SKY_MEASURE
                if (a.dbg & 2) {                                   // loads only
                    if (v[u][0] == -12345.0) atomicMin(&s_min[0], 0ull);
                    continue;
                }
#endif
                float f[D];
#pragma unroll
                for (int d = 0; d < D; d++) f[d] = (float)v[u][d];
                // all M2 criteria first, then all M2 current minima read together (one LDS
                // round trip per row, not two per criterion), then the winning atomics
                unsigned long long ev[M2], cur[M2];
                unsigned long long *mrow = s_minw + kk[u] * MS;
#pragma unroll
                for (int c = 0; c < M2; c++) {
                    float cv = 0.0f;
#pragma unroll
                    for (int d = 0; d < D; d++) cv += s_wt[c * D + d] * f[d];
                    ev[c] = cv != cv ? ~0ull : ((unsigned long long)f32_order_key(cv) << 32) | j;
                }
#pragma unroll
                for (int c = 0; c < M2; c++) cur[c] = mrow[c];
#ifdef SKY_MEASURE
                if (a.dbg & 1) {                                   // no atomics
                    if (ev[0] < cur[1] && ev[2] == 7ull) atomicMin(&mrow[0], ev[0]);
                    continue;
                }
#endif
#pragma unroll
                for (int c = 0; c < M2; c++)
                    if (ev[c] < cur[c]) atomicMin(&mrow[c], ev[c]);
            }
        };
        for (uint32_t j0 = tid; j0 < ns; j0 += TU * NT) cand_min_rows(j0, NT);
        __syncthreads();
        if (ncopy > 1 || (r == 0 && a.cmin0)) {
            for (int q = tid; q < Kp * MS; q += NT) {
                unsigned long long mn = s_min[q];
                for (int w = 1; w < ncopy; w++) mn = min(mn, s_min[w * Kp * MS + q]);
                if (r == 0 && a.cmin0 && q % MS < M2) mn = a.cmin0[(q / MS) * M2 + q % MS];
                s_min[q] = mn;
            }
            __syncthreads();
        }
        }
        TINY_CLK(2);
        // k_cand_pick: one wave per partition, winners deduplicated and mutually non-dominated
        for (int k = wave; k < Kp; k += NW) {
            const unsigned long long w = lane < M2 ? s_min[k * MS + lane] : ~0ull;
            const bool has = w != ~0ull && TINY_OK((uint32_t)(w & 0xffffffffu), rcap, 2);
            double c[D];
            if (has) {
                load_trow<double, D>(rows + (size_t)(uint32_t)(w & 0xffffffffu) * DP, c);
            } else {
#pragma unroll
                for (int d = 0; d < D; d++) c[d] = 0.0;
            }
            const uint64_t hm = __ballot(has);
            bool ok = has;
            for (int q = 0; q < M2; q++) {
                bool le = true, lt = false, eq = true;
#pragma unroll
                for (int d = 0; d < D; d++) {
                    const double x = __shfl(c[d], q, 64);
                    le &= x <= c[d];
                    lt |= x < c[d];
                    eq &= x == c[d];
                }
                if (q != lane && ((hm >> q) & 1ull) && ((le && lt) || (eq && q < lane))) ok = false;
            }
            const uint64_t b = __ballot(ok);
            if (ok) {
                const int pos = (int)lanes_below(b);
#pragma unroll
                for (int d = 0; d < D; d++) s_pr[(size_t)k * PS + pos * D + d] = c[d];
            }
            if (lane == 0) s_np[k] = __popcll(b);
        }
        __syncthreads();
        TINY_CLK(3);
        // k_cand_filter + scan + k_cand_compact: the live slots, TU per thread and batch (loads
        // first), one block scan per batch, the survivors written from registers.  The compacted
        // order is the batch order, not the slot order: nothing downstream depends on slot order
        // (the brute pass, the fates and the counts are per slot; pruner_slot follows livepos)
        double *rows2 = a.rows_r[r];
        uint64_t *key2 = a.key_r[r];
        uint32_t *src2 = a.src_r[r];
        uint32_t base = 0;
        for (int q = tid; q < KM; q += NT) s_ps2[q] = -1;          // (a pruner slot past mt: dropped)
        __syncthreads();
        for (uint32_t j0 = 0; j0 < mt; j0 += TU * NT) {            // block-uniform
            double v[TU][D];
            uint64_t kv[TU];
            uint32_t sv[TU];
            bool liv[TU];
#pragma unroll
            for (int u = 0; u < TU; u++) {
                const uint32_t jc = min(j0 + u * NT + tid, mt - 1u);
                const bool okc = TINY_OK(jc, rcap, 3);
                kv[u] = okc ? keys[jc] : 0ull;
                sv[u] = okc ? src[jc] : 0u;
                load_trow<double, D>(rows + (size_t)(okc ? jc : 0u) * DP, v[u]);
            }
            uint32_t c = 0;
#pragma unroll
            for (int u = 0; u < TU; u++) {
                const uint32_t j = j0 + u * NT + tid;
                liv[u] = false;
                if (j < mt) {
                    const int k = (int)(kv[u] >> 56);
                    const double *pr = s_pr + (size_t)k * PS;
                    const int np = s_np[k];
                    bool dom = false;
                    // four pruners' rows read together per step (LDS latency, not bandwidth, bound)
                    for (int q0 = 0; q0 < np; q0 += 4) {
                        double x[4][D];
#pragma unroll
                        for (int i = 0; i < 4; i++)
#pragma unroll
                            for (int d = 0; d < D; d++) x[i][d] = pr[min(q0 + i, M2 - 1) * D + d];
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            bool le = true, lt = false;
#pragma unroll
                            for (int d = 0; d < D; d++) {
                                le &= x[i][d] <= v[u][d];
                                lt |= x[i][d] < v[u][d];
                            }
                            dom |= le & lt & (q0 + i < np);
                        }
                    }
                    liv[u] = !dom;
                    c += liv[u] ? 1u : 0u;
                }
            }
            uint32_t tot;
            uint32_t pos = base + tiny_scan_excl(c, s_w, tot);
#pragma unroll
            for (int u = 0; u < TU; u++) {
                const uint32_t j = j0 + u * NT + tid;
                if (j < mt) {
                    if (liv[u] && TINY_OK(pos, wcap, 5)) {
                        store_row<double, D>(rows2 + (size_t)pos * DP, v[u]);
                        key2[pos] = kv[u];
                        src2[pos] = sv[u];
                    }
                    if (sv[u] & 0x80000000u)                        // a pruner slot: its new index
                        s_ps2[s_ent[sv[u] & 0x7fffffffu]] = liv[u] ? (int32_t)pos : -1;
                    pos += liv[u] ? 1u : 0u;
                }
            }
            base += tot;
        }
        __syncthreads();
        TINY_CLK(4);
        __syncthreads();
        for (int q = tid; q < KM; q += NT) s_ps[q] = s_ps2[q];
        if (tid == 0) {
            a.totals[11 + r] = base;
            if (r == 0) t_tot[11] = base;
            else if (r == 1) t_tot[12] = base;
            else t_tot[13] = base;
        }
        cnt = base;
        rows = rows2;
        keys = key2;
        src = src2;
        rcap = wcap;
        __syncthreads();
        TINY_CLK(5);
    }

    // ---- 3. the brute pair pass over the final slots (exact f64 tests) + k_brute_finish
    const uint32_t fin = min(a.bound[rounds], cnt);
    if (tid == 0) {
        a.totals[14] = fin;
        t_tot[14] = fin;
    }
    constexpr uint32_t BR = tiny_brute_rows(D);
    if (fin > BR) {                                                // block-uniform
        if (lflags) atomicOr(&s_fl, lflags);
        __syncthreads();
        if (tid == 0) {
            const uint32_t f = s_fl | kFlagTinyMiss;
            atomicOr(ap.flags, f);
            if (a.pin) {
#pragma unroll
                for (int i = 0; i < 16; i++) a.pin[i] = t_tot[i];
                a.pin[a.pin_off[3]] = f_start | f;
            }
        }
        return;
    }
    double *s_row = reinterpret_cast<double *>(s_arena);                          // [BR][D]
    uint32_t *s_part = reinterpret_cast<uint32_t *>(s_row + (size_t)BR * D);       // [BR]
    uint32_t *s_dom = s_part + BR;                                                 // [BR]
    uint32_t *s_src = s_dom + BR;                                                  // [BR]
    unsigned long long *s_l = reinterpret_cast<unsigned long long *>(s_src + BR + (BR & 1u));   // [kMaxK]
    unsigned long long *s_s = s_l + kMaxK;                                         // [kMaxK]
    uint32_t *s_tc = reinterpret_cast<uint32_t *>(s_s + kMaxK);                   // [kTinyTiles]
    uint32_t *s_sn = s_tc + kTinyTiles, *s_sa = s_sn + kMaxK;                       // [kMaxK] x 2
    uint8_t *s_pf = reinterpret_cast<uint8_t *>(s_sa + kMaxK);                     // [kHistMaxKM]
    uint8_t *s_gq = s_pf + kHistMaxKM;                         // [kHistMaxKM] pruner groups in G
    uint32_t *s_ng = reinterpret_cast<uint32_t *>(s_gq + kHistMaxKM);              // [1]
    {                                                              // <= BR * D / NT values per thread
        constexpr int LU = (BR * D + NT - 1) / NT;
        double tv[LU];
#pragma unroll
        for (int u = 0; u < LU; u++) {
            const uint32_t q = tid + u * NT;
            tv[u] = q < fin * D && TINY_OK(q / D, rcap, 7) ? rows[(size_t)(q / D) * DP + q % D] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < LU; u++)
            if (tid + u * NT < fin * D) s_row[tid + u * NT] = tv[u];
    }
    for (uint32_t q = tid; q < fin; q += NT) {
        const bool okq = TINY_OK(q, rcap, 7);
        s_part[q] = okq ? (uint32_t)(keys[q] >> 56) : 0u;
        s_src[q] = okq ? src[q] : 0x80000000u;
        if (!TINY_OK(s_part[q], Kp, 13)) s_part[q] = 0;
        s_dom[q] = 0u;
    }
    for (int q = tid; q < kMaxK; q += NT) {
        s_l[q] = 0;
        s_s[q] = 0;
        s_sn[q] = 0;
        s_sa[q] = 0;
    }
    for (uint32_t q = tid; q < a.ntiles; q += NT) s_tc[q] = 0u;
    __syncthreads();
    TINY_CLK(6);
    for (uint32_t pq = tid; pq < fin * fin; pq += NT) {
        const uint32_t y = pq / fin, x = pq - y * fin;
        if (x == y) continue;
        bool le = true, lt = false;
#pragma unroll
        for (int d = 0; d < D; d++) {
            const double xv = s_row[x * D + d], yv = s_row[y * D + d];
            le &= xv <= yv;
            lt |= xv < yv;
        }
        if (le & lt) atomicOr(&s_dom[y], s_part[x] == s_part[y] ? 3u : 2u);
    }
    __syncthreads();
    TINY_CLK(7);
    for (uint32_t j = tid; j < fin; j += NT) {
        const uint32_t f = s_dom[j];
        const bool in_l = !(f & 1u);
        const bool in_g = a.gmerge ? !(f & 2u) : in_l;
        if (TINY_OK(j, a.cap[5], 8)) {
            a.alive_l[j] = in_l ? 1 : 0;
            a.alive_g[j] = in_g ? 1 : 0;
            a.slot_rep[j] = j;
        }
        s_dom[j] = (in_l ? 1u : 0u) | (in_g ? 2u : 0u);           // from here on: the slot's fate
        atomicAdd(&s_sn[s_part[j]], 1u);
        if (in_l) atomicAdd(&s_sa[s_part[j]], 1u);
    }
    __syncthreads();
    for (int q = tid; q < Kp; q += NT) {
        if (s_sn[q]) atomicAdd(&a.segn[q], s_sn[q]);
        if (s_sa[q]) atomicAdd(&a.segalive[q], s_sa[q]);
    }

    // ---- 4. the fate tables (k_fate_tables, slot stats)
    for (uint32_t j = tid; j < fin; j += NT) {
        const uint32_t sj = s_src[j];
        if (sj & 0x80000000u) continue;                            // appended pruner slots: below
        if (!TINY_OK(sj, a.cap[6], 10)) continue;
        const uint32_t f = s_dom[j];
        const uint16_t s0 = a.status[sj];
        a.status[sj] = (uint16_t)((s0 & 0xff00u) | (kCodeFate0 + f));
        if ((f & 2u) && TINY_OK(sj / kTile, a.ntiles, 11)) atomicAdd(&s_tc[sj / kTile], 1u);
        const int k = s0 >> 8;
        if (!TINY_OK(k, a.K, 14)) continue;
        if (f & 1u) {
            atomicAdd(&s_l[k], 1ull);
            if (f & 2u) atomicAdd(&s_s[k], 1ull);
        }
    }
    for (int q = tid; q < KM; q += NT) {
        const int32_t ps = s_ps[q];
        ap.pruner_slot[q] = ps;                                    // (the final slots' index, as the chain leaves it)
        uint32_t f = 0;
        if (ps >= 0 && (uint32_t)ps < fin) {
            f = s_dom[ps];
            const unsigned long long w = s_dupc[q];
            const int k = q / M;
            if (f & 1u) {
                atomicAdd(&s_l[k], w);
                if (f & 2u) atomicAdd(&s_s[k], w);
            }
        }
        a.pruner_fate[q] = (uint8_t)f;
        s_pf[q] = (uint8_t)f;
    }
    __syncthreads();
    TINY_CLK(8);
    for (int q = tid; q < a.K; q += NT) {                          // k_stat_reduce
        a.statk[q] = s_l[q];
        a.statk[a.K + q] = s_s[q];
    }

    // ---- 5. per-tile output counts (k_out_hist_count) and their exclusive scan: only the
    // duplicate groups whose pruner is in G count, listed first (usually a handful)
    if (wave == 0) {
        uint32_t ng = 0;
        for (int q0 = 0; q0 < KM; q0 += 64) {
            const bool g = q0 + lane < KM && (s_pf[q0 + lane] & 2u);
            const uint64_t b = __ballot(g);
            if (g) s_gq[ng + lanes_below(b)] = (uint8_t)(q0 + lane);
            ng += (uint32_t)__popcll(b);
        }
        if (lane == 0) *s_ng = ng;
    }
    __syncthreads();
    const uint32_t ng = *s_ng;
    uint32_t base = 0;
    for (uint32_t t0 = 0; t0 < a.ntiles; t0 += NT) {                // block-uniform
        const uint32_t t = t0 + tid;
        uint32_t c = 0;
        if (t < a.ntiles) {
            const uint32_t *h = a.tile_hist + (size_t)t * KM;
#pragma unroll 8
            for (uint32_t i = 0; i < ng; i++) c += h[s_gq[i]];
            c += s_tc[t];
        }
        uint32_t tot;
        const uint32_t off = base + tiny_scan_excl(c, s_w, tot);
        if (t < a.ntiles) {
            a.out_cnt[t] = c;
            a.out_off[t] = off;
        }
        base += tot;
    }
    if (tid == 0) {
        a.totals[3] = base;
        t_tot[3] = base;
    }
    if (lflags) atomicOr(&s_fl, lflags);
    __syncthreads();
    // ---- 6. the flags, and the final read's words into the host-mapped buffer (the flags word as
    // it stands after this kernel: the earlier kernels' bits, read at the start, and this one's)
    if (tid == 0) {
        if (s_fl) atomicOr(ap.flags, s_fl);
        if (a.pin) {
#pragma unroll
            for (int i = 0; i < 16; i++) a.pin[i] = t_tot[i];
            a.pin[a.pin_off[3]] = f_start | s_fl;
        }
    }
    if (a.pin) {
        for (int q = tid; q < a.K; q += NT) {
            a.pin[a.pin_off[0] + 2 * q] = (uint32_t)s_l[q];
            a.pin[a.pin_off[0] + 2 * q + 1] = (uint32_t)(s_l[q] >> 32);
            a.pin[a.pin_off[0] + 2 * (a.K + q)] = (uint32_t)s_s[q];
            a.pin[a.pin_off[0] + 2 * (a.K + q) + 1] = (uint32_t)(s_s[q] >> 32);
        }
        for (int q = tid; q < Kp; q += NT) {
            a.pin[a.pin_off[1] + q] = s_sa[q];
            a.pin[a.pin_off[2] + q] = s_sn[q];
        }
        for (int q = tid; q < KM; q += NT) a.pin[a.pin_off[4] + q] = s_dupc[q];
    }
    TINY_CLK(9);
}

bool tiny_fits(int D, int Kp, int M2, int KM, int K, uint32_t tiles) {
    const size_t pre = (size_t)Kp * (M2 + 1) * 8 + (size_t)((M2 * D + 3) & ~3) * 4 + (size_t)Kp * (M2 * D + 1) * 8 + 64;
    const size_t brute = (size_t)tiny_brute_rows(D) * (D * 8 + 12) + kTinyFixed;
    return M2 == kTinyM2 && KM <= kHistMaxKM && K <= kMaxK && Kp <= kMaxK && tiles <= kTinyTiles &&
           pre <= kTinyArena && brute <= kTinyArena;
}

void launch_tiny_tail(int D, const TinyArgs &a, hipStream_t st) {
    SKY_DISPATCH_D(D, (k_tiny_tail<DD><<<1, kTinyThreads, kTinyArena, st>>>(a)));
}

void launch_append_pruners(int D, const AppendArgs &a, hipStream_t st) {
    SKY_DISPATCH_D(D, (k_append_pruners<DD><<<1, kThreads, 0, st>>>(a)));
}

void launch_cand_prefilter(int D, const CandArgs &a, hipStream_t st) {
    if (!a.mt) return;
    // <= 256 workgroups (a few rows per thread): each adds up to Kp*M2 global minima
    const unsigned g = std::min<unsigned>(nblk(a.mt, kThreads), 256u);
    SKY_DISPATCH_D(D, (k_cand_min<DD><<<g, kThreads, 0, st>>>(a.rows, a.key, a.mt, a.d_mt, a.Kp, a.M2, a.cmin)));
    SKY_DISPATCH_D(D, (k_cand_pick<DD><<<a.Kp, 64, 0, st>>>(a.rows, a.cmin, a.M2, a.pr2, a.npr2)));
    // the pruner image in LDS up to 32 KB (Kp x M2 x D doubles: 16 KB for C4's 16 x 16 x 8); beyond
    // that (hundreds of partitions at high D) the rows are read from global memory
    const size_t lds = (size_t)a.Kp * a.M2 * D * sizeof(double);
    if (lds <= 32768) {
        SKY_DISPATCH_D(D, (k_cand_filter<DD, true><<<nblk(a.mt, kThreads), kThreads, lds, st>>>(
                              a.rows, a.key, a.mt, a.d_mt, a.Kp, a.M2, a.pr2, a.npr2, a.live)));
    } else {
        SKY_DISPATCH_D(D, (k_cand_filter<DD, false><<<nblk(a.mt, kThreads), kThreads, 0, st>>>(
                              a.rows, a.key, a.mt, a.d_mt, a.Kp, a.M2, a.pr2, a.npr2, a.live)));
    }
}

void launch_cand_min(int D, const CandArgs &a, hipStream_t st) {
    if (!a.mt) return;
    const unsigned g = std::min<unsigned>(nblk(a.mt, kThreads), 256u);
    SKY_DISPATCH_D(D, (k_cand_min<DD><<<g, kThreads, 0, st>>>(a.rows, a.key, a.mt, a.d_mt, a.Kp, a.M2, a.cmin)));
}

bool cand_fused_fits(int D, int Kp, int M2) {
    return M2 <= 64 && (size_t)Kp * (M2 * D + 1) * sizeof(double) <= 32768;
}

void launch_cand_fused(int D, const CandArgs &a, hipStream_t st) {
    if (!a.mt) return;
    const size_t lds = (size_t)a.Kp * (a.M2 * D + 1) * sizeof(double);
    if (a.picked) {
        SKY_DISPATCH_D(D, (k_cand_pick<DD><<<a.Kp, 64, 0, st>>>(a.rows, a.cmin, a.M2, a.pr2, a.npr2)));
        SKY_DISPATCH_D(D, (k_cand_fused<DD, 1, true><<<cand_fused_tiles(a.mt, true), kThreads, lds, st>>>(a)));
    } else {
        SKY_DISPATCH_D(D, (k_cand_fused<DD, 4, false><<<cand_fused_tiles(a.mt, false), kThreads, lds, st>>>(a)));
    }
}

void launch_cand_compact(int D, const CandArgs &a, const uint32_t *pos, double *rows2, uint64_t *key2, uint32_t *src2,
                         int32_t *pruner_slot, int KM, hipStream_t st) {
    const uint32_t n = std::max<uint32_t>(a.mt, (uint32_t)KM);
    if (!n) return;
    SKY_DISPATCH_D(D, (k_cand_compact<DD><<<nblk(n, kThreads), kThreads, 0, st>>>(a.mt, a.d_mt, a.live, pos, a.rows, a.key,
                                                                                 a.src, rows2, key2, src2, pruner_slot,
                                                                                 KM)));
}

void launch_fate_tables(const FateArgs &a, hipStream_t st) {
    const size_t tot = (size_t)a.mt + a.KM;
    if (tot) k_fate_tables<<<nblk(tot, kThreads), kThreads, 0, st>>>(a);
}

void launch_gather_runs(int D, bool f64, const RepArgs &a, hipStream_t st) {
    if (f64) { SKY_DISPATCH_D(D, (k_gather_runs<double, DD><<<nblk(a.mt, kThreads), kThreads, 0, st>>>(a))); }
    else { SKY_DISPATCH_D(D, (k_gather_runs<float, DD><<<nblk(a.mt, kThreads), kThreads, 0, st>>>(a))); }
}
void launch_run_first(const RepArgs &a, hipStream_t st) {
    k_run_first<<<nblk(a.mt, kThreads), kThreads, 0, st>>>(a);
}
void launch_rep_of(int D, bool f64, const RepArgs &a, hipStream_t st) {
    if (f64) { SKY_DISPATCH_D(D, (k_rep_of<double, DD><<<nblk(a.mt, kThreads), kThreads, 0, st>>>(a))); }
    else { SKY_DISPATCH_D(D, (k_rep_of<float, DD><<<nblk(a.mt, kThreads), kThreads, 0, st>>>(a))); }
}
void launch_build_reps(int D, bool f64, const RepArgs &a, hipStream_t st) {
    if (f64) { SKY_DISPATCH_D(D, (k_build_reps<double, DD><<<nblk(a.mt, kThreads), kThreads, 0, st>>>(a))); }
    else { SKY_DISPATCH_D(D, (k_build_reps<float, DD><<<nblk(a.mt, kThreads), kThreads, 0, st>>>(a))); }
}
void launch_seg_bounds(const uint64_t *rep_key, uint32_t mt, const uint32_t *d_mr, uint32_t *seg_begin,
                       uint32_t *seg_end, hipStream_t st) {
    if (mt) k_seg_bounds<<<nblk(mt, kThreads), kThreads, 0, st>>>(rep_key, d_mr, seg_begin, seg_end);
}
void launch_rep_mult(uint32_t mt, const uint32_t *perm, const uint32_t *slot_src, const uint32_t *rep_of_sorted,
                     const int64_t *given_w, const uint32_t *dup_cnt, const int32_t *pr_entries,
                     unsigned long long *mult, hipStream_t st) {
    if (mt) k_rep_mult<<<nblk(mt, kThreads), kThreads, 0, st>>>(mt, perm, slot_src, rep_of_sorted, given_w, dup_cnt,
                                                                pr_entries, mult);
}
// SKY_OUT_TPB in {4, 8, 16}: tiles per count-pass workgroup (A/B knob)
static int out_tpb() {
    static const int v = [] {
        const char *e = SKY_MEASURE_ENV("SKY_OUT_TPB");
        const int t = e ? atoi(e) : 4;
        return t == 8 || t == 16 ? t : 4;
    }();
    return v;
}
template <int TPB>
static void out_count_t(const OutArgs &a, hipStream_t st) {
    const unsigned g = nblk(nblk(a.n, kTile), TPB);
    const bool go = a.given_origin != nullptr, gw = a.given_w != nullptr;
    if (go && gw) k_out_count<true, true, TPB><<<g, kThreads, 0, st>>>(a);
    else if (go) k_out_count<true, false, TPB><<<g, kThreads, 0, st>>>(a);
    else if (gw) k_out_count<false, true, TPB><<<g, kThreads, 0, st>>>(a);
    else k_out_count<false, false, TPB><<<g, kThreads, 0, st>>>(a);
}
void launch_out_count(const OutArgs &a, hipStream_t st) {
    if (!a.n) return;
    const int t = out_tpb();
    if (nblk(a.n, kTile) < 4u * 1024u) out_count_t<1>(a, st);   // < 1024 workgroups at 4 tiles: fill the GPU
    else if (t == 8) out_count_t<8>(a, st);
    else if (t == 16) out_count_t<16>(a, st);
    else out_count_t<4>(a, st);
}
void launch_out_fused(const OutArgs &a, unsigned long long *lb, uint32_t *ticket, uint32_t *d_total, uint32_t *err,
                      int64_t cap, hipStream_t st) {
    const uint32_t tiles = (a.n + kTile - 1) / kTile;
    if (tiles) k_out_fused<<<tiles, kThreads, 0, st>>>(a, lb, ticket, d_total, err, cap);
}

uint32_t out_hist_scan_blocks(uint32_t ntiles) { return (ntiles + kThreads - 1) / kThreads; }

void launch_out_hist_scan(const uint32_t *hist, const uint32_t *tile_cand, const uint8_t *pruner_fate, int KM,
                          uint32_t ntiles, uint32_t *out_cnt, uint32_t *out_off, uint32_t *d_total,
                          unsigned long long *lb, uint32_t epoch, uint32_t *err, hipStream_t st) {
    if (!ntiles) return;
    k_out_hist_scan<<<out_hist_scan_blocks(ntiles), kThreads, 0, st>>>(hist, tile_cand, pruner_fate, KM, ntiles, out_cnt,
                                                                       out_off, d_total, lb, epoch & 0x3fffffffu, err);
}

void launch_out_hist_count(const uint32_t *hist, const uint32_t *tile_cand, const uint8_t *pruner_fate, int KM,
                           uint32_t ntiles, uint32_t *out_cnt, hipStream_t st) {
    if (ntiles) k_out_hist_count<<<nblk(ntiles, kThreads / 64), kThreads, 0, st>>>(hist, tile_cand, pruner_fate, KM,
                                                                                  ntiles, out_cnt);
}

void launch_out_write(const OutArgs &a, hipStream_t st) {
    if (!a.n) return;
    const unsigned g = nblk(a.n, kTile) + (a.ep_pin ? (uint32_t)a.K + 1u : 0u);
    if (a.sparse_ids) k_out_write<true><<<g, kThreads, 0, st>>>(a);
    else k_out_write<false><<<g, kThreads, 0, st>>>(a);
}
// sky_profile_pairs_dev: caller rows -> the slot format of the brute pass (f64 rows padded to
// 16 B, sort key = partition | f32 score | hash, as k_filter appends candidates)
template <int D>
__global__ __launch_bounds__(kThreads) void k_prof_slots(const double *__restrict__ vals,
                                                        const int32_t *__restrict__ keys, uint32_t n,
                                                        double *__restrict__ rows, uint64_t *__restrict__ key,
                                                        uint32_t *__restrict__ flags) {
    constexpr int DP = padded_dims<double>(D);
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    uint32_t lf = 0;
    if (j < n) {
        double v[D];
#pragma unroll
        for (int d = 0; d < D; d++) {
            v[d] = vals[(size_t)j * D + d];
            if ((double)(float)v[d] != v[d]) lf |= kFlagNotF32;
        }
#pragma unroll
        for (int d = 0; d < DP; d++) rows[(size_t)j * DP + d] = d < D ? v[d] : 0.0;
        key[j] = make_sortkey<double, D>(v, (uint32_t)keys[j], lf);
    }
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) lf |= (uint32_t)__shfl_xor((int)lf, s, 64);
    if ((threadIdx.x & 63) == 0 && lf) atomicOr(flags, lf);
}

void launch_prof_slots(int D, const double *vals, const int32_t *keys, uint32_t n, double *rows, uint64_t *key,
                       uint32_t *flags, hipStream_t st) {
    if (!n) return;
    SKY_DISPATCH_D(D, (k_prof_slots<DD><<<(n + kThreads - 1) / kThreads, kThreads, 0, st>>>(vals, keys, n, rows, key,
                                                                                           flags)));
}

}  // namespace sky
