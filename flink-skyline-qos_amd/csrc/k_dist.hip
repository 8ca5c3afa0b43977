// k_dist.hip — device side of the multi-GPU step (one process per GPU, include/skyline_hip.h
// "multi-GPU"): every kernel here takes its counts from device memory, so a whole step —
// local phase, export block, (the caller's RCCL all-gather), own-vector fates against the
// union, output, (the caller's RCCL all-reduce of the stats) — runs without a host read
// until sky_dist_finish.
//
// Block of one rank (int64 words, (cap + 1) rows of RW = D + 2 words):
//   row 0:        count (vectors exported, may exceed cap), verdict bits, shard tuples, dims
//   rows 1..cap:  D words of f64 value bits, partition key, multiplicity
// The reference's exchange is Flink's keyBy shuffle into one reducer per query
// (FlinkSkyline.java:138, :171-174); the merge rule is GlobalSkylineAggregator's
// (:548-566) applied to each rank's own vectors only.
#include <algorithm>

#include "sky_internal.h"

namespace sky {

static inline unsigned nblk_d(size_t n, int per) { return (unsigned)((n + per - 1) / per); }

// ---- the planned route's checks, on the device -----------------------------------------
// The same assumptions pipe_finish verifies on the host after its final read (no NaN, no slot
// overflow, every count within the bound its launches were sized for, the small-set size, the
// compare type), evaluated where the data is: the verdict travels in the block header, so every
// rank learns after the all-gather whether some rank has to re-run its local phase.
__global__ void k_plan_verdict(const uint32_t *__restrict__ tot, const uint32_t *__restrict__ flags, PlanCheck pc,
                               uint32_t *__restrict__ verdict) {
    if (threadIdx.x != 0) return;
    const uint32_t f = *flags;
    uint32_t v = 0;
    if (f & kFlagNaN) v |= kDistNaN;
    if (f & (kFlagRadixSpin | kFlagMbrQueue)) v |= kDistError;
    if (pc.planned) {
        const uint32_t m = tot[0], nps = tot[5];
        bool ok = (uint64_t)m + nps <= pc.cap;
        ok &= tot[10] <= pc.bound[0];
        for (int r = 0; r < pc.rounds; r++) ok &= tot[11 + r] <= pc.bound[r + 1];
        const uint32_t fin = pc.rounds ? tot[10 + pc.rounds] : tot[10];
        ok &= fin <= pc.brute_max;
        const bool f64 = (f & kFlagNotF32) != 0, ints = !f64 && (f & kFlagNotU16) == 0;
        ok &= pc.k_u16 ? ints : (pc.k_f32 ? !f64 : true);
        if (!ok) v |= kDistReplan;
    }
    *verdict = v;
}

// alive u8 -> u32 over a device-sized unit range (units >= *d_n count 0)
__global__ __launch_bounds__(kThreads) void k_dist_flags(const uint8_t *__restrict__ alive, uint32_t n,
                                                        const uint32_t *__restrict__ d_n, uint32_t *__restrict__ out) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= n) return;
    const uint32_t nd = d_n ? min(n, *d_n) : n;
    out[j] = j < nd && alive[j] ? 1u : 0u;
}

// the exported rows of the alive units: slot mode (f64 slot rows, multiplicity from the slot's
// source: a candidate tuple or a pruner's duplicate group) or representative mode (f32 / f64
// rep rows, multiplicity summed by k_rep_mult)
template <typename T, int D>
__global__ __launch_bounds__(kThreads) void k_dist_rows(const T *__restrict__ rows, const uint64_t *__restrict__ key,
                                                       const uint32_t *__restrict__ flag, const uint32_t *__restrict__ pos,
                                                       uint32_t n, const uint32_t *__restrict__ slot_src,
                                                       const uint32_t *__restrict__ dup_cnt,
                                                       const int32_t *__restrict__ pr_entries,
                                                       const unsigned long long *__restrict__ mult,
                                                       int64_t *__restrict__ block, uint32_t cap) {
    constexpr int DP = padded_dims<T>(D);
    constexpr int RW = D + 2;
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= n || !flag[j]) return;
    const uint32_t e = pos[j];
    if (e >= cap) return;                                  // counted; the exchange re-runs larger
    int64_t *o = block + (size_t)(e + 1) * RW;
    const T *r = rows + (size_t)j * DP;
#pragma unroll
    for (int d = 0; d < D; d++) o[d] = __double_as_longlong((double)r[d]);
    o[D] = (int64_t)(key[j] >> 56);
    unsigned long long w;
    if (mult) {
        w = mult[j];
    } else {
        const uint32_t src = slot_src[j];
        w = (src & 0x80000000u) ? (unsigned long long)dup_cnt[pr_entries[src & 0x7fffffffu]] : 1ull;
    }
    o[D + 1] = (int64_t)w;
}

__global__ void k_dist_header(const uint32_t *__restrict__ d_count, const uint32_t *__restrict__ verdict, uint32_t n,
                              int D, int64_t *__restrict__ block) {
    const int t = threadIdx.x;
    if (t < D + 2) {
        int64_t v = 0;
        if (t == 0) v = d_count ? (int64_t)*d_count : 0;
        else if (t == 1) v = verdict ? (int64_t)*verdict : 0;
        else if (t == 2) v = (int64_t)n;
        else if (t == 3) v = D;
        block[t] = v;
    }
}

// ---- the merge -------------------------------------------------------------------------
// sum[0] = largest count of any block, [1] = OR of the verdicts, [2] = this rank's verdict,
// [3] = union rows held by the blocks (sum of min(count, cap)), [4] = this rank's own rows held,
// [6] = where they start in the compacted union, [7] = union vectors exported (sum of counts),
// [8] = this rank's exported vectors; [16 + b] = block b's start in the compacted union
__global__ void k_dist_summary(const int64_t *__restrict__ blocks, int world, int rank, uint32_t cap, int RW,
                               unsigned long long *__restrict__ sum) {
    __shared__ unsigned long long s_max, s_or, s_tot, s_all;
    if (threadIdx.x == 0) { s_max = 0; s_or = 0; s_tot = 0; s_all = 0; }
    __syncthreads();
    const size_t bstride = (size_t)(cap + 1) * RW;
    for (int b = threadIdx.x; b < world; b += blockDim.x) {
        const int64_t c = blocks[(size_t)b * bstride], v = blocks[(size_t)b * bstride + 1];
        const unsigned long long cu = c < 0 ? 0ull : (unsigned long long)c;
        atomicMax(&s_max, cu);
        atomicOr(&s_or, (unsigned long long)v);
        atomicAdd(&s_tot, cu < cap ? cu : (unsigned long long)cap);
        atomicAdd(&s_all, cu);
        if (b == rank) {
            sum[2] = (unsigned long long)v;
            sum[4] = cu < cap ? cu : (unsigned long long)cap;
            sum[8] = cu;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        sum[0] = s_max;
        sum[1] = s_or;
        sum[3] = s_tot;
        sum[7] = s_all;
        // [16 + b]: where block b's rows start in the compacted union (serial: world is small)
        unsigned long long off = 0;
        for (int b = 0; b < world; b++) {
            sum[16 + b] = off;
            const int64_t c = blocks[(size_t)b * bstride];
            const unsigned long long cu = c < 0 ? 0ull : (unsigned long long)c;
            off += cu < cap ? cu : (unsigned long long)cap;
            if (b == rank) sum[6] = sum[16 + b];
        }
    }
}

// the union as contiguous rows for the bounding-box path: f64 rows padded to 16 B, keys in the
// top byte (the pass's partition), multiplicities; sum[5] |= row type flags (kFlagNotF32 /
// kFlagNotU16) over every value
template <int D>
__global__ __launch_bounds__(kThreads) void k_dist_compact(const int64_t *__restrict__ blocks, int world, uint32_t cap,
                                                           unsigned long long *__restrict__ sum,
                                                           double *__restrict__ urows, uint64_t *__restrict__ ukey,
                                                           int64_t *__restrict__ umult) {
    constexpr int RW = D + 2;
    constexpr int DP = padded_dims<double>(D);
    const size_t bstride = (size_t)(cap + 1) * RW;
    const uint64_t total = (uint64_t)world * cap;
    uint32_t lf = 0;
    for (uint64_t q = (uint64_t)blockIdx.x * kThreads + threadIdx.x; q < total; q += (uint64_t)gridDim.x * kThreads) {
        const uint32_t b = (uint32_t)(q / cap), i = (uint32_t)(q - (uint64_t)b * cap);
        const int64_t *blk = blocks + (size_t)b * bstride;
        const int64_t c = blk[0];
        if ((int64_t)i >= c) continue;
        const int64_t *r = blk + (size_t)(i + 1) * RW;
        const size_t o = (size_t)sum[16 + b] + i;
        double v[DP];
#pragma unroll
        for (int d = 0; d < DP; d++) v[d] = d < D ? __longlong_as_double(r[d]) : 0.0;
#pragma unroll
        for (int d = 0; d < D; d++) {
            const double x = v[d];
            if ((double)(float)x != x) lf |= kFlagNotF32;
            if (!((x >= 0.0) && (x <= 65535.0) && (x == floor(x)) &&
                  (__double_as_longlong(x) != (long long)0x8000000000000000ull)))
                lf |= kFlagNotU16;
        }
        double2 *dst = reinterpret_cast<double2 *>(urows + o * DP);
#pragma unroll
        for (int d = 0; d < DP / 2; d++) dst[d] = make_double2(v[2 * d], v[2 * d + 1]);
        ukey[o] = (uint64_t)r[D] << 56;
        umult[o] = r[D + 1];
    }
    // one atomic per wave
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) lf |= (uint32_t)__shfl_xor((int)lf, s, 64);
    if ((threadIdx.x & 63) == 0 && lf) atomicOr(&sum[5], (unsigned long long)lf);
}

// f64 rows -> the bounding-box pass's row format: packed u16 pairs (fmt 0, W words) or f32 (fmt 1)
template <int D, int W>
__global__ __launch_bounds__(kThreads) void k_dist_pack(const double *__restrict__ rows, uint32_t m, int fmt,
                                                        uint32_t *__restrict__ out) {
    constexpr int DP = padded_dims<double>(D);
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= m) return;
    const double *r = rows + (size_t)j * DP;
    if (fmt == 0) {
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
    } else {
        constexpr int FP = padded_dims<float>(D);
        float f[FP];
#pragma unroll
        for (int d = 0; d < FP; d++) f[d] = d < D ? (float)r[d] : 0.0f;
        float4 *o = reinterpret_cast<float4 *>(out + (size_t)j * FP);
#pragma unroll
        for (int q = 0; q < FP / 4; q++) o[q] = make_float4(f[4 * q], f[4 * q + 1], f[4 * q + 2], f[4 * q + 3]);
    }
}

// own vectors (this rank's block) against every union row, straight from the gathered blocks:
// v (key k) is in L_k iff no union row of key k dominates it, in G iff no union row does
// (the union of every rank's local skylines holds a dominator of every dominated tuple).  Full
// dominance test (equal vectors never dominate: the same vector can come from several ranks);
// x dominates y => sum(x) <= sum(y) (rounding is monotone; values clamped to +-1e300 so that
// infinities never meet): larger sums skip the compare.  Per-rank stat shares: multiplicities of the own vectors
// in L_k / G (FlinkSkyline.java:593-608), summed over the ranks by the caller's all-reduce.
constexpr int kDistTile = 256;
template <int D>
// limit: the route was chosen from the previous step's sizes; if this step's |own| x |union|
// (k_dist_summary's sum[4] x sum[3]) exceeds it, no fate is written and *miss = 1 (the caller's
// all-reduce carries it: every rank returns SKY_E_RETRY and this rank re-runs on the sized route).
__global__ __launch_bounds__(kThreads) void k_dist_union_fate(const int64_t *__restrict__ blocks, int world, int rank,
                                                              uint32_t cap, int K, uint8_t *__restrict__ flags,
                                                              unsigned long long *__restrict__ lsz,
                                                              unsigned long long *__restrict__ surv,
                                                              const unsigned long long *__restrict__ sum,
                                                              unsigned long long limit,
                                                              unsigned long long *__restrict__ miss) {
    constexpr int RW = D + 2;
    if (sum[4] * sum[3] > limit) {
        if (blockIdx.x == 0 && threadIdx.x == 0) *miss = 1ull;
        return;
    }
    __shared__ double s_x[kDistTile * D];
    __shared__ double s_s[kDistTile];
    __shared__ int32_t s_k[kDistTile];
    const size_t bstride = (size_t)(cap + 1) * RW;
    const int64_t *own = blocks + (size_t)rank * bstride;
    const uint32_t n_own = (uint32_t)min((unsigned long long)max(own[0], (int64_t)0), (unsigned long long)cap);
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    const bool valid = j < n_own;
    double y[D];
#pragma unroll
    for (int d = 0; d < D; d++) y[d] = valid ? __longlong_as_double(own[(size_t)(j + 1) * RW + d]) : 0.0;
    const int32_t ky = valid ? (int32_t)own[(size_t)(j + 1) * RW + D] : -1;
    auto score = [](const double *v) {
        double s = 0.0;
#pragma unroll
        for (int d = 0; d < D; d++) s += v[d] > 1e300 ? 1e300 : (v[d] < -1e300 ? -1e300 : v[d]);
        return s;
    };
    const double sy = score(y);
    bool dom_l = false, dom_g = false;
    if (!__syncthreads_or(valid)) return;
    for (int b = 0; b < world; b++) {
        const int64_t *blk = blocks + (size_t)b * bstride;
        const uint32_t nb = (uint32_t)min((unsigned long long)max(blk[0], (int64_t)0), (unsigned long long)cap);
        bool go = true;
        for (uint32_t t0 = 0; t0 < nb && go; t0 += kDistTile) {
            const uint32_t cn = nb - t0 < (uint32_t)kDistTile ? nb - t0 : (uint32_t)kDistTile;
            __syncthreads();
            for (uint32_t q = threadIdx.x; q < cn * D; q += kThreads) {
                const uint32_t row = q / D, d = q - row * D;
                s_x[q] = __longlong_as_double(blk[(size_t)(t0 + row + 1) * RW + d]);
            }
            for (uint32_t q = threadIdx.x; q < cn; q += kThreads) s_k[q] = (int32_t)blk[(size_t)(t0 + q + 1) * RW + D];
            __syncthreads();
            for (uint32_t q = threadIdx.x; q < cn; q += kThreads) s_s[q] = score(s_x + (size_t)q * D);
            __syncthreads();
            if (valid && !dom_l) {
                for (uint32_t i = 0; i < cn; i++) {
                    if (s_s[i] <= sy && dominates_full<D, double>(s_x + (size_t)i * D, y)) {
                        dom_g = true;
                        if (s_k[i] == ky) {
                            dom_l = true;
                            break;
                        }
                    }
                }
            }
            go = __syncthreads_or(valid && !dom_l) != 0;
        }
        if (!go) break;
    }
    if (!valid) return;
    flags[j] = (uint8_t)((dom_l ? 0u : 1u) | (dom_g ? 0u : 2u));
    if (ky >= 0 && ky < K) {
        const unsigned long long m = (unsigned long long)own[(size_t)(j + 1) * RW + D + 1];
        if (!dom_l) atomicAdd(&lsz[ky], m);
        if (!dom_g) atomicAdd(&surv[ky], m);
    }
}

// the global level of this rank's units from the own-vector fates (export position -> flags)
__global__ __launch_bounds__(kThreads) void k_dist_alive_g(const uint32_t *__restrict__ flag,
                                                          const uint32_t *__restrict__ pos, uint32_t n,
                                                          const uint8_t *__restrict__ own_flags, uint32_t cap,
                                                          uint8_t *__restrict__ alive_g) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= n) return;
    const uint32_t e = pos[j];
    alive_g[j] = flag[j] && e < cap && (own_flags[e] & 2u) ? 1 : 0;
}

// ---- host launchers --------------------------------------------------------------------
void launch_plan_verdict(const uint32_t *totals, const uint32_t *flags, const PlanCheck &pc, uint32_t *verdict,
                         hipStream_t st) {
    k_plan_verdict<<<1, 64, 0, st>>>(totals, flags, pc, verdict);
}

void launch_dist_flags(const uint8_t *alive, uint32_t n, const uint32_t *d_n, uint32_t *out, hipStream_t st) {
    if (n) k_dist_flags<<<nblk_d(n, kThreads), kThreads, 0, st>>>(alive, n, d_n, out);
}

void launch_dist_rows(int D, bool f64, const void *rows, const uint64_t *key, const uint32_t *flag, const uint32_t *pos,
                      uint32_t n, const uint32_t *slot_src, const uint32_t *dup_cnt, const int32_t *pr_entries,
                      const unsigned long long *mult, int64_t *block, uint32_t cap, hipStream_t st) {
    if (!n) return;
    if (f64) {
        SKY_DISPATCH_D(D, (k_dist_rows<double, DD><<<nblk_d(n, kThreads), kThreads, 0, st>>>(
                              (const double *)rows, key, flag, pos, n, slot_src, dup_cnt, pr_entries, mult, block, cap)));
    } else {
        SKY_DISPATCH_D(D, (k_dist_rows<float, DD><<<nblk_d(n, kThreads), kThreads, 0, st>>>(
                              (const float *)rows, key, flag, pos, n, slot_src, dup_cnt, pr_entries, mult, block, cap)));
    }
}

void launch_dist_header(const uint32_t *d_count, const uint32_t *verdict, uint32_t n, int D, int64_t *block,
                        hipStream_t st) {
    k_dist_header<<<1, 64, 0, st>>>(d_count, verdict, n, D, block);
}

void launch_dist_summary(const int64_t *blocks, int world, int rank, uint32_t cap, int D, unsigned long long *sum,
                         hipStream_t st) {
    k_dist_summary<<<1, kThreads, 0, st>>>(blocks, world, rank, cap, D + 2, sum);
}

void launch_dist_compact(int D, const int64_t *blocks, int world, uint32_t cap, unsigned long long *sum, double *urows,
                         uint64_t *ukey, int64_t *umult, hipStream_t st) {
    const uint64_t total = (uint64_t)world * cap;
    if (!total) return;
    unsigned g = (unsigned)std::min<uint64_t>((total + kThreads - 1) / kThreads, 8192);
    SKY_DISPATCH_D(D, (k_dist_compact<DD><<<g, kThreads, 0, st>>>(blocks, world, cap, sum, urows, ukey, umult)));
}

void launch_dist_pack(int D, const double *rows, uint32_t m, int fmt, uint32_t *out, hipStream_t st) {
    if (!m) return;
    if (D <= 8) {
        SKY_DISPATCH_D(D, (k_dist_pack<DD, 4><<<nblk_d(m, kThreads), kThreads, 0, st>>>(rows, m, fmt, out)));
    } else {
        SKY_DISPATCH_D(D, (k_dist_pack<DD, 8><<<nblk_d(m, kThreads), kThreads, 0, st>>>(rows, m, fmt, out)));
    }
}

void launch_dist_union_fate(int D, const int64_t *blocks, int world, int rank, uint32_t cap, int K, uint8_t *flags,
                            unsigned long long *lsz, unsigned long long *surv, const unsigned long long *sum,
                            unsigned long long limit, unsigned long long *miss, hipStream_t st) {
    if (!cap) return;
    SKY_DISPATCH_D(D, (k_dist_union_fate<DD><<<nblk_d(cap, kThreads), kThreads, 0, st>>>(
                          blocks, world, rank, cap, K, flags, lsz, surv, sum, limit, miss)));
}

// merge-time errors into the all-reduced stat words: a look-back that exceeded its spin bound in
// the union pass (flags, kFlagRadixSpin), or its work queue's overflow (kFlagMbrQueue) -> err = 1
// (every rank then returns SKY_E_HIP)
__global__ void k_dist_merge_err(const uint32_t *__restrict__ flags, unsigned long long *__restrict__ err) {
    if (threadIdx.x == 0) *err = (flags[0] & (kFlagRadixSpin | kFlagMbrQueue)) ? 1ull : 0ull;
}
void launch_dist_merge_err(const uint32_t *flags, unsigned long long *err, hipStream_t st) {
    k_dist_merge_err<<<1, 64, 0, st>>>(flags, err);
}

void launch_dist_alive_g(const uint32_t *flag, const uint32_t *pos, uint32_t n, const uint8_t *own_flags, uint32_t cap,
                         uint8_t *alive_g, hipStream_t st) {
    if (n) k_dist_alive_g<<<nblk_d(n, kThreads), kThreads, 0, st>>>(flag, pos, n, own_flags, cap, alive_g);
}

}  // namespace sky
