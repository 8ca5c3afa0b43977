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
__device__ __forceinline__ uint32_t plan_verdict_value(const uint32_t *__restrict__ tot,
                                                       const uint32_t *__restrict__ flags, const PlanCheck &pc) {
    const uint32_t f = *flags;
    uint32_t v = 0;
    if (f & kFlagNaN) v |= kDistNaN;
    if (f & (kFlagRadixSpin | kFlagMbrQueue | kFlagTinyOob)) v |= kDistError;
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
    return v;
}

__global__ void k_plan_verdict(const uint32_t *__restrict__ tot, const uint32_t *__restrict__ flags, PlanCheck pc,
                               uint32_t *__restrict__ verdict) {
    if (threadIdx.x == 0) *verdict = plan_verdict_value(tot, flags, pc);
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

// The slot-mode export tail in ONE workgroup (the planned small-set route's shards: a few
// thousand units): the run's verdict (k_plan_verdict), the alive flags (k_dist_flags), their
// exclusive scan, the exported rows (k_dist_rows) and the header (k_dist_header) -- five dependent
// launches of 4-6 us each before.  flag / pos stay written for the merge's k_dist_alive_g.
constexpr int kDistExportThreads = 1024;
constexpr uint32_t kDistExportOneMax = 32768;        // units the one-workgroup tail takes
template <int D>
__global__ __launch_bounds__(kDistExportThreads) void k_dist_export_one(
    const uint32_t *__restrict__ tot, const uint32_t *__restrict__ flags, PlanCheck pc, uint32_t *__restrict__ verdict,
    const uint8_t *__restrict__ alive, uint32_t n_units, const uint32_t *__restrict__ d_n, uint32_t *__restrict__ flag,
    uint32_t *__restrict__ pos, uint32_t *__restrict__ d_count, const double *__restrict__ rows,
    const uint64_t *__restrict__ key, const uint32_t *__restrict__ slot_src, const uint32_t *__restrict__ dup_cnt,
    const int32_t *__restrict__ pr_entries, int64_t *__restrict__ block, uint32_t cap, uint32_t n_tuples) {
    constexpr int DP = padded_dims<double>(D);
    constexpr int RW = D + 2;
    constexpr int NW = kDistExportThreads / 64;
    __shared__ uint32_t s_w[NW], s_v;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) s_v = plan_verdict_value(tot, flags, pc);
    const uint32_t nd = d_n ? min(n_units, *d_n) : n_units;
    uint32_t base = 0;
    for (uint32_t j0 = 0; j0 < n_units; j0 += kDistExportThreads) {     // block-uniform
        const uint32_t j = j0 + tid;
        const uint32_t f = j < nd && alive[j] ? 1u : 0u;
        uint32_t inc = f;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(inc, o, 64);
            if (lane >= o) inc += y;
        }
        if (lane == 63) s_w[wave] = inc;
        __syncthreads();
        uint32_t wb = 0, bt = 0;
#pragma unroll
        for (int w = 0; w < NW; w++) {
            const uint32_t c = s_w[w];
            wb += w < wave ? c : 0u;
            bt += c;
        }
        __syncthreads();
        const uint32_t e = base + wb + inc - f;
        if (j < n_units) {
            flag[j] = f;
            pos[j] = e;
        }
        if (f && e < cap) {                   // counted past cap: the exchange re-runs larger
            int64_t *o = block + (size_t)(e + 1) * RW;
            const double *r = rows + (size_t)j * DP;
#pragma unroll
            for (int d = 0; d < D; d++) o[d] = __double_as_longlong(r[d]);
            o[D] = (int64_t)(key[j] >> 56);
            const uint32_t src = slot_src[j];
            o[D + 1] = (src & 0x80000000u) ? (int64_t)dup_cnt[pr_entries[src & 0x7fffffffu]] : 1ll;
        }
        base += bt;
    }
    __syncthreads();
    if (tid == 0) {
        *verdict = s_v;
        *d_count = base;
        pos[n_units] = base;                  // (the scan's total slot, as scan_excl_u32 leaves it)
        block[0] = (int64_t)base;
        block[1] = (int64_t)s_v;
        block[2] = (int64_t)n_tuples;
        if (D + 2 > 3) block[3] = D;
    }
    if (tid >= 4 && tid < D + 2) block[tid] = 0;
}

void launch_dist_export_one(int D, const uint32_t *tot, const uint32_t *flags, const PlanCheck &pc, uint32_t *verdict,
                            const uint8_t *alive, uint32_t n_units, const uint32_t *d_n, uint32_t *flag, uint32_t *pos,
                            uint32_t *d_count, const double *rows, const uint64_t *key, const uint32_t *slot_src,
                            const uint32_t *dup_cnt, const int32_t *pr_entries, int64_t *block, uint32_t cap,
                            uint32_t n_tuples, hipStream_t st) {
    SKY_DISPATCH_D(D, (k_dist_export_one<DD><<<1, kDistExportThreads, 0, st>>>(
                          tot, flags, pc, verdict, alive, n_units, d_n, flag, pos, d_count, rows, key, slot_src, dup_cnt,
                          pr_entries, block, cap, n_tuples)));
}
uint32_t dist_export_one_max() { return kDistExportOneMax; }

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
// infinities never meet): a union row whose sum exceeds every live own vector's is skipped.
//
// A 2D work space walked grid-stride by a fixed grid: item = (64 own vectors, kUnionX union
// rows).  The union rows of an item are staged in LDS once (f64 row, key, sum); the four waves
// of the workgroup hold the same 64 own vectors (lane = own vector) and take a quarter of the
// rows each (every lane reads the same LDS address: a broadcast); the dominated bits are
// OR-reduced in LDS and leave as one global atomic per own vector and item.  Consecutive
// workgroups take consecutive own tiles of the same union rows (the rows stay in L2).
// k_dist_union_finish turns the bits into fates and per-rank stat shares (FlinkSkyline.java:
// 593-608), and clears them for the next step.
//
// limit: the route was chosen from the previous step's sizes; if this step's |own| x |union|
// (k_dist_summary's sum[4] x sum[3]) exceeds it, no fate is written and *miss = 1 (the caller's
// all-reduce carries it: every rank returns SKY_E_RETRY and this rank re-runs on the sized route).
constexpr int kUnionY = 64;
constexpr int kUnionOffLds = 256;       // block offsets staged in LDS up to this world size
template <int D>
constexpr int union_rows() { return D <= 8 ? 512 : 256; }

__device__ __forceinline__ uint32_t union_block_of(uint32_t u, int world, const uint32_t *s_off,
                                                   const unsigned long long *sum) {
    // the last block whose compacted start is <= u (empty blocks share their successor's start)
    int lo = 0, hi = world - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        const uint32_t o = world <= kUnionOffLds ? s_off[mid] : (uint32_t)sum[16 + mid];
        if (o <= u) lo = mid;
        else hi = mid - 1;
    }
    return (uint32_t)lo;
}

template <int D>
__global__ __launch_bounds__(kThreads) void k_dist_union_pairs(const int64_t *__restrict__ blocks, int world, int rank,
                                                               uint32_t cap, unsigned long long *__restrict__ sum,
                                                               unsigned long long limit,
                                                               unsigned long long *__restrict__ miss,
                                                               uint32_t *__restrict__ dom, int fused_summary) {
    constexpr int RW = D + 2;
    constexpr int CH = union_rows<D>();
    __shared__ double s_x[CH * D];
    __shared__ int32_t s_k[CH];
    __shared__ uint32_t s_off[kUnionOffLds];
    __shared__ uint32_t s_bits[kUnionY];
    __shared__ uint32_t s_cnt;
    __shared__ unsigned long long s_sum[2];                  // this launch's |union|, |own|
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const size_t bstride = (size_t)(cap + 1) * RW;
    if (fused_summary) {
        // k_dist_summary's words from the gathered headers (world <= kUnionOffLds), in every
        // workgroup; workgroup 0 also stores them for the later kernels and the host's finish
        if (tid == 0) {
            unsigned long long mx = 0, vor = 0, tot = 0, all = 0, mine = 0, mine_all = 0, mine_v = 0, off_own = 0;
            for (int b = 0; b < world; b++) {
                const int64_t c = blocks[(size_t)b * bstride], v = blocks[(size_t)b * bstride + 1];
                const unsigned long long cu = c < 0 ? 0ull : (unsigned long long)c;
                const unsigned long long held = cu < cap ? cu : (unsigned long long)cap;
                s_off[b] = (uint32_t)tot;
                if (b == rank) { mine = held; mine_all = cu; mine_v = (unsigned long long)v; off_own = tot; }
                mx = cu > mx ? cu : mx;
                vor |= (unsigned long long)v;
                tot += held;
                all += cu;
            }
            s_sum[0] = tot;
            s_sum[1] = mine;
            if (blockIdx.x == 0) {
                sum[0] = mx;
                sum[1] = vor;
                sum[2] = mine_v;
                sum[3] = tot;
                sum[4] = mine;
                sum[6] = off_own;
                sum[7] = all;
                sum[8] = mine_all;
                for (int b = 0; b < world; b++) sum[16 + b] = s_off[b];
            }
        }
    } else {
        for (int b = tid; b < world && b < kUnionOffLds; b += kThreads) s_off[b] = (uint32_t)sum[16 + b];
        if (tid == 0) { s_sum[0] = sum[3]; s_sum[1] = sum[4]; }
    }
    __syncthreads();
    const unsigned long long n_own = s_sum[1], n_union = s_sum[0];
    if (n_own * n_union > limit) {
        if (blockIdx.x == 0 && threadIdx.x == 0 && miss) *miss = 1ull;
        return;
    }
    if (!n_own || !n_union) return;
    const int64_t *own = blocks + (size_t)rank * bstride;
    const uint32_t ytiles = (uint32_t)((n_own + kUnionY - 1) / kUnionY);
    // union rows per item: enough items to spread over the grid (>= 2 per workgroup), at least
    // 16 rows per wave, at most what LDS holds
    const unsigned long long want = (n_union * ytiles + 2ull * gridDim.x - 1) / (2ull * gridDim.x);
    const uint32_t per = (uint32_t)min((unsigned long long)CH, max(64ull, (want + 63) & ~63ull));
    const uint32_t xch = (uint32_t)((n_union + per - 1) / per);
    const uint64_t items = (uint64_t)ytiles * xch;
    auto score = [](const double *v) {
        double s = 0.0;
#pragma unroll
        for (int d = 0; d < D; d++) s += v[d] > 1e300 ? 1e300 : (v[d] < -1e300 ? -1e300 : v[d]);
        return s;
    };
    for (uint64_t it = blockIdx.x; it < items; it += gridDim.x) {
        const uint32_t yt = (uint32_t)(it % ytiles), xc = (uint32_t)(it / ytiles);
        // this lane's own vector (the four waves hold the same 64)
        const uint32_t j = yt * kUnionY + lane;
        const bool valid = j < n_own;
        double y[D];
#pragma unroll
        for (int d = 0; d < D; d++) y[d] = valid ? __longlong_as_double(own[(size_t)(j + 1) * RW + d]) : 0.0;
        const int32_t ky = valid ? (int32_t)own[(size_t)(j + 1) * RW + D] : -1;
        double smax = valid ? score(y) : -INFINITY;
#pragma unroll
        for (int s = 32; s >= 1; s >>= 1) smax = fmax(smax, __shfl_xor(smax, s, 64));
        // stage the item's union rows that can dominate one of the 64 (sum <= their largest)
        __syncthreads();                                  // the previous item's readers are done
        if (tid == 0) s_cnt = 0;
        if (tid < kUnionY) s_bits[tid] = 0;
        __syncthreads();
        const uint32_t u0 = xc * per;
        const uint32_t cn = (uint32_t)min((unsigned long long)per, n_union - u0);
        for (uint32_t r0 = 0; r0 < cn; r0 += kThreads) {
            const uint32_t r = r0 + tid;
            double v[D];
            int32_t kx = 0;
            bool take = false;
            if (r < cn) {
                const uint32_t u = u0 + r;
                const uint32_t b = union_block_of(u, world, s_off, sum);
                const uint32_t ob = world <= kUnionOffLds ? s_off[b] : (uint32_t)sum[16 + b];
                const int64_t *row = blocks + (size_t)b * bstride + (size_t)(u - ob + 1) * RW;
#pragma unroll
                for (int d = 0; d < D; d++) v[d] = __longlong_as_double(row[d]);
                kx = (int32_t)row[D];
                take = score(v) <= smax;
            }
            const unsigned long long m = __ballot(take);
            uint32_t base = 0;
            if (lane == 0 && m) base = atomicAdd(&s_cnt, (uint32_t)__popcll(m));
            base = __shfl(base, 0, 64);
            if (take) {
                const uint32_t q = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
#pragma unroll
                for (int d = 0; d < D; d++) s_x[q * D + d] = v[d];
                s_k[q] = kx;
            }
        }
        __syncthreads();
        // rows wave, wave + 4, ... against the 64 own vectors (broadcast LDS reads)
        const uint32_t nr = s_cnt;
        bool dl = false, dg = false;
        for (uint32_t i0 = wave; i0 < nr; i0 += 4 * 16) {
            if (__ballot(valid && !dl) == 0ull) break;      // every own vector settled
            const uint32_t ie = min(nr, i0 + 4 * 16);
#pragma unroll 2
            for (uint32_t i = i0; i < ie; i += 4) {
                const double *x = s_x + i * D;
                bool gt = false, lt = false;
#pragma unroll
                for (int d = 0; d < D; d++) {
                    gt |= x[d] > y[d];
                    lt |= x[d] < y[d];
                }
                const bool dm = !gt & lt;
                dg |= dm;
                dl |= dm & (s_k[i] == ky);
            }
        }
        const uint32_t bits = (dl ? 1u : 0u) | (dg ? 2u : 0u);
        if (valid && bits) atomicOr(&s_bits[lane], bits);
        __syncthreads();
        if (tid < kUnionY) {
            const uint32_t w = s_bits[tid], jj = yt * kUnionY + tid;
            if (w && jj < n_own) atomicOr(&dom[jj], w);
        }
    }
}

// the own vectors' fates from the pair bits (bit 0: a union row of its key dominates it, bit
// 1: some union row does) -> flags (bit 0: in L_k, bit 1: in G) and this rank's stat shares;
// the bits are cleared for the next step
template <int D>
__global__ __launch_bounds__(kThreads) void k_dist_union_finish(const int64_t *__restrict__ blocks, int rank, uint32_t cap,
                                                                int K, const unsigned long long *__restrict__ sum,
                                                                unsigned long long limit, uint32_t *__restrict__ dom,
                                                                uint8_t *__restrict__ flags,
                                                                unsigned long long *__restrict__ lsz,
                                                                unsigned long long *__restrict__ surv) {
    constexpr int RW = D + 2;
    const unsigned long long n_own = sum[4];
    if (n_own * sum[3] > limit) return;
    __shared__ unsigned long long s_l[kMaxK], s_g[kMaxK];
    const bool lds = K <= kMaxK;
    for (int k = threadIdx.x; lds && k < K; k += kThreads) { s_l[k] = 0; s_g[k] = 0; }
    __syncthreads();
    const int64_t *own = blocks + (size_t)rank * (size_t)(cap + 1) * RW;
    for (uint64_t j = (uint64_t)blockIdx.x * kThreads + threadIdx.x; j < n_own; j += (uint64_t)gridDim.x * kThreads) {
        const uint32_t w = dom[j];
        if (w) dom[j] = 0;
        const bool dl = w & 1u, dg = (w & 2u) != 0;
        flags[j] = (uint8_t)((dl ? 0u : 1u) | (dg ? 0u : 2u));
        const int32_t ky = (int32_t)own[(j + 1) * RW + D];
        if (ky >= 0 && ky < K && !dl) {
            const unsigned long long m = (unsigned long long)own[(j + 1) * RW + D + 1];
            if (lds) {
                atomicAdd(&s_l[ky], m);
                if (!dg) atomicAdd(&s_g[ky], m);
            } else {
                atomicAdd(&lsz[ky], m);
                if (!dg) atomicAdd(&surv[ky], m);
            }
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; lds && k < K; k += kThreads) {
        if (s_l[k]) atomicAdd(&lsz[k], s_l[k]);
        if (s_g[k]) atomicAdd(&surv[k], s_g[k]);
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

bool dist_summary_fused(int world) { return world <= kUnionOffLds; }

void launch_dist_union_fate(int D, const int64_t *blocks, int world, int rank, uint32_t cap, int K, uint8_t *flags,
                            uint32_t *dom, unsigned long long *lsz, unsigned long long *surv,
                            unsigned long long *sum, unsigned long long limit, unsigned long long *miss,
                            hipStream_t st) {
    if (!cap) return;
    // the grid walks the (own tile, union rows) items; its size bounds them from the capacity
    const uint64_t ytiles = (cap + kUnionY - 1) / kUnionY;
    const uint64_t items = ytiles * (((uint64_t)world * cap + 63) / 64);
    const unsigned g = (unsigned)std::min<uint64_t>(items, 1024);
    const unsigned gf = (unsigned)std::min<uint64_t>(((uint64_t)cap + kThreads - 1) / kThreads, 256);
    // the summary words are computed inside the pair pass while the block offsets fit its LDS
    // (the caller then launched no k_dist_summary: dist_summary_fused)
    const int fused = world <= kUnionOffLds ? 1 : 0;
    SKY_DISPATCH_D(D, (k_dist_union_pairs<DD><<<g, kThreads, 0, st>>>(blocks, world, rank, cap, sum, limit, miss, dom,
                                                                      fused)));
    SKY_DISPATCH_D(D, (k_dist_union_finish<DD><<<gf, kThreads, 0, st>>>(blocks, rank, cap, K, sum, limit, dom, flags,
                                                                         lsz, surv)));
}

// merge-time errors into the all-reduced stat words: a look-back that exceeded its spin bound in
// the union pass (flags, kFlagRadixSpin), or its work queue's overflow (kFlagMbrQueue) -> err = 1
// (every rank then returns SKY_E_HIP)
// ... and this rank's share words (statk, err included) into the caller's buffer: one launch
// instead of the error word's kernel and a device-to-device copy
__global__ void k_dist_merge_err(const uint32_t *__restrict__ flags, unsigned long long *__restrict__ statk,
                                 int err_word, int words, int64_t *__restrict__ out) {
    const unsigned long long e = (flags[0] & (kFlagRadixSpin | kFlagMbrQueue | kFlagTinyOob)) ? 1ull : 0ull;
    for (int t = threadIdx.x; t < words; t += blockDim.x) {
        const unsigned long long v = t == err_word ? e : statk[t];
        if (t == err_word) statk[t] = e;
        out[t] = (int64_t)v;
    }
}
void launch_dist_merge_err(const uint32_t *flags, unsigned long long *statk, int err_word, int words, int64_t *out,
                           hipStream_t st) {
    k_dist_merge_err<<<1, 256, 0, st>>>(flags, statk, err_word, words, out);
}

void launch_dist_alive_g(const uint32_t *flag, const uint32_t *pos, uint32_t n, const uint8_t *own_flags, uint32_t cap,
                         uint8_t *alive_g, hipStream_t st) {
    if (n) k_dist_alive_g<<<nblk_d(n, kThreads), kThreads, 0, st>>>(flag, pos, n, own_flags, cap, alive_g);
}

}  // namespace sky
