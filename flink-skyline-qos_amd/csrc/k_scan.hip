// k_scan.hip — device-wide exclusive prefix sums (u32), reduce-then-scan.
// Used for order-preserving stream compaction (candidate slots, output ids)
// and for the radix-sort digit offsets.  Wave64 scans via __shfl_up.
#include "sky_internal.h"

namespace sky {

constexpr int kScanThreads = 256;
constexpr int kScanItems = 16;
constexpr int kScanTile = kScanThreads * kScanItems;   // 4096

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

// exclusive scan of one value per thread across a 256-thread block
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *s_w, uint32_t &total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = wave_incl_scan(v);
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    uint32_t wbase = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kScanThreads / 64; i++) {
        uint32_t c = s_w[i];
        wbase += i < w ? c : 0;
        tot += c;
    }
    __syncthreads();
    total = tot;
    return wbase + inc - v;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_reduce(const uint32_t *__restrict__ in, size_t n,
                                                              uint32_t *__restrict__ partial,
                                                              const uint32_t *__restrict__ d_n) {
    __shared__ uint32_t s_w[4];
    if (d_n) n = min(n, (size_t)*d_n);         // device-sized: n is the bound
    const size_t base = (size_t)blockIdx.x * kScanTile + (size_t)threadIdx.x * kScanItems;
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; i++) s += base + i < n ? in[base + i] : 0u;
    uint32_t total;
    block_excl_scan(s, s_w, total);
    if (threadIdx.x == 0) partial[blockIdx.x] = total;
}

// scans `n` items of one tile per block, adding offs[blockIdx.x] (if given)
__global__ __launch_bounds__(kScanThreads) void k_scan_tile(const uint32_t *__restrict__ in, size_t n,
                                                            uint32_t *__restrict__ out,
                                                            const uint32_t *__restrict__ offs,
                                                            uint32_t *__restrict__ total_out,
                                                            const uint32_t *__restrict__ d_n) {
    __shared__ uint32_t s_w[4];
    if (d_n) n = min(n, (size_t)*d_n);
    const size_t base = (size_t)blockIdx.x * kScanTile + (size_t)threadIdx.x * kScanItems;
    uint32_t v[kScanItems];
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; i++) { v[i] = base + i < n ? in[base + i] : 0u; s += v[i]; }
    uint32_t total;
    uint32_t run = block_excl_scan(s, s_w, total) + (offs ? offs[blockIdx.x] : 0u);
#pragma unroll
    for (int i = 0; i < kScanItems; i++) {
        if (base + i < n) out[base + i] = run;
        run += v[i];
    }
    if (total_out && threadIdx.x == kScanThreads - 1 && gridDim.x == 1) *total_out = run;
}

// single-block scan of a short array (the per-tile partials), in place, writes total
__global__ __launch_bounds__(1024) void k_scan_small(uint32_t *__restrict__ a, size_t n,
                                                     uint32_t *__restrict__ total_out) {
    __shared__ uint32_t s_w[16];
    __shared__ uint32_t s_carry;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (size_t base = 0; base < n; base += 1024) {
        const size_t i = base + threadIdx.x;
        const uint32_t v = i < n ? a[i] : 0u;
        const uint32_t inc = wave_incl_scan(v);
        if (lane == 63) s_w[w] = inc;
        __syncthreads();
        uint32_t wbase = 0, tot = 0;
        for (int k = 0; k < 16; k++) { wbase += k < w ? s_w[k] : 0u; tot += s_w[k]; }
        const uint32_t carry = s_carry;
        if (i < n) a[i] = carry + wbase + inc - v;
        __syncthreads();
        if (threadIdx.x == 0) s_carry = carry + tot;
        __syncthreads();
    }
    if (threadIdx.x == 0 && total_out) *total_out = s_carry;
}

// one workgroup, n <= kScanOneMax: thread t owns the contiguous items [t*per, t*per + per),
// all loaded up front by unconditional (clamped) loads, one block scan, written back.  Beyond
// 16 items per thread the strided loads cost more than the three-kernel path (64 per thread:
// 62 us for 48.8k items, vs ~15 us).
constexpr int kScanOneThreads = 1024;
constexpr int kScanOnePer = 16;
constexpr size_t kScanOneMax = (size_t)kScanOneThreads * kScanOnePer;
__global__ __launch_bounds__(kScanOneThreads) void k_scan_one(const uint32_t *__restrict__ in, uint32_t n,
                                                              uint32_t *__restrict__ out,
                                                              uint32_t *__restrict__ total_out,
                                                              const uint32_t *__restrict__ d_n) {
    __shared__ uint32_t s_w[kScanOneThreads / 64];
    if (d_n) n = min(n, *d_n);
    if (n == 0) {
        if (threadIdx.x == 0 && total_out) *total_out = 0;
        return;
    }
    const uint32_t per = (n + kScanOneThreads - 1) / kScanOneThreads;
    const uint32_t b = threadIdx.x * per;
    uint32_t v[kScanOnePer];
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < kScanOnePer; j++) {
        const uint32_t x = in[min(b + j, n - 1u)];
        v[j] = (uint32_t)j < per && b + j < n ? x : 0u;
        s += v[j];
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t inc = wave_incl_scan(s);
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    uint32_t run = inc - s, tot = 0;
#pragma unroll
    for (int k = 0; k < kScanOneThreads / 64; k++) {
        run += k < w ? s_w[k] : 0u;
        tot += s_w[k];
    }
#pragma unroll
    for (int j = 0; j < kScanOnePer; j++) {
        if ((uint32_t)j < per && b + j < n) out[b + j] = run;
        run += v[j];
    }
    if (threadIdx.x == 0 && total_out) *total_out = tot;
}

// One tile per workgroup as k_scan_tile, its prefix from a decoupled look-back (wave 0 reads 64
// earlier tiles' words per step; blockIdx order: every earlier workgroup was dispatched first on
// its XCD).  Words: bits 63..34 epoch, 33..32 state (1 aggregate, 2 inclusive prefix), 31..0 count.
__global__ __launch_bounds__(kScanThreads) void k_scan_lb(const uint32_t *__restrict__ in, size_t n,
                                                          uint32_t *__restrict__ out, uint32_t *__restrict__ total_out,
                                                          unsigned long long *__restrict__ lb, uint32_t epoch,
                                                          uint32_t *__restrict__ err) {
    __shared__ uint32_t s_w[4];
    __shared__ uint32_t s_prefix;
    const uint32_t b = blockIdx.x;
    const size_t base = (size_t)b * kScanTile + (size_t)threadIdx.x * kScanItems;
    uint32_t v[kScanItems];
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; i++) { v[i] = base + i < n ? in[base + i] : 0u; s += v[i]; }
    uint32_t total;
    uint32_t run = block_excl_scan(s, s_w, total);
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x & 63;
        const unsigned long long tag = (unsigned long long)epoch << 34;
        uint32_t excl = 0;
        if (lane == 0)
            __hip_atomic_store(lb + b, tag | ((b == 0 ? 2ull : 1ull) << 32) | total, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        if (b > 0) {
            int64_t end = (int64_t)b - 1;
            uint32_t spins = 0;
            for (;;) {
                const int64_t idx = end - lane;
                const unsigned long long w = idx >= 0 ? __hip_atomic_load(lb + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                                      : (tag | (2ull << 32));
                const uint32_t state = (w >> 34) == (unsigned long long)epoch ? (uint32_t)(w >> 32) & 3u : 0u;
                const uint64_t inc = __ballot(state == 2u), zero = __ballot(state == 0u);
                const int first = inc ? __ffsll((unsigned long long)inc) - 1 : 64;
                const uint64_t upto = first >= 63 ? ~0ull : ((2ull << first) - 1ull);
                if (zero & upto) {
                    if (++spins > (1u << 22)) {
                        if (lane == 0 && err) *err = 1u;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                uint32_t c = lane <= first ? (uint32_t)w : 0u;
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
                excl += c;
                if (first < 64) break;
                end -= 64;
            }
            if (lane == 0)
                __hip_atomic_store(lb + b, tag | (2ull << 32) | (uint32_t)(excl + total), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) {
            s_prefix = excl;
            if (b == gridDim.x - 1 && total_out) *total_out = excl + total;
        }
    }
    __syncthreads();
    run += s_prefix;
#pragma unroll
    for (int i = 0; i < kScanItems; i++) {
        if (base + i < n) out[base + i] = run;
        run += v[i];
    }
}

size_t scan_lb_words(size_t n) { return (n + kScanTile - 1) / kScanTile + 1; }

void scan_excl_u32_lb(const uint32_t *in, uint32_t *out, size_t n, uint32_t *d_total, unsigned long long *lb,
                      uint32_t epoch, uint32_t *err, hipStream_t st) {
    const size_t tiles = (n + kScanTile - 1) / kScanTile;
    if (n == 0 || tiles == 1 || n <= kScanOneMax) {       // one workgroup: no look-back words needed
        scan_excl_u32(in, out, n, d_total, nullptr, st);
        return;
    }
    k_scan_lb<<<(unsigned)tiles, kScanThreads, 0, st>>>(in, n, out, d_total, lb, epoch, err);
}

// out[i] = sum(in[0..i)), *d_total = sum(in) ; `scratch` needs scan_scratch_words(n) words
size_t scan_scratch_words(size_t n) {
    size_t tiles = (n + kScanTile - 1) / kScanTile;
    return tiles + 64;
}

void scan_excl_u32(const uint32_t *in, uint32_t *out, size_t n, uint32_t *d_total, uint32_t *scratch,
                   hipStream_t st, const uint32_t *d_n) {
    if (n == 0) {
        if (d_total) hipMemsetAsync(d_total, 0, 4, st);
        return;
    }
    const size_t tiles = (n + kScanTile - 1) / kScanTile;
    if (tiles == 1) {
        k_scan_tile<<<1, kScanThreads, 0, st>>>(in, n, out, nullptr, d_total, d_n);
        return;
    }
    if (n <= kScanOneMax) {                    // one launch instead of reduce / partials / tiles
        k_scan_one<<<1, kScanOneThreads, 0, st>>>(in, (uint32_t)n, out, d_total, d_n);
        return;
    }
    uint32_t *partial = scratch;
    k_scan_reduce<<<(unsigned)tiles, kScanThreads, 0, st>>>(in, n, partial, d_n);
    k_scan_small<<<1, 1024, 0, st>>>(partial, tiles, d_total);
    k_scan_tile<<<(unsigned)tiles, kScanThreads, 0, st>>>(in, n, out, partial, nullptr, d_n);
}

}  // namespace sky
