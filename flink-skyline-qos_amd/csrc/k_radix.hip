// k_radix.hip — stable LSD radix sort of (u64 key, u32 value) pairs, 8-bit digits.
//
// Per pass:  k_radix_hist   (per-tile digit histogram, LDS atomics, per-wave copies)
//            scan           (digit-major [256][tiles] offsets, k_scan.hip)
//            k_radix_scatter(stable tile-local ranks from wave64 ballots; the tile is
//                            staged in LDS in digit order and written out as
//                            contiguous runs, so HBM writes are coalesced)
// Only bytes that differ between keys are sorted (OR/AND reduction first).
#include "sky_internal.h"

namespace sky {

constexpr int kRadixThreads = 256;
constexpr int kRadixItems = 16;
constexpr int kRadixTile = kRadixThreads * kRadixItems;   // 4096

__global__ __launch_bounds__(256) void k_key_orand(const uint64_t *__restrict__ keys, uint32_t m,
                                                   unsigned long long *__restrict__ orand) {
    uint64_t o = 0, a = ~0ull;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
        uint64_t k = keys[i];
        o |= k; a &= k;
    }
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) {
        o |= __shfl_xor(o, s, 64);
        a &= __shfl_xor(a, s, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicOr(&orand[0], (unsigned long long)o);
        atomicAnd(&orand[1], (unsigned long long)a);
    }
}

__global__ __launch_bounds__(kRadixThreads) void k_radix_hist(const uint64_t *__restrict__ keys, uint32_t m,
                                                              int shift, uint32_t ntiles,
                                                              uint32_t *__restrict__ hist) {
    __shared__ uint32_t s_h[4][256];
    const int t = threadIdx.x, w = t >> 6;
#pragma unroll
    for (int i = 0; i < 4; i++) s_h[i][t] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * kRadixTile;
#pragma unroll
    for (int r = 0; r < kRadixItems; r++) {
        const uint32_t i = base + r * kRadixThreads + t;
        if (i < m) atomicAdd(&s_h[w][(uint32_t)(keys[i] >> shift) & 255u], 1u);
    }
    __syncthreads();
    hist[(size_t)t * ntiles + blockIdx.x] = s_h[0][t] + s_h[1][t] + s_h[2][t] + s_h[3][t];
}

__global__ __launch_bounds__(kRadixThreads) void k_radix_scatter(
    const uint64_t *__restrict__ keys_in, const uint32_t *__restrict__ vals_in,
    uint64_t *__restrict__ keys_out, uint32_t *__restrict__ vals_out, uint32_t m, int shift,
    uint32_t ntiles, const uint32_t *__restrict__ offs) {
    __shared__ uint64_t s_key[kRadixTile];
    __shared__ uint32_t s_val[kRadixTile];
    __shared__ uint32_t s_cnt[4][256];
    __shared__ uint32_t s_wb[4][256];
    __shared__ uint32_t s_run[256];
    __shared__ uint32_t s_start[256];
    __shared__ uint32_t s_goff[256];
    __shared__ uint32_t s_w[4];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint32_t base = blockIdx.x * kRadixTile;
#pragma unroll
    for (int i = 0; i < 4; i++) s_cnt[i][t] = 0;
    s_run[t] = 0;
    s_goff[t] = offs[(size_t)t * ntiles + blockIdx.x];
    __syncthreads();

    uint64_t k[kRadixItems];
    uint32_t v[kRadixItems];
    uint32_t rk[kRadixItems];
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
    for (int r = 0; r < kRadixItems; r++) {
        const uint32_t i = base + r * kRadixThreads + t;
        const bool valid = i < m;
        k[r] = valid ? keys_in[i] : 0ull;
        v[r] = valid ? vals_in[i] : 0u;
        const uint32_t d = (uint32_t)(k[r] >> shift) & 255u;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        const uint32_t pre = __popcll(peers & lt_mask);
        if (valid && pre == 0) s_cnt[w][d] = __popcll(peers);
        __syncthreads();
        {
            const uint32_t c0 = s_cnt[0][t], c1 = s_cnt[1][t], c2 = s_cnt[2][t], c3 = s_cnt[3][t];
            const uint32_t run = s_run[t];
            s_wb[0][t] = run;
            s_wb[1][t] = run + c0;
            s_wb[2][t] = run + c0 + c1;
            s_wb[3][t] = run + c0 + c1 + c2;
            s_run[t] = run + c0 + c1 + c2 + c3;
            s_cnt[0][t] = 0; s_cnt[1][t] = 0; s_cnt[2][t] = 0; s_cnt[3][t] = 0;
        }
        __syncthreads();
        rk[r] = valid ? s_wb[w][d] + pre : 0xffffffffu;
    }
    // tile-local digit starts
    {
        const int lanei = t & 63;
        uint32_t c = s_run[t];
        uint32_t inc = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            uint32_t y = __shfl_up(inc, o, 64);
            if (lanei >= o) inc += y;
        }
        if (lanei == 63) s_w[w] = inc;
        __syncthreads();
        uint32_t wb = 0;
        for (int i = 0; i < w; i++) wb += s_w[i];
        s_start[t] = wb + inc - c;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRadixItems; r++) {
        if (rk[r] != 0xffffffffu) {
            const uint32_t d = (uint32_t)(k[r] >> shift) & 255u;
            const uint32_t p = s_start[d] + rk[r];
            s_key[p] = k[r];
            s_val[p] = v[r];
        }
    }
    __syncthreads();
    const uint32_t nvalid = m - base < (uint32_t)kRadixTile ? m - base : (uint32_t)kRadixTile;
#pragma unroll
    for (int r = 0; r < kRadixItems; r++) {
        const uint32_t q = r * kRadixThreads + t;
        if (q < nvalid) {
            const uint64_t kk = s_key[q];
            const uint32_t d = (uint32_t)(kk >> shift) & 255u;
            const uint32_t dst = s_goff[d] + (q - s_start[d]);
            keys_out[dst] = kk;
            vals_out[dst] = s_val[q];
        }
    }
}

size_t radix_scratch_words(size_t m) {
    size_t tiles = (m + kRadixTile - 1) / kRadixTile;
    return 2 * 256 * tiles + scan_scratch_words(256 * tiles) + 16;
}

// Sorts (keys, vals) by key; ping-pongs with (keys_alt, vals_alt).  Returns true if
// the result ended in the alt buffers.  `orand_host` = {OR, AND} of all keys (host
// computed by caller via radix_key_orand) selects which bytes to sort.
bool radix_sort_pairs(uint64_t *keys, uint32_t *vals, uint64_t *keys_alt, uint32_t *vals_alt, uint32_t m,
                      uint64_t varying_bits, uint32_t *scratch, hipStream_t st) {
    if (m <= 1 || varying_bits == 0) return false;
    const uint32_t tiles = (m + kRadixTile - 1) / kRadixTile;
    uint32_t *hist = scratch;
    uint32_t *offs = scratch + 256 * (size_t)tiles;
    uint32_t *scan_tmp = offs + 256 * (size_t)tiles;
    bool alt = false;
    for (int byte = 0; byte < 8; byte++) {
        if (((varying_bits >> (8 * byte)) & 0xffull) == 0) continue;
        const int shift = 8 * byte;
        const uint64_t *kin = alt ? keys_alt : keys;
        const uint32_t *vin = alt ? vals_alt : vals;
        uint64_t *kout = alt ? keys : keys_alt;
        uint32_t *vout = alt ? vals : vals_alt;
        k_radix_hist<<<tiles, kRadixThreads, 0, st>>>(kin, m, shift, tiles, hist);
        scan_excl_u32(hist, offs, 256 * (size_t)tiles, nullptr, scan_tmp, st);
        k_radix_scatter<<<tiles, kRadixThreads, 0, st>>>(kin, vin, kout, vout, m, shift, tiles, offs);
        alt = !alt;
    }
    return alt;
}

void radix_key_orand(const uint64_t *keys, uint32_t m, unsigned long long *d_orand, hipStream_t st) {
    unsigned long long init[2] = {0ull, ~0ull};
    hipMemcpyAsync(d_orand, init, sizeof(init), hipMemcpyHostToDevice, st);
    unsigned blocks = (unsigned)((m + 255) / 256);
    if (blocks > 2048) blocks = 2048;
    if (blocks == 0) blocks = 1;
    k_key_orand<<<blocks, 256, 0, st>>>(keys, m, d_orand);
}

}  // namespace sky
