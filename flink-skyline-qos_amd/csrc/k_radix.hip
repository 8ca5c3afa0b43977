// k_radix.hip — stable LSD radix sort of (u64 key, u32 value) pairs, 8-bit digits,
// one kernel per pass ("onesweep": decoupled look-back instead of a per-pass scan).
//
//   k_rs_hist_all   digit histograms of EVERY pass in one read of the keys (the
//                   global count of a digit does not depend on the key order)
//   k_rs_scan_all   per pass: exclusive scan -> global digit bases
//   k_rs_onesweep   per pass: a tile (taken in launch order from an atomic ticket)
//                   ranks its keys stably (wave64 ballots), publishes its digit
//                   counts, looks back over the earlier tiles' published counts for
//                   its exclusive prefix (bounded spin), then writes the tile staged
//                   in LDS in digit order as contiguous runs (coalesced)
// Only bytes that differ between keys are sorted (OR/AND reduction first).
#include <cstdlib>
#include "knobs.h"

#include "sky_internal.h"

namespace sky {

constexpr int kRadixThreads = 256;
constexpr int kRadixItems = 4;
constexpr int kRadixTile = kRadixThreads * kRadixItems;   // 1024 (short tiles: more workgroups in flight)

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

struct RsShifts { int s[8]; };

__global__ __launch_bounds__(kRadixThreads) void k_rs_hist_all(const uint64_t *__restrict__ keys, uint32_t m,
                                                               RsShifts shifts, int npass,
                                                               uint32_t *__restrict__ ghist) {
    __shared__ uint32_t s_h[8][256];
    const int t = threadIdx.x;
    for (int p = 0; p < 8; p++) s_h[p][t] = 0;
    __syncthreads();
    int sh[8];
#pragma unroll
    for (int p = 0; p < 8; p++) sh[p] = p < npass ? shifts.s[p] : 0;
    for (uint32_t i = blockIdx.x * kRadixThreads + t; i < m; i += gridDim.x * kRadixThreads) {
        const uint64_t k = keys[i];
#pragma unroll
        for (int p = 0; p < 8; p++)
            if (p < npass) atomicAdd(&s_h[p][(uint32_t)(k >> sh[p]) & 255u], 1u);
    }
    __syncthreads();
    for (int p = 0; p < npass; p++)
        if (s_h[p][t]) atomicAdd(&ghist[p * 256 + t], s_h[p][t]);
}

__global__ __launch_bounds__(256) void k_rs_scan_all(uint32_t *__restrict__ ghist, int npass) {
    __shared__ uint32_t s_w[4];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    for (int p = 0; p < npass; p++) {
        const uint32_t c = ghist[p * 256 + t];
        uint32_t inc = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(inc, o, 64);
            if (lane >= o) inc += y;
        }
        if (lane == 63) s_w[w] = inc;
        __syncthreads();
        uint32_t wb = 0;
        for (int i = 0; i < w; i++) wb += s_w[i];
        ghist[p * 256 + t] = wb + inc - c;
        __syncthreads();
    }
}

// order-preserving compression of the varying key bits (the constant bits are equal
// in every key, so comparing the remaining bits in significance order is comparing
// the keys): runs of consecutive varying bits, LSB first
constexpr int kRsMaxRuns = 8;          // more runs of varying bits: sort the raw bytes
struct RsRuns { int n; int start[kRsMaxRuns], len[kRsMaxRuns]; };

__global__ __launch_bounds__(256) void k_rs_compress(const uint64_t *__restrict__ keys, uint32_t m, RsRuns runs,
                                                     uint64_t *__restrict__ dense) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const uint64_t k = keys[i];
    uint64_t o = 0;
    int pos = 0;
    // constant indices only: the run table stays in SGPRs loaded at wave start (a
    // dynamically indexed by-value kernel-argument array is read from the kernarg
    // buffer by late waves, and late waves of a long grid read it corrupted)
#pragma unroll
    for (int r = 0; r < kRsMaxRuns; r++) {
        if (r < runs.n) {
            const int l = runs.len[r];
            const uint64_t msk = l >= 64 ? ~0ull : ((1ull << l) - 1ull);
            o |= ((k >> runs.start[r]) & msk) << pos;
            pos += l;
        }
    }
    dense[i] = o;
}

// inverse of k_rs_compress: scatter the dense bits back and restore the constant bits;
// vals_src != nullptr: also move the values into the alt buffer (a kernel, not an
// async copy: a DMA copy engine read the previous kernel's values stale)
__global__ __launch_bounds__(256) void k_rs_expand(const uint64_t *__restrict__ dense, uint32_t m, RsRuns runs,
                                                   uint64_t const_bits, uint64_t *__restrict__ keys,
                                                   const uint32_t *__restrict__ vals_src,
                                                   uint32_t *__restrict__ vals_dst) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    if (vals_src) vals_dst[i] = vals_src[i];
    const uint64_t d = dense[i];
    uint64_t k = const_bits;
    int pos = 0;
#pragma unroll
    for (int r = 0; r < kRsMaxRuns; r++) {
        if (r < runs.n) {
            const int l = runs.len[r];
            const uint64_t msk = l >= 64 ? ~0ull : ((1ull << l) - 1ull);
            k |= ((d >> pos) & msk) << runs.start[r];
            pos += l;
        }
    }
    keys[i] = k;
}

constexpr uint32_t kRsAgg = 1u << 30, kRsInc = 2u << 30, kRsCount = (1u << 30) - 1;

// One LSD pass over ITEMS*256-key tiles.  Wave w of a tile owns the contiguous chunk
// [w*64*ITEMS, (w+1)*64*ITEMS): it ranks its keys digit by digit with 8 ballots per item
// and a per-wave running count in LDS (the peer group's leader updates it; the others get
// the old value by a shuffle), so the ranking needs no workgroup barrier per item; the
// order (wave, item, lane) is the index order, so the pass is stable.  Then: tile digit
// counts published, decoupled look-back for the exclusive prefix, keys staged in LDS in
// digit order, coalesced writes of each digit run.  Large tiles (ITEMS = 16) keep the
// runs of one digit long (write coalescing); short tiles (ITEMS = 4) keep more
// workgroups in flight for the small candidate sorts of a query.
template <int ITEMS>
__global__ __launch_bounds__(kRadixThreads) void k_rs_onesweep(
    const uint64_t *__restrict__ keys_in, const uint32_t *__restrict__ vals_in,
    uint64_t *__restrict__ keys_out, uint32_t *__restrict__ vals_out, uint32_t m, int shift,
    const uint32_t *__restrict__ gbase, uint32_t *__restrict__ status, uint32_t *__restrict__ ticket,
    uint32_t *__restrict__ err) {
    constexpr int TILE = kRadixThreads * ITEMS;
    constexpr int WCH = 64 * ITEMS;
    __shared__ uint64_t s_key[TILE];
    __shared__ uint32_t s_val[TILE];
    __shared__ uint32_t s_wc[4][256];
    __shared__ uint32_t s_run[256];
    __shared__ uint32_t s_start[256];
    __shared__ uint32_t s_goff[256];
    __shared__ uint32_t s_w[4];
    __shared__ uint32_t s_tile;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    // tiles are numbered in the order workgroups start: a tile only ever waits for
    // tiles that started before it (forward progress of the look-back)
    if (t == 0) s_tile = atomicAdd(ticket, 1u);
#pragma unroll
    for (int i = 0; i < 4; i++) s_wc[i][t] = 0;
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint32_t base = tile * TILE;

    uint64_t k[ITEMS];
    uint32_t v[ITEMS];
    uint32_t rk[ITEMS];
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        const uint32_t i = base + w * WCH + r * 64 + lane;
        const bool valid = i < m;
        k[r] = valid ? keys_in[i] : 0ull;
        v[r] = valid ? vals_in[i] : 0u;
    }
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        const uint32_t i = base + w * WCH + r * 64 + lane;
        const bool valid = i < m;
        const uint32_t d = (uint32_t)(k[r] >> shift) & 255u;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        const uint32_t pre = __popcll(peers & lt_mask);
        uint32_t old = 0;
        if (valid && pre == 0) {
            old = s_wc[w][d];
            s_wc[w][d] = old + __popcll(peers);
        }
        const int leader = peers ? __ffsll((long long)peers) - 1 : 0;
        old = __shfl(old, leader, 64);
        rk[r] = valid ? old + pre : 0xffffffffu;
    }
    __syncthreads();
    {   // digit t: wave bases within the tile and the tile aggregate
        const uint32_t c0 = s_wc[0][t], c1 = s_wc[1][t], c2 = s_wc[2][t], c3 = s_wc[3][t];
        s_wc[0][t] = 0;
        s_wc[1][t] = c0;
        s_wc[2][t] = c0 + c1;
        s_wc[3][t] = c0 + c1 + c2;
        s_run[t] = c0 + c1 + c2 + c3;
    }
    // publish this tile's digit count, look back for the exclusive prefix
    {
        const uint32_t agg = s_run[t];
        uint32_t *mine = status + (size_t)tile * 256 + t;
        uint32_t excl = 0;
        if (tile == 0) {
            __hip_atomic_store(mine, kRsInc | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_store(mine, kRsAgg | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            int64_t pt = (int64_t)tile - 1;
            uint32_t spins = 0;
            while (pt >= 0) {
                const uint32_t sv = __hip_atomic_load(status + (size_t)pt * 256 + t, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t f = sv & ~kRsCount;
                if (f == 0u) {
                    if (++spins > (1u << 24)) { atomicOr(err, kFlagRadixSpin); break; }   // bounded spin
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                excl += sv & kRsCount;
                if (f == kRsInc) break;
                pt--;
            }
            __hip_atomic_store(mine, kRsInc | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        s_goff[t] = gbase[t] + excl;
    }
    // tile-local digit starts
    {
        uint32_t c = s_run[t];
        uint32_t inc = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            uint32_t y = __shfl_up(inc, o, 64);
            if (lane >= o) inc += y;
        }
        if (lane == 63) s_w[w] = inc;
        __syncthreads();
        uint32_t wb = 0;
        for (int i = 0; i < w; i++) wb += s_w[i];
        s_start[t] = wb + inc - c;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        if (rk[r] != 0xffffffffu) {
            const uint32_t d = (uint32_t)(k[r] >> shift) & 255u;
            const uint32_t p = s_start[d] + s_wc[w][d] + rk[r];
            s_key[p] = k[r];
            s_val[p] = v[r];
        }
    }
    __syncthreads();
    const uint32_t nvalid = m - base < (uint32_t)TILE ? m - base : (uint32_t)TILE;
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
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

static thread_local int g_radix_last_passes = 0;
int radix_last_passes() { return g_radix_last_passes; }

// debug check (SKY_DEBUG >= 4): sorted, a permutation, keys match their source slots
__global__ __launch_bounds__(256) void k_rs_check(const uint64_t *__restrict__ orig, const uint64_t *__restrict__ skey,
                                                  const uint32_t *__restrict__ perm, uint32_t m,
                                                  uint32_t *__restrict__ seen, uint32_t *__restrict__ bad) {
    const uint32_t j = blockIdx.x * 256 + threadIdx.x;
    if (j >= m) return;
    if (j > 0 && skey[j - 1] > skey[j]) atomicOr(bad, 1u);
    const uint32_t s = perm[j];
    if (s >= m) { atomicOr(bad, 2u); return; }
    if (orig[s] != skey[j]) atomicOr(bad, 4u);
    if (atomicAdd(&seen[s], 1u) != 0u) atomicOr(bad, 8u);
}

void radix_debug_check(const uint64_t *orig, const uint64_t *skey, const uint32_t *perm, uint32_t m, uint32_t *seen,
                       uint32_t *bad, hipStream_t st) {
    (void)hipMemsetAsync(seen, 0, (size_t)m * 4, st);
    if (m) k_rs_check<<<(m + 255) / 256, 256, 0, st>>>(orig, skey, perm, m, seen, bad);
}

size_t radix_scratch_words(size_t m) {
    const size_t tiles = (m + kRadixTile - 1) / kRadixTile;
    return 8 * 256 + 8 * 256 * tiles + 8 + 8 + 64 + 4 * m + 4 + 2 * m;
}

// Sorts (keys, vals) by key; ping-pongs with (keys_alt, vals_alt).  Returns true if
// the result ended in the alt buffers.  key_or / key_and: OR and AND of all keys; the
// varying bits are compressed into dense keys first when that saves passes (the
// scratch holds the dense ping-pong pair and an index array; the original keys
// are gathered back at the end).
bool radix_sort_pairs(uint64_t *keys, uint32_t *vals, uint64_t *keys_alt, uint32_t *vals_alt, uint32_t m,
                      uint64_t key_or, uint64_t key_and, uint32_t *scratch, uint32_t *err, hipStream_t st,
                      hipError_t *launch_err) {
    const uint64_t varying_bits = key_or ^ key_and;
    if (launch_err) *launch_err = hipSuccess;
    g_radix_last_passes = 0;
    if (m <= 1 || varying_bits == 0) return false;
    // 6144-key tiles for large sorts (fewer tiles: less look-back, longer digit runs per tile;
    // 100M pairs: 24 keys per thread 5.86 ms, 16: 6.99, 12: 7.45, 8: 8.44, 32 (1 wave per SIMD):
    // 7.43), 1024 for the query's candidates
    const bool big = m >= (1u << 22);
    static const int big_items = [] {   // SKY_RADIX_ITEMS: keys per thread of the large-sort tiles (A/B knob)
        const char *e = SKY_MEASURE_ENV("SKY_RADIX_ITEMS");
        const int v = e ? atoi(e) : 24;
        return v == 8 || v == 12 || v == 16 || v == 24 || v == 32 ? v : 24;
    }();
    const uint32_t tile_sz = big ? (uint32_t)(kRadixThreads * big_items) : (uint32_t)kRadixTile;
    const uint32_t tiles = (m + tile_sz - 1) / tile_sz;
    RsRuns runs{};
    int nbits = 0;
    bool too_many_runs = false;
    for (int b = 0; b < 64;) {
        if (!((varying_bits >> b) & 1ull)) { b++; continue; }
        int e = b;
        while (e < 64 && ((varying_bits >> e) & 1ull)) e++;
        if (runs.n == kRsMaxRuns) { too_many_runs = true; break; }
        runs.start[runs.n] = b;
        runs.len[runs.n] = e - b;
        runs.n++;
        nbits += e - b;
        b = e;
    }
    int byte_passes = 0;
    for (int byte = 0; byte < 8; byte++) byte_passes += ((varying_bits >> (8 * byte)) & 0xffull) ? 1 : 0;
    const int dense_passes = (nbits + 7) / 8;
    static const int comp_mode = [] {            // SKY_RADIX_COMPRESS=0 disables (debug)
        const char *e = SKY_MEASURE_ENV("SKY_RADIX_COMPRESS");
        return e ? atoi(e) : 1;
    }();
    const bool compress = comp_mode && !too_many_runs && dense_passes < byte_passes;
    RsShifts shifts{};
    int npass = 0;
    if (compress) {
        for (int p = 0; p < dense_passes; p++) shifts.s[npass++] = 8 * p;
    } else {
        for (int byte = 0; byte < 8; byte++)
            if ((varying_bits >> (8 * byte)) & 0xffull) shifts.s[npass++] = 8 * byte;
    }
    uint32_t *ghist = scratch;                                   // [8][256]
    uint32_t *status = ghist + 8 * 256;                          // [8][tiles][256]
    uint32_t *tickets = status + (size_t)8 * 256 * tiles;        // [8]
    uint64_t *dense = reinterpret_cast<uint64_t *>(
        (reinterpret_cast<uintptr_t>(tickets + 16) + 15) & ~uintptr_t(15));   // [2][m]
    FillSet fill;                                                // histograms, look-back status, tickets
    fill.add(scratch, ((size_t)8 * 256 + (size_t)npass * 256 * tiles) * 4);
    fill.add(tickets, 8 * 4);
    const hipError_t fe = fill.launch(st);
    if (fe != hipSuccess && launch_err) *launch_err = fe;
    uint64_t *k0 = keys, *k1 = keys_alt;
    if (compress) {
        k0 = dense;
        k1 = dense + m;
        k_rs_compress<<<(m + 255) / 256, 256, 0, st>>>(keys, m, runs, k0);
    }
    unsigned hb = tiles < 1024 ? tiles : 1024;
    k_rs_hist_all<<<hb, kRadixThreads, 0, st>>>(k0, m, shifts, npass, ghist);
    k_rs_scan_all<<<1, 256, 0, st>>>(ghist, npass);
    bool alt = false;
    g_radix_last_passes = npass;
    for (int p = 0; p < npass; p++) {
        const uint64_t *kin = alt ? k1 : k0;
        const uint32_t *vin = alt ? vals_alt : vals;
        uint64_t *kout = alt ? k0 : k1;
        uint32_t *vout = alt ? vals : vals_alt;
        if (big) {
            uint32_t *stp = status + (size_t)p * 256 * tiles;
            const uint32_t *gb = ghist + p * 256;
            if (big_items == 8)
                k_rs_onesweep<8><<<tiles, kRadixThreads, 0, st>>>(kin, vin, kout, vout, m, shifts.s[p], gb, stp, tickets + p, err);
            else if (big_items == 12)
                k_rs_onesweep<12><<<tiles, kRadixThreads, 0, st>>>(kin, vin, kout, vout, m, shifts.s[p], gb, stp, tickets + p, err);
            else if (big_items == 32)
                k_rs_onesweep<32><<<tiles, kRadixThreads, 0, st>>>(kin, vin, kout, vout, m, shifts.s[p], gb, stp, tickets + p, err);
            else if (big_items == 24)
                k_rs_onesweep<24><<<tiles, kRadixThreads, 0, st>>>(kin, vin, kout, vout, m, shifts.s[p], gb, stp, tickets + p, err);
            else
                k_rs_onesweep<16><<<tiles, kRadixThreads, 0, st>>>(kin, vin, kout, vout, m, shifts.s[p], gb, stp, tickets + p, err);
        }
        else
            k_rs_onesweep<kRadixItems><<<tiles, kRadixThreads, 0, st>>>(kin, vin, kout, vout, m, shifts.s[p],
                                                                        ghist + p * 256,
                                                                        status + (size_t)p * 256 * tiles,
                                                                        tickets + p, err);
        alt = !alt;
    }
    if (!compress) return alt;
    // sorted keys -> keys_alt (expanded back), values -> vals_alt
    k_rs_expand<<<(m + 255) / 256, 256, 0, st>>>(alt ? k1 : k0, m, runs, key_and & ~varying_bits, keys_alt,
                                                 alt ? nullptr : vals, vals_alt);
    return true;
}

void radix_key_orand(const uint64_t *keys, uint32_t m, unsigned long long *d_orand, hipStream_t st) {
    // OR accumulator = 0, AND accumulator = all ones (memsets: no host buffer whose
    // lifetime would have to outlast an asynchronous copy)
    hipMemsetAsync(d_orand, 0, 8, st);
    hipMemsetAsync(d_orand + 1, 0xff, 8, st);
    unsigned blocks = (unsigned)((m + 255) / 256);
    if (blocks > 2048) blocks = 2048;
    if (blocks == 0) blocks = 1;
    k_key_orand<<<blocks, 256, 0, st>>>(keys, m, d_orand);
}

}  // namespace sky
