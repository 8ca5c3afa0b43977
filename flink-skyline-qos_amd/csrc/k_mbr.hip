// k_mbr.hip — both skyline levels of a LARGE representative set in one all-pairs pass
// with bounding-box pruning: no SFS rounds, no host round trips.
//
// Representatives (distinct candidate vectors, FlinkSkyline.java:417-444 / :548-566 as a
// set computation): y is in L_k iff no rep of its partition dominates it, and in G iff no
// rep at all dominates it (a dominator outside the union of the L_k is itself dominated
// by a member of it: transitivity), the same rule as the small-set brute path (k_sfs.hip).
//
//   k_mbr_minmax   per-dimension min / max of an order-preserving u32 image of the values
//   k_mbr_code     sort key = partition << (b*D) | Hilbert index of the values quantised to
//                  b bits per dimension (nearby vectors -> nearby positions)
//   radix sort     (k_radix.hip) of the keys, rep index as value
//   k_mbr_tiles    one wave per tile of 64 consecutive positions: rows gathered into tile
//                  order, the tile's bounding box (per-dimension min and max), partition
//                  range and its sub-box min corners (8 rows each for packed u16 rows)
//   k_mbr_groups   min corner + partition range of 64 consecutive tiles
//   k_mbr_cost /   the work queue: per y tile the number of x groups its box reaches, split
//   k_mbr_order    above the average into items, heaviest first
//   k_mbr_pairs    persistent one-wave workgroups take items (a y tile, lane = y, or a share
//                  of its reachable groups).  The x groups' and tiles' min corners are scanned
//                  64 at a time (lane = group / tile) against the y tile's max corner; for a
//                  passing tile every live y is tested against the sub-box corners (scalar
//                  loads, one ballot per sub-box), the surviving (y, sub-box) entries are
//                  compared 8 per wave instruction from LDS, hits are LDS atomic ORs into the
//                  y's fate word.  A lane is done once a rep of its own partition dominates it.
//   k_mbr_finish   alive_l / alive_g per rep
//
// The order only decides how much is pruned, never the result: any bounding box contains
// its rows, so a skipped tile holds no dominator.  On the labelled std-anti 8D stream about
// 2 % of the tile pairs survive the box test (tools/mbr_sim note in DESIGN.md §2.2).
#include "sky_internal.h"
#include "knobs.h"

namespace sky {

typedef unsigned short mbr_u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pk_satsub(uint32_t x, uint32_t y) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(__builtin_bit_cast(mbr_u16x2, x),
                                                                      __builtin_bit_cast(mbr_u16x2, y)));
}
__device__ __forceinline__ uint32_t pk_min(uint32_t x, uint32_t y) {
    return __builtin_bit_cast(uint32_t,
                              __builtin_elementwise_min(__builtin_bit_cast(mbr_u16x2, x), __builtin_bit_cast(mbr_u16x2, y)));
}
__device__ __forceinline__ uint32_t pk_max(uint32_t x, uint32_t y) {
    return __builtin_bit_cast(uint32_t,
                              __builtin_elementwise_max(__builtin_bit_cast(mbr_u16x2, x), __builtin_bit_cast(mbr_u16x2, y)));
}
// (an LDS-DMA variant of the pair pass's x-tile prefetch measured slower: profiles/r05_dominance_ab.txt)
__device__ __forceinline__ uint64_t wballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
// set bits of m below this lane (two VALU: mbcnt)
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint32_t ord_f32(float f) {       // order-preserving image (no NaN here)
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// ---- row formats: NW 32-bit words per row ------------------------------------------
// packed u16 pairs (k_dom16.hip layout): x <= y everywhere  <=>  OR_w sat(x_w - y_w) == 0
template <int D, int W>
struct RowU16 {
    static constexpr int NW = W;
    using Pair = RowU16<2 * W, W>;                 // the pair pass reads only the W words
    static __device__ __forceinline__ bool le(const uint32_t *x, const uint32_t *y) {
        uint32_t r = 0;
#pragma unroll
        for (int w = 0; w < W; w++) r |= pk_satsub(x[w], y[w]);
        return r == 0u;
    }
    static __device__ __forceinline__ void cmin(uint32_t *a, const uint32_t *b) {
#pragma unroll
        for (int w = 0; w < W; w++) a[w] = pk_min(a[w], b[w]);
    }
    static __device__ __forceinline__ void cmax(uint32_t *a, const uint32_t *b) {
#pragma unroll
        for (int w = 0; w < W; w++) a[w] = pk_max(a[w], b[w]);
    }
    static __device__ __forceinline__ void ident_min(uint32_t *a) {
#pragma unroll
        for (int w = 0; w < W; w++) a[w] = 0xffffffffu;
    }
    static __device__ __forceinline__ void ident_max(uint32_t *a) {
#pragma unroll
        for (int w = 0; w < W; w++) a[w] = 0u;
    }
    static __device__ __forceinline__ uint32_t ord(const uint32_t *r, int d) {
        return (r[d >> 1] >> ((d & 1) * 16)) & 0xffffu;
    }
};

// f32 values (every candidate value exactly an f32), rows padded to 4 floats
template <int D>
struct RowF32 {
    static constexpr int NW = padded_dims<float>(D);
    using Pair = RowF32<D>;
    static __device__ __forceinline__ bool le(const uint32_t *x, const uint32_t *y) {
        bool r = true;
#pragma unroll
        for (int d = 0; d < D; d++) r &= __uint_as_float(x[d]) <= __uint_as_float(y[d]);
        return r;
    }
    static __device__ __forceinline__ void cmin(uint32_t *a, const uint32_t *b) {
#pragma unroll
        for (int d = 0; d < D; d++) a[d] = __float_as_uint(fminf(__uint_as_float(a[d]), __uint_as_float(b[d])));
    }
    static __device__ __forceinline__ void cmax(uint32_t *a, const uint32_t *b) {
#pragma unroll
        for (int d = 0; d < D; d++) a[d] = __float_as_uint(fmaxf(__uint_as_float(a[d]), __uint_as_float(b[d])));
    }
    static __device__ __forceinline__ void ident_min(uint32_t *a) {
#pragma unroll
        for (int w = 0; w < NW; w++) a[w] = 0x7f800000u;       // +inf
    }
    static __device__ __forceinline__ void ident_max(uint32_t *a) {
#pragma unroll
        for (int w = 0; w < NW; w++) a[w] = 0xff800000u;       // -inf
    }
    static __device__ __forceinline__ uint32_t ord(const uint32_t *r, int d) { return ord_f32(__uint_as_float(r[d])); }
};

// f64 values, rows padded to 2 doubles
template <int D>
struct RowF64 {
    static constexpr int NW = 2 * padded_dims<double>(D);
    using Pair = RowF64<D>;
    static __device__ __forceinline__ double get(const uint32_t *r, int d) {
        return __hiloint2double((int)r[2 * d + 1], (int)r[2 * d]);
    }
    static __device__ __forceinline__ void put(uint32_t *r, int d, double v) {
        r[2 * d] = (uint32_t)__double2loint(v);
        r[2 * d + 1] = (uint32_t)__double2hiint(v);
    }
    static __device__ __forceinline__ bool le(const uint32_t *x, const uint32_t *y) {
        bool r = true;
#pragma unroll
        for (int d = 0; d < D; d++) r &= get(x, d) <= get(y, d);
        return r;
    }
    static __device__ __forceinline__ void cmin(uint32_t *a, const uint32_t *b) {
#pragma unroll
        for (int d = 0; d < D; d++) put(a, d, fmin(get(a, d), get(b, d)));
    }
    static __device__ __forceinline__ void cmax(uint32_t *a, const uint32_t *b) {
#pragma unroll
        for (int d = 0; d < D; d++) put(a, d, fmax(get(a, d), get(b, d)));
    }
    static __device__ __forceinline__ void ident_min(uint32_t *a) {
#pragma unroll
        for (int d = 0; d < NW / 2; d++) put(a, d, __longlong_as_double(0x7ff0000000000000ll));
    }
    static __device__ __forceinline__ void ident_max(uint32_t *a) {
#pragma unroll
        for (int d = 0; d < NW / 2; d++) put(a, d, __longlong_as_double((long long)0xfff0000000000000ull));
    }
    static __device__ __forceinline__ uint32_t ord(const uint32_t *r, int d) { return ord_f32((float)get(r, d)); }
};

// ---- the sort key --------------------------------------------------------------------
template <class R, int D>
__global__ __launch_bounds__(kThreads) void k_mbr_minmax(const uint32_t *__restrict__ rows, uint32_t mr,
                                                         uint32_t *__restrict__ mm) {
    uint32_t lo[D], hi[D];
#pragma unroll
    for (int d = 0; d < D; d++) { lo[d] = 0xffffffffu; hi[d] = 0u; }
    for (uint32_t j = blockIdx.x * kThreads + threadIdx.x; j < mr; j += gridDim.x * kThreads) {
        const uint32_t *r = rows + (size_t)j * R::NW;
#pragma unroll
        for (int d = 0; d < D; d++) {
            const uint32_t o = R::ord(r, d);
            lo[d] = min(lo[d], o);
            hi[d] = max(hi[d], o);
        }
    }
    __shared__ uint32_t s_lo[kThreads / 64][D], s_hi[kThreads / 64][D];
#pragma unroll
    for (int d = 0; d < D; d++) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            lo[d] = min(lo[d], (uint32_t)__shfl_xor((int)lo[d], o, 64));
            hi[d] = max(hi[d], (uint32_t)__shfl_xor((int)hi[d], o, 64));
        }
        if ((threadIdx.x & 63) == 0) {
            s_lo[threadIdx.x >> 6][d] = lo[d];
            s_hi[threadIdx.x >> 6][d] = hi[d];
        }
    }
    __syncthreads();
    if (threadIdx.x < D) {          // one atomic per dimension and block
        uint32_t a = s_lo[0][threadIdx.x], b = s_hi[0][threadIdx.x];
        for (int q = 1; q < kThreads / 64; q++) {
            a = min(a, s_lo[q][threadIdx.x]);
            b = max(b, s_hi[q][threadIdx.x]);
        }
        atomicMin(&mm[threadIdx.x], a);
        atomicMax(&mm[D + threadIdx.x], b);
    }
}

template <class R, int D>
__global__ __launch_bounds__(kThreads) void k_mbr_code(const uint32_t *__restrict__ rows,
                                                       const uint64_t *__restrict__ rep_key, uint32_t mr, int bits,
                                                       const uint32_t *__restrict__ mm, int hilbert,
                                                       uint64_t *__restrict__ code, uint32_t *__restrict__ idx) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= mr) return;
    const uint32_t *r = rows + (size_t)j * R::NW;
    uint32_t q[D];
#pragma unroll
    for (int d = 0; d < D; d++) {
        const uint64_t span = (uint64_t)mm[D + d] - mm[d] + 1u;
        q[d] = (uint32_t)((((uint64_t)(R::ord(r, d) - mm[d])) << bits) / span);
    }
    if (hilbert) {
        // Hilbert order instead of Morton: no jumps across the cell boundaries, so the 64-row
        // tiles' boxes are tighter (by simulation on std-anti 8D, tools/mbr_sim.py: 40 % fewer
        // reachable tiles per y, 33 % fewer pair tests).  Skilling's axes -> transposed index
        // (AIP Conf. Proc. 707, 2004); interleaving the transposed bits gives the index.
        for (uint32_t Q = 1u << (bits - 1); Q > 1u; Q >>= 1) {
            const uint32_t Pm = Q - 1u;
#pragma unroll
            for (int d = 0; d < D; d++) {
                if (q[d] & Q) {
                    q[0] ^= Pm;
                } else {
                    const uint32_t t = (q[0] ^ q[d]) & Pm;
                    q[0] ^= t;
                    q[d] ^= t;
                }
            }
        }
#pragma unroll
        for (int d = 1; d < D; d++) q[d] ^= q[d - 1];
        uint32_t t = 0;
        for (uint32_t Q = 1u << (bits - 1); Q > 1u; Q >>= 1)
            if (q[D - 1] & Q) t ^= Q - 1u;
#pragma unroll
        for (int d = 0; d < D; d++) q[d] ^= t;
    }
    uint64_t c = 0;
    for (int b = bits - 1; b >= 0; b--)
#pragma unroll
        for (int d = 0; d < D; d++) c = (c << 1) | ((q[d] >> b) & 1u);
    code[j] = ((rep_key[j] >> 56) << (bits * D)) | c;
    idx[j] = j;
}

// ---- tiles: rows in sorted order, bounding boxes, partition ranges ---------------------
constexpr int kMbrT = 64;   // rows per tile (= one wave)
// sub-boxes per tile whose min corners the pair pass tests each y against before comparing rows:
// 8 boxes of 8 rows for packed u16 rows (the corners of a tile are 32 words: one pair of scalar
// loads), 4 of 16 rows for f32 / f64 rows (32 / 64 words).  tsub holds kMbrSubMax corners per tile.
// (4-row boxes for packed u16 rows, 16 per tile: 3.7x fewer pair tests at std-anti 8D 10M but twice
// the sub-box passes; the pass took 21.1 vs 19.6 ms, profiles/r05_dominance_ab.txt)
template <class R>
constexpr int mbr_subs() { return R::NW <= 4 ? 8 : 4; }

template <class R>
__global__ __launch_bounds__(kThreads) void k_mbr_tiles(const uint32_t *__restrict__ rows,
                                                        const uint64_t *__restrict__ rep_key,
                                                        const uint32_t *__restrict__ perm, uint32_t mr,
                                                        uint32_t ntiles, uint32_t *__restrict__ trows,
                                                        uint32_t *__restrict__ tpart, uint32_t *__restrict__ tmin,
                                                        uint32_t *__restrict__ tmax, uint32_t *__restrict__ tprange,
                                                        uint32_t *__restrict__ tsub) {
    constexpr int NW = R::NW;
    const uint32_t tile = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    if (tile >= ntiles) return;
    const uint32_t pos = tile * kMbrT + (threadIdx.x & 63);
    const bool valid = pos < mr;
    uint32_t v[NW], mn[NW], mx[NW];
    uint32_t pk = 0xffffffffu, pl, ph;
    if (valid) {
        const uint32_t rep = perm[pos];
        const uint32_t *r = rows + (size_t)rep * NW;
#pragma unroll
        for (int w = 0; w < NW; w++) v[w] = r[w];
#pragma unroll
        for (int w = 0; w < NW; w++) trows[(size_t)pos * NW + w] = v[w];
        pk = (uint32_t)(rep_key[rep] >> 56);
        tpart[pos] = pk;
#pragma unroll
        for (int w = 0; w < NW; w++) { mn[w] = v[w]; mx[w] = v[w]; }
        pl = ph = pk;
    } else {
        R::ident_min(mn);
        R::ident_max(mx);
        pl = 0xffffffffu;
        ph = 0u;
    }
    // offsets below the sub-box size first: the sub-boxes' min corners (k_mbr_pairs tests a y
    // against them before comparing rows), then the rest: the whole tile
    constexpr int S = mbr_subs<R>(), RS = kMbrT / S;
#pragma unroll
    for (int o = 1; o <= 32; o <<= 1) {
        uint32_t a[NW], b[NW];
#pragma unroll
        for (int w = 0; w < NW; w++) {
            a[w] = (uint32_t)__shfl_xor((int)mn[w], o, 64);
            b[w] = (uint32_t)__shfl_xor((int)mx[w], o, 64);
        }
        R::cmin(mn, a);
        R::cmax(mx, b);
        pl = min(pl, (uint32_t)__shfl_xor((int)pl, o, 64));
        ph = max(ph, (uint32_t)__shfl_xor((int)ph, o, 64));
        if (o == RS / 2 && (threadIdx.x & (RS - 1)) == 0) {
#pragma unroll
            for (int w = 0; w < NW; w++) tsub[((size_t)tile * S + ((threadIdx.x & 63) / RS)) * NW + w] = mn[w];
        }
    }
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int w = 0; w < NW; w++) {
            tmin[(size_t)w * ntiles + tile] = mn[w];
            tmax[(size_t)w * ntiles + tile] = mx[w];
        }
        tprange[tile] = pl | (ph << 16);
    }
}

// groups of 64 consecutive tiles: min corner and partition range (one wave per group); the
// pair pass skips a whole group whose corner is not <= the y tile's max corner
constexpr int kMbrG = 64;   // tiles per group

template <class R>
__global__ __launch_bounds__(kThreads) void k_mbr_groups(const uint32_t *__restrict__ tmin,
                                                         const uint32_t *__restrict__ tprange, uint32_t ntiles,
                                                         uint32_t ngroups, uint32_t *__restrict__ gmin,
                                                         uint32_t *__restrict__ gprange) {
    constexpr int NW = R::NW;
    const uint32_t g = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    if (g >= ngroups) return;
    const uint32_t t = g * kMbrG + (threadIdx.x & 63);
    uint32_t mn[NW], pl = 0xffffffffu, ph = 0u;
    R::ident_min(mn);
    if (t < ntiles) {
#pragma unroll
        for (int w = 0; w < NW; w++) mn[w] = tmin[(size_t)w * ntiles + t];
        const uint32_t r = tprange[t];
        pl = r & 0xffffu;
        ph = r >> 16;
    }
#pragma unroll
    for (int o = 1; o <= 32; o <<= 1) {
        uint32_t a[NW];
#pragma unroll
        for (int w = 0; w < NW; w++) a[w] = (uint32_t)__shfl_xor((int)mn[w], o, 64);
        R::cmin(mn, a);
        pl = min(pl, (uint32_t)__shfl_xor((int)pl, o, 64));
        ph = max(ph, (uint32_t)__shfl_xor((int)ph, o, 64));
    }
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int w = 0; w < NW; w++) gmin[(size_t)w * ngroups + g] = mn[w];
        gprange[g] = pl | (ph << 16);
    }
}

// threads per workgroup of the pair pass: ONE wave.  A workgroup's resources are held until its
// last wave exits, and the y tiles' work varies by orders of magnitude, so 4-wave workgroups kept
// slots occupied by finished waves (measured: ~2 resident waves per SIMD of the 6 the registers
// allow)
constexpr int kMbrPairThreads = 64;

// the y tiles of the pair pass (the x tiles' set, or another: the multi-GPU merge's own rows)
struct MbrYSet {
    const uint32_t *trows, *tpart, *tmax, *tprange;
    uint32_t mr, ntiles;
};

// ---- the pair pass's work queue ----------------------------------------------------------
// The work of a y tile varies by orders of magnitude (a loose box reaches many x tiles), and a
// launch waits for its slowest wave: on std-anti 8D 2M one y tile took the whole 6.6 ms pass
// while the rest of the chip idled for its second half (SKY_MBR_DBG=8 work-item timeline,
// DESIGN.md §2.2).  So the work is cut into items and handed out heaviest first: a y tile's
// cost is the number of x groups its box reaches (k_mbr_cost); a tile above the average cost
// is split into up to kMbrSplitMax items that take every s-th reachable group (the reachable
// groups cluster, so interleaving balances the parts), and every wave of the pair pass takes
// items from a ticket counter until none is left.
template <class R, int YT>
__global__ __launch_bounds__(kThreads) void k_mbr_cost(const uint32_t *__restrict__ gmin, uint32_t ngroups,
                                                       MbrYSet ys, uint32_t *__restrict__ lpt) {
    // lane = y unit (YT consecutive y tiles, k_mbr_pairs' work item): the groups' min corners are
    // wave-uniform (scalar loads, read once per wave instead of once per unit), one box test per
    // (unit, group) against the unit's max corner
    constexpr int NW = R::NW;
    const uint32_t nyu = (ys.ntiles + YT - 1) / YT;
    const uint32_t yt = blockIdx.x * kThreads + threadIdx.x;
    const bool valid = yt < nyu;
    uint32_t ymax[NW];
    R::ident_max(ymax);
#pragma unroll
    for (int t = 0; t < YT; t++) {
        const uint32_t tt = min(min(yt, nyu - 1u) * YT + t, ys.ntiles - 1u);
        uint32_t tm[NW];
#pragma unroll
        for (int w = 0; w < NW; w++) tm[w] = ys.tmax[(size_t)w * ys.ntiles + tt];
        R::cmax(ymax, tm);
    }
    uint32_t cnt = 0;
#pragma unroll 4
    for (uint32_t g = 0; g < ngroups; g++) {
        uint32_t gc[NW];
#pragma unroll
        for (int w = 0; w < NW; w++) gc[w] = gmin[(size_t)w * ngroups + g];
        cnt += R::le(gc, ymax) ? 1u : 0u;
    }
    if (valid) lpt[kMbrLptHead + yt] = cnt;
    unsigned long long t = valid ? cnt : 0u;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) t += __shfl_xor(t, o, 64);
    if ((threadIdx.x & 63) == 0 && t) atomicAdd(reinterpret_cast<unsigned long long *>(lpt + 36), t);
}

// one workgroup: the split of every y tile, bucket counts of the items' costs (log2), offsets
// heaviest bucket first, then every item to its slot; lpt[33] = the number of items.  qcap: the
// items the queue holds (the host's mbr_items_max).  The split rule keeps the items within it;
// should a rule change ever break that bound, nothing is written past the queue: the kernel
// raises kFlagMbrQueue in *err, leaves the queue empty (the pair pass then does nothing) and the
// host returns SKY_E_HIP for the query
__global__ __launch_bounds__(1024) void k_mbr_order(uint32_t nyt, uint32_t qcap, uint32_t *__restrict__ lpt,
                                                    uint32_t *__restrict__ err) {
    __shared__ uint32_t s_cnt[32], s_off[32], s_over;
    if (threadIdx.x < 32) s_cnt[threadIdx.x] = 0;
    __syncthreads();
    // the cost per item: total / max(nyt, 4096), rounded UP, so that the items
    // sum_t ceil(c_t / c0) <= nyt + total / c0 <= nyt + max(nyt, 4096) = mbr_items_max(nyt) fit the
    // queue (rounding down overflowed it: c0 = 1 split every tile into c_t items)
    const unsigned long long total = *reinterpret_cast<const unsigned long long *>(lpt + 36);
    const unsigned long long M = (unsigned long long)max(nyt, 4096u);
    const unsigned long long c0 = max(1ull, (total + M - 1) / M);
    const uint32_t *cost = lpt + kMbrLptHead;
    auto split = [&](uint32_t c) -> uint32_t {
        return c == 0 ? 0u : (uint32_t)min((unsigned long long)min(c, (uint32_t)kMbrSplitMax), (c + c0 - 1) / c0);
    };
    for (uint32_t yt = threadIdx.x; yt < nyt; yt += 1024) {
        const uint32_t c = cost[yt], s = split(c);
        if (s) atomicAdd(&s_cnt[31 - __clz((c + s - 1) / s)], s);   // bucket = floor(log2(item cost))
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long o = 0;
        for (int b = 31; b >= 0; b--) {
            s_off[b] = (uint32_t)min(o, 0xffffffffull);
            o += s_cnt[b];
        }
        s_over = o > qcap ? 1u : 0u;
        lpt[33] = o > qcap ? 0u : (uint32_t)o;
        if (o > qcap) atomicOr(err, kFlagMbrQueue);
    }
    __syncthreads();
    if (s_over) return;                            // nothing past the queue; no items at all
    uint32_t *items = lpt + kMbrLptHead + nyt;
    for (uint32_t yt = threadIdx.x; yt < nyt; yt += 1024) {
        const uint32_t c = cost[yt], s = split(c);
        if (!s) continue;                          // no reachable group: nothing dominates its rows
        const uint32_t o = atomicAdd(&s_off[31 - __clz((c + s - 1) / s)], s);
        for (uint32_t i = 0; i < s && o + i < qcap; i++) {   // o + s <= total <= qcap here
            items[2 * (o + i)] = yt;
            items[2 * (o + i) + 1] = i | (s << 16);
        }
    }
}

// the next work item of this wave (wave-uniform); false when the queue is empty
__device__ __forceinline__ bool mbr_next_item(uint32_t *__restrict__ lpt, uint32_t nyt, uint32_t &item, uint32_t &yt,
                                              uint32_t &part, uint32_t &parts) {
    uint32_t t = 0;
    if ((threadIdx.x & 63) == 0) t = atomicAdd(&lpt[32], 1u);
    item = __builtin_amdgcn_readfirstlane(__shfl((int)t, 0, 64));
    if (item >= __builtin_amdgcn_readfirstlane(lpt[33])) return false;
    const uint32_t *it = lpt + kMbrLptHead + nyt + 2 * (size_t)item;
    yt = __builtin_amdgcn_readfirstlane(it[0]);
    const uint32_t ps = __builtin_amdgcn_readfirstlane(it[1]);
    part = ps & 0xffffu;
    parts = ps >> 16;
    return true;
}

// this item's share of a chunk of reachable groups m (wave-uniform): the groups whose ordinal
// among the y tile's reachable groups is = part (mod parts); ord carries the ordinal mod parts.
// Reachability here is the box test alone (the static set k_mbr_cost counted): every reachable
// group belongs to exactly one item whatever the items' live lanes do.
__device__ __forceinline__ uint64_t mbr_share(uint64_t m, uint32_t &ord, uint32_t part, uint32_t parts) {
    if (parts == 1) return ~0ull;
    uint64_t keep = 0;
    while (m) {
        const int b = __builtin_ctzll(m);
        m &= m - 1;
        if (ord == part) keep |= 1ull << b;
        ord = ord + 1 == parts ? 0u : ord + 1;
    }
    return keep;
}

// ---- the pair pass -------------------------------------------------------------------
// FULL: the complete test (x <= y and not y <= x) — given partition keys may repeat a
// vector across partitions, and f32/f64 rows may hold -0.0 / +0.0 twins; otherwise the rows
// are distinct vectors and "x <= y, x at another position" is dominance.
// GM: the global level is wanted (bit 1); else only the same-partition bit matters.
// The y tiles (ys) may be another set than the x tiles (the multi-GPU merge: own vectors against
// the union, FULL only); for one set they are the same arrays.
//
// A work item is a y UNIT: YT consecutive y tiles (64 YT y's, Hilbert neighbours), one wave,
// lane = y of each tile.  The units' x work overlaps strongly (tools: per y tile the x tiles
// that pass the whole-corner test drop from 283 to 177 at YT = 2 on std-anti 8D 2M), so the
// per-x-tile costs -- group and tile scans, row and corner loads, the LDS staging, the fate
// read-back -- are paid once for YT tiles.  For every x tile whose min corner is <= the unit's
// max corner (found 64 tiles at a time per reachable group):
//  * the whole tile's min corner against every live y (NW readlanes, one ballot per y tile);
//  * sub-box stage, lane = (pre y, sub-box): the y's that passed are listed in LDS, each pass
//    tests 64 / S of them against all S sub-box corners at once (the corner of box lane % S came
//    in with the tile's rows), and the passing (y, box) entries are appended to an LDS list;
//  * row stage, lane = (entry, row): the tile's rows (loaded one tile ahead, two register sets
//    used alternately) are staged in LDS and S entries are compared per wave instruction (lane r
//    of entry g: row r of its sub-box against its y);
//  * a hit is one LDS atomic OR into the y's fate word; the fates are read back once per tile to
//    retire the y's a rep of their own partition dominates.
// With 8-row sub-boxes (packed u16 rows) a y meets 2.6x fewer rows than with 16-row ones.
// packed-u16 rows: the register budget capped for 6 waves per SIMD (79 VGPRs at YT = 2, no spill;
// the 5 waves the 82-VGPR default allows: 19.1 vs 18.8 ms at std-anti 8D 10M)
// waves per SIMD the pair pass's register budget is sized for: 7 for one-tile work items (2M: pass
// 3.54 -> 3.40 ms), 6 for the two-tile items of >= 65536 y tiles (10M: 7 is 1.5 % slower;
// profiles/r05_dominance_ab.txt)
#ifndef SKY_MBR_WPE
#define SKY_MBR_WPE 6
#endif
#ifndef SKY_MBR_WPE1
#define SKY_MBR_WPE1 7
#endif
template <class R, bool FULL, bool GM, int YT>
__global__ __launch_bounds__(kMbrPairThreads) __attribute__((amdgpu_waves_per_eu(R::NW <= 4 ? (YT == 1 ? SKY_MBR_WPE1 : SKY_MBR_WPE) : 1))) void k_mbr_pairs(const uint32_t *__restrict__ trows,
                                                         const uint32_t *__restrict__ tpart,
                                                         const uint32_t *__restrict__ tmin,
                                                         const uint32_t *__restrict__ tprange,
                                                         const uint32_t *__restrict__ tsub,
                                                         const uint32_t *__restrict__ gmin,
                                                         const uint32_t *__restrict__ gprange, uint32_t mr,
                                                         uint32_t ntiles, MbrYSet ys, int dbg,
                                                         uint32_t *__restrict__ domf,
                                                         unsigned long long *__restrict__ pairs,
                                                         uint32_t *__restrict__ lpt,
                                                         unsigned long long *__restrict__ trace) {
    constexpr int NW = R::NW;
    constexpr int S = mbr_subs<R>(), RS = kMbrT / S;
    constexpr int NY = 64 * YT;                    // y's per work item
    static_assert(NY <= 256 && S <= 16, "entries are (y << 4 | box) in 16 bits, pre y's in 8");
    uint64_t npairs = 0, ntested = 0;
    uint32_t ngrp = 0, nbox = 0, npre = 0;
    const uint32_t ngroups = (ntiles + kMbrG - 1) / kMbrG;
    const uint32_t nyu = (ys.ntiles + YT - 1) / YT;
    const uint32_t lane = threadIdx.x & 63;
    // row stage: RL lanes per entry, each comparing two rows of the entry's sub-box (er and
    // er + RL) with the entry's y: 64 / RL entries per wave instruction
    constexpr int RL = RS / 2;
    const uint32_t eg = lane / RL, er = lane % RL;   // this lane's entry slot and first row within it
    __shared__ uint4 s_y[NY * NW / 4];            // this item's y rows (compare operands)
    __shared__ uint32_t s_py[NY], s_hit[NY];       // y partitions; y fate words (bit 1 any, bit 0 same)
    __shared__ uint4 s_x[64 * NW / 4];            // the x tile under test
    __shared__ uint32_t s_px[64];
    __shared__ uint16_t s_e[NY * S];              // (y << 4 | sub-box) entries
    __shared__ uint8_t s_pl[NY];                  // the y's that passed the tile's whole-corner test
    uint32_t *sy = reinterpret_cast<uint32_t *>(s_y), *sx = reinterpret_cast<uint32_t *>(s_x);
#ifdef SKY_MEASURE
    // SKY_MBR_DBG & 16 (measurement builds): shader-clock time per region of the pass, charged to
    // the region running when the next one starts: 0 item setup / super-groups, 1 group and tile
    // scans, 2 whole-corner pretests, 3 row / corner loads issued, 4 sub-box stage, 5 row stage
    uint64_t t_acc[6] = {0, 0, 0, 0, 0, 0}, t_last = 0;
    int t_cur = 0;
    const bool timing = (dbg & 16) != 0;
    if (timing) t_last = __builtin_amdgcn_s_memtime();
    auto tick = [&](int k) {
        if (!timing) return;
        const uint64_t t = __builtin_amdgcn_s_memtime();
#pragma unroll
        for (int i = 0; i < 6; i++)
            if (i == t_cur) t_acc[i] += t - t_last;
        t_last = t;
        t_cur = k;
    };
#else
    auto tick = [](int) {};
#endif
    uint32_t witem, yu, part, parts;
    while (mbr_next_item(lpt, nyu, witem, yu, part, parts)) {
    const unsigned long long t_start = trace ? __builtin_amdgcn_s_memrealtime() : 0ull;
    tick(0);
    const uint64_t np0 = npairs, nt0 = ntested;
    uint32_t gord = 0;
    const uint32_t yt0 = yu * YT;
    uint32_t y[YT][NW], ymax[NW];
    uint64_t live[YT];
    uint32_t f[YT];
    uint32_t ypl = 0xffffffffu, yph = 0u;
    R::ident_max(ymax);
#pragma unroll
    for (int t = 0; t < YT; t++) {
        const uint32_t jt = (yt0 + t) * kMbrT + lane;
        const bool valid = jt < ys.mr;
        const uint4 *src = reinterpret_cast<const uint4 *>(ys.trows + (size_t)min(jt, ys.mr - 1u) * NW);
#pragma unroll
        for (int q = 0; q < NW / 4; q++) {
            const uint4 v = src[q];
            y[t][4 * q] = v.x;
            y[t][4 * q + 1] = v.y;
            y[t][4 * q + 2] = v.z;
            y[t][4 * q + 3] = v.w;
        }
        if (yt0 + t < ys.ntiles) {                 // wave-uniform
            uint32_t tm[NW];
#pragma unroll
            for (int w = 0; w < NW; w++) tm[w] = ys.tmax[(size_t)w * ys.ntiles + yt0 + t];
            R::cmax(ymax, tm);
            const uint32_t yr = ys.tprange[yt0 + t];
            ypl = min(ypl, yr & 0xffffu);
            yph = max(yph, yr >> 16);
        }
#pragma unroll
        for (int w = 0; w < NW; w++) sy[(t * 64 + lane) * NW + w] = y[t][w];
        s_py[t * 64 + lane] = valid ? ys.tpart[min(jt, ys.mr - 1u)] : 0xffffffffu;
        s_hit[t * 64 + lane] = 0u;
        live[t] = __ballot(valid);
        f[t] = 0u;
    }
    // the unit's static max corner: what decides which split item owns which group (mbr_share),
    // whatever the items' live lanes do; ymax itself shrinks with the live y's (refresh_ymax)
    uint32_t ymax0[NW];
#pragma unroll
    for (int w = 0; w < NW; w++) ymax0[w] = ymax[w];
    __builtin_amdgcn_wave_barrier();
    auto any_live = [&]() -> bool {
        uint64_t a = 0;
#pragma unroll
        for (int t = 0; t < YT; t++) a |= live[t];
        return a != 0ull;
    };
    // some live y still lacks a dominator of any partition (GM: the scans cannot restrict
    // themselves to the unit's partitions yet)
    auto need_any = [&]() -> bool {
        uint64_t a = 0;
#pragma unroll
        for (int t = 0; t < YT; t++) a |= live[t] & __ballot(!(f[t] & 2u));
        return a != 0ull;
    };

    // the rows + partition of x tile xt, one row per lane (clamped: past mr masked by nx), and the
    // min corner of its sub-box (lane % S): the sub-box stage's operand
    auto load_x = [&](uint32_t xt, uint32_t (&xv)[NW], uint32_t (&cv)[NW], uint32_t &px) {
        tick(3);
        const uint32_t xi = min(xt * kMbrT + lane, mr - 1u);
        const uint4 *src = reinterpret_cast<const uint4 *>(trows + (size_t)xi * NW);
        const uint4 *csrc = reinterpret_cast<const uint4 *>(tsub + ((size_t)xt * S + (lane % S)) * NW);
#pragma unroll
        for (int q = 0; q < NW / 4; q++) {
            const uint4 v = src[q];
            xv[4 * q] = v.x;
            xv[4 * q + 1] = v.y;
            xv[4 * q + 2] = v.z;
            xv[4 * q + 3] = v.w;
            const uint4 c = csrc[q];
            cv[4 * q] = c.x;
            cv[4 * q + 1] = c.y;
            cv[4 * q + 2] = c.z;
            cv[4 * q + 3] = c.w;
        }
        px = tpart[xi];
    };
    // the live y's max corner: as y's are retired (a rep of their own partition dominates them) the
    // box the x scan tests against shrinks; recomputed (wave max) when live changed since
    uint64_t live_ymax[YT];
#pragma unroll
    for (int t = 0; t < YT; t++) live_ymax[t] = live[t];
    auto refresh_ymax = [&]() {
        bool same = true;
#pragma unroll
        for (int t = 0; t < YT; t++) same &= live[t] == live_ymax[t];
        if (same) return;
        uint32_t m[NW];
        R::ident_max(m);
#pragma unroll
        for (int t = 0; t < YT; t++) {
            live_ymax[t] = live[t];
            if ((live[t] >> lane) & 1ull) R::cmax(m, y[t]);
        }
#pragma unroll
        for (int o = 1; o <= 32; o <<= 1) {
            uint32_t b[NW];
#pragma unroll
            for (int w = 0; w < NW; w++) b[w] = (uint32_t)__shfl_xor((int)m[w], o, 64);
            R::cmax(m, b);
        }
#pragma unroll
        for (int w = 0; w < NW; w++) ymax[w] = (uint32_t)__builtin_amdgcn_readfirstlane((int)m[w]);
    };
    uint32_t tg[NW];                                // min corners of the group's tiles (lane = tile)
    // the next tile of the group (bits tm) whose whole min corner is <= some live y (the corner
    // came in with the tile scan: NW readlanes); pm[t] = those y of y tile t.  Tiles that can
    // dominate no live y are dropped here, before their rows are loaded and their corners read
    auto next_tile = [&](uint64_t &tm, uint32_t g, uint32_t &xt, uint64_t (&pm)[YT]) -> bool {
        tick(2);
        while (tm) {
            const int ti = (int)__builtin_ctzll(tm);
            tm &= tm - 1;
            uint32_t tc[NW];
#pragma unroll
            for (int w = 0; w < NW; w++) tc[w] = (uint32_t)__builtin_amdgcn_readlane((int)tg[w], ti);
            uint64_t a = 0;
#pragma unroll
            for (int t = 0; t < YT; t++) {
                pm[t] = __ballot(R::le(tc, y[t])) & live[t];
                a |= pm[t];
            }
            if (a) {
                xt = g + (uint32_t)ti;
                return true;
            }
        }
        return false;
    };
    // One x tile against the y's that passed its whole-tile test (pre, P of them): the sub-box
    // stage, the row stage and the fate read-back described above the kernel
    auto test_tile = [&](uint32_t xt, const uint32_t (&xv)[NW], const uint32_t (&cv)[NW], uint32_t px,
                         const uint64_t (&pm)[YT]) {
        tick(4);
        uint32_t P = 0;
#pragma unroll
        for (int t = 0; t < YT; t++) {             // live may have shrunk since the tile was picked
            const uint64_t pre = pm[t] & live[t];
            if ((pre >> lane) & 1ull) s_pl[P + lanes_below(pre)] = (uint8_t)(t * 64 + lane);
            P += (uint32_t)__popcll(pre);
        }
        if (!P) return;
        npre++;
        const uint32_t nx = mr - xt * kMbrT < (uint32_t)kMbrT ? mr - xt * kMbrT : (uint32_t)kMbrT;
        __builtin_amdgcn_wave_barrier();
        const uint32_t bl = lane % S;
        const bool bvalid = bl * RS < nx;          // a box past the tile's last row holds no row
        // each lane tests two pre y's (j and j + 64 / S) against its box: 2 * 64 / S y's per pass
        constexpr uint32_t YP = 64 / S;
        uint32_t E = 0;
        for (uint32_t j0 = 0; j0 < P; j0 += 2 * YP) {
            const uint32_t ja = j0 + lane / S, jb = ja + YP;
            const uint32_t yia = s_pl[min(ja, P - 1u)], yib = s_pl[min(jb, P - 1u)];
            uint32_t ya[NW], yb[NW];
#pragma unroll
            for (int q = 0; q < NW / 4; q++) {
                const uint4 a = s_y[yia * (NW / 4) + q], b = s_y[yib * (NW / 4) + q];
                ya[4 * q] = a.x; ya[4 * q + 1] = a.y; ya[4 * q + 2] = a.z; ya[4 * q + 3] = a.w;
                yb[4 * q] = b.x; yb[4 * q + 1] = b.y; yb[4 * q + 2] = b.z; yb[4 * q + 3] = b.w;
            }
            const bool pa = (ja < P) & bvalid & R::le(cv, ya), pb = (jb < P) & bvalid & R::le(cv, yb);
            const uint64_t ba = wballot(pa), bb = wballot(pb);
            const uint32_t na = (uint32_t)__popcll(ba);
            if (pa) s_e[E + lanes_below(ba)] = (uint16_t)((yia << 4) | bl);
            if (pb) s_e[E + na + lanes_below(bb)] = (uint16_t)((yib << 4) | bl);
            E += na + (uint32_t)__popcll(bb);
        }
        npairs += (uint64_t)RS * E;
        if ((dbg & 1) || !E) return;
        ntested++;
        tick(5);
#pragma unroll
        for (int w = 0; w < NW; w++) sx[lane * NW + w] = xv[w];
        s_px[lane] = px;
        __builtin_amdgcn_wave_barrier();
        bool any = false;
        for (uint32_t e0 = 0; e0 < E; e0 += 64 / RL) {
            const bool ev = e0 + eg < E;
            const uint32_t ent = s_e[min(e0 + eg, E - 1u)];
            const uint32_t yb = ent >> 4, xr0 = (ent & 15u) * RS + er, xr1 = xr0 + RL;
            uint32_t xa[NW], xb[NW], yw[NW];
#pragma unroll
            for (int q = 0; q < NW / 4; q++) {
                const uint4 a = s_x[xr0 * (NW / 4) + q], c = s_x[xr1 * (NW / 4) + q], b = s_y[yb * (NW / 4) + q];
                xa[4 * q] = a.x; xa[4 * q + 1] = a.y; xa[4 * q + 2] = a.z; xa[4 * q + 3] = a.w;
                xb[4 * q] = c.x; xb[4 * q + 1] = c.y; xb[4 * q + 2] = c.z; xb[4 * q + 3] = c.w;
                yw[4 * q] = b.x; yw[4 * q + 1] = b.y; yw[4 * q + 2] = b.z; yw[4 * q + 3] = b.w;
            }
            // bitwise, not short-circuit: no exec-masked branches per test
            bool d0 = ev & (xr0 < nx) & R::le(xa, yw), d1 = ev & (xr1 < nx) & R::le(xb, yw);
            if constexpr (FULL) {
                d0 = d0 & !R::le(yw, xa);
                d1 = d1 & !R::le(yw, xb);
            } else {
                const bool own = xt == yt0 + (yb >> 6);
                d0 = d0 & !(own && xr0 == (yb & 63u));
                d1 = d1 & !(own && xr1 == (yb & 63u));
            }
            if (d0 | d1) {
                const uint32_t py = s_py[yb];
                const uint32_t h0 = d0 ? (s_px[xr0] == py ? 3u : 2u) : 0u, h1 = d1 ? (s_px[xr1] == py ? 3u : 2u) : 0u;
                atomicOr(&s_hit[yb], h0 | h1);
                any = true;
            }
        }
        if (__ballot(any)) {
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int t = 0; t < YT; t++) {
                f[t] |= s_hit[t * 64 + lane];
                live[t] &= __ballot(!(f[t] & 1u));
            }
        }
        __builtin_amdgcn_wave_barrier();
    };

    // super-groups of 64 groups first (their min corners follow the groups' in gmin): a super-group
    // whose corner is not <= the unit's max corner holds no reachable group, and is skipped whole
    const uint32_t nsup = (ngroups + kMbrG - 1) / kMbrG;
    const uint32_t *sgmin = gmin + (size_t)NW * ngroups;
    for (uint32_t u0 = 0; u0 < nsup && any_live(); u0 += 64) {
    uint64_t sm;
    {
        const uint32_t q = min(u0 + lane, nsup - 1u);
        uint32_t sc[NW];
#pragma unroll
        for (int w = 0; w < NW; w++) sc[w] = sgmin[(size_t)w * nsup + q];
        sm = __ballot(u0 + lane < nsup && R::le(sc, parts == 1 ? ymax : ymax0));   // shares count static groups
    }
    while (sm && any_live()) {
        const uint32_t s0 = (u0 + (uint32_t)__builtin_ctzll(sm)) * 64;
        sm &= sm - 1;
        refresh_ymax();
        uint64_t gm;
        {
            const uint32_t q = min(s0 + lane, ngroups - 1u);
            uint32_t gc[NW];
#pragma unroll
            for (int w = 0; w < NW; w++) gc[w] = gmin[(size_t)w * ngroups + q];
            const uint32_t gr = gprange[q];
            const bool na = GM && need_any();
            const bool reach = s0 + lane < ngroups && R::le(gc, ymax0);
            bool cand = reach && R::le(gc, ymax);
            if (cand && !na) cand = (gr & 0xffffu) <= yph && (gr >> 16) >= ypl;
            gm = __ballot(cand) & mbr_share(__ballot(reach), gord, part, parts);
        }
        ngrp += (uint32_t)__popcll(gm);
        while (gm && any_live()) {
            const uint32_t g = (s0 + (uint32_t)__builtin_ctzll(gm)) * kMbrG;
            gm &= gm - 1;
            tick(1);
            refresh_ymax();
            uint64_t tm;
            {
                const uint32_t t = min(g + lane, ntiles - 1u);
#pragma unroll
                for (int w = 0; w < NW; w++) tg[w] = tmin[(size_t)w * ntiles + t];
                const uint32_t tr = tprange[t];
                const bool na = GM && need_any();
                bool cand = g + lane < ntiles && R::le(tg, ymax);
                if (cand && !na) cand = (tr & 0xffffu) <= yph && (tr >> 16) >= ypl;
                tm = __ballot(cand);
            }
            if (dbg & 2) tm = 0;
            nbox += (uint32_t)__popcll(tm);
            if (!tm) continue;
            // the group's tiles that pass the whole-tile test, the next one's rows in flight while
            // one is tested (two register sets used alternately: no copy at the back-edge that would
            // wait for them; past the last tile the current one is re-loaded, a cache hit)
            uint32_t xa, xb;
            uint64_t ma[YT], mb[YT];
            if (!next_tile(tm, g, xa, ma)) continue;
            uint32_t va[NW], vb[NW], ca[NW], cb[NW], pa, pb;
            load_x(xa, va, ca, pa);
            for (;;) {
                const bool hb = next_tile(tm, g, xb, mb);
                if (!hb) xb = xa;
                load_x(xb, vb, cb, pb);
                test_tile(xa, va, ca, pa, ma);
                if (!hb || !any_live()) break;
                const bool ha = next_tile(tm, g, xa, ma);
                if (!ha) xa = xb;
                load_x(xa, va, ca, pa);
                test_tile(xb, vb, cb, pb, mb);
                if (!ha || !any_live()) break;
            }
        }
    }
    }                                               // the next reachable super-group
    tick(0);
#pragma unroll
    for (int t = 0; t < YT; t++) {
        const uint32_t jt = (yt0 + t) * kMbrT + lane;
        if (jt < ys.mr && f[t]) atomicOr(&domf[jt], f[t]);   // domf zeroed by the caller
    }
    if (trace && lane == 0) {
        trace[4 * (size_t)witem] = t_start;
        trace[4 * (size_t)witem + 1] = __builtin_amdgcn_s_memrealtime();
        trace[4 * (size_t)witem + 2] = ntested - nt0;
        trace[4 * (size_t)witem + 3] = npairs - np0;
    }
    __builtin_amdgcn_wave_barrier();               // the next item rewrites s_y / s_py / s_hit
    }                                               // the next work item
    if ((threadIdx.x & 63) == 0 && pairs) {
        atomicAdd(pairs, (unsigned long long)npairs);
        atomicAdd(pairs + 1, (unsigned long long)ntested);
        if (dbg & 4) {
            atomicAdd(pairs + 2, (unsigned long long)ngrp);
            atomicAdd(pairs + 3, (unsigned long long)nbox);
            atomicAdd(pairs + 4, (unsigned long long)npre);
        }
#ifdef SKY_MEASURE
        if (timing)
            for (int i = 0; i < 6; i++) atomicAdd(pairs + 8 + i, (unsigned long long)t_acc[i]);
#endif
    }
}

__global__ __launch_bounds__(kThreads) void k_mbr_finish(const uint32_t *__restrict__ perm,
                                                         const uint32_t *__restrict__ domf, uint32_t mr, int gmerge,
                                                         uint8_t *__restrict__ alive_l, uint8_t *__restrict__ alive_g) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= mr) return;
    const uint32_t f = domf[j], rep = perm[j];
    const bool in_l = !(f & 1u);
    alive_l[rep] = in_l ? 1 : 0;
    alive_g[rep] = (gmerge ? !(f & 2u) : in_l) ? 1 : 0;
}

// ---- host side -----------------------------------------------------------------------
int mbr_row_words(int D, int fmt) {
    if (fmt == 0) return dom16_words(D);
    if (fmt == 1) return padded_dims<float>(D);
    return 2 * padded_dims<double>(D);
}

// SKY_MBR_ORDER=morton: the Morton order of round 2 (A/B knob, read per build)
static bool mbr_hilbert() {
    const char *e = SKY_MEASURE_ENV("SKY_MBR_ORDER");
    return !(e && e[0] == 'm');
}

static int mbr_bits(int D) {
    int b = 32 / D;
    return b < 2 ? 2 : (b > 16 ? 16 : b);
}

size_t mbr_tiles(uint32_t mr) { return (mr + kMbrT - 1) / kMbrT; }
size_t mbr_groups(uint32_t mr) { return (mbr_tiles(mr) + kMbrG - 1) / kMbrG; }
// words per row-word of gmin (and entries of gprange): the groups, then their super-groups of 64
size_t mbr_group_slots(uint32_t mr) {
    const size_t g = mbr_groups(mr);
    return g + (g + kMbrG - 1) / kMbrG;
}

// Hilbert order + 64-row tiles (+ groups of 64 tiles) of one row set; returns the sorted order
template <class R, int D>
static const uint32_t *mbr_build(const uint32_t *rows, const uint64_t *rep_key, uint32_t mr, uint32_t *mm,
                                 uint64_t *code, uint64_t *code_alt, uint32_t *idx, uint32_t *idx_alt,
                                 uint32_t *radix_scratch, uint32_t *err, uint32_t *trows, uint32_t *tpart,
                                 uint32_t *tmin, uint32_t *tmax, uint32_t *tprange, uint32_t *tsub, uint32_t *gmin,
                                 uint32_t *gprange, hipStream_t st, hipError_t *lerr) {
    const uint32_t ntiles = (uint32_t)mbr_tiles(mr);
    const unsigned gb = (unsigned)((mr + kThreads - 1) / kThreads);
    const int bits = mbr_bits(D);
    k_mbr_minmax<R, D><<<gb < 512 ? gb : 512, kThreads, 0, st>>>(rows, mr, mm);
    k_mbr_code<R, D><<<gb, kThreads, 0, st>>>(rows, rep_key, mr, bits, mm, mbr_hilbert() ? 1 : 0, code, idx);
    const int tb = bits * D + 8;
    const uint64_t kor = tb >= 64 ? ~0ull : ((1ull << tb) - 1ull);
    const bool alt = radix_sort_pairs(code, idx, code_alt, idx_alt, mr, kor, 0ull, radix_scratch, err, st, lerr);
    const uint32_t *perm = alt ? idx_alt : idx;
    k_mbr_tiles<R><<<(ntiles + 3) / 4, kThreads, 0, st>>>(rows, rep_key, perm, mr, ntiles, trows, tpart, tmin, tmax,
                                                          tprange, tsub);
    if (gmin) {
        const uint32_t ngroups = (uint32_t)mbr_groups(mr);
        k_mbr_groups<R><<<(ngroups + 3) / 4, kThreads, 0, st>>>(tmin, tprange, ntiles, ngroups, gmin, gprange);
        const uint32_t nsup = (ngroups + kMbrG - 1) / kMbrG;   // the same reduction over the groups
        k_mbr_groups<R><<<(nsup + 3) / 4, kThreads, 0, st>>>(gmin, gprange, ngroups, nsup,
                                                             gmin + (size_t)R::NW * ngroups, gprange + ngroups);
    }
    return perm;
}

// one-wave workgroups of the pair pass: each takes work items until the queue is empty; more
// than stay resident at once (8 per SIMD on 1024 SIMDs), fewer when there are fewer items
static unsigned mbr_pair_waves(uint32_t ytiles) {
    return (unsigned)std::min<size_t>(mbr_items_max(ytiles), 8192);
}

// the work items of the pair pass, heaviest first (lpt: kMbrLptHead words zeroed by the caller)
// the queue's capacity in items: what mbr_lpt_words sized (SKY_MBR_QCAP, measurement builds only,
// shrinks it: the overflow test)
static uint32_t mbr_qcap(uint32_t ytiles) {
    const size_t cap = mbr_items_max(ytiles);
    const char *e = SKY_MEASURE_ENV("SKY_MBR_QCAP");
    return (uint32_t)(e ? std::min<size_t>(cap, strtoull(e, nullptr, 10)) : cap);
}

// y tiles per work item of the pair pass (k_mbr_pairs: the x-side work of Hilbert neighbours is
// shared).  Two pay once the y tiles are many: std-anti 8D 10M (156k tiles) 18.8 vs 19.9 ms; at
// 2M (31k tiles, 2.5 units per wave) one is faster (3.49 vs 3.61 ms)
// SKY_MBR_YT=1|2 (measurement builds): the item size forced at any size (the two-tile items' test)
static int mbr_yt(uint32_t ytiles) {
    const char *e = SKY_MEASURE_ENV("SKY_MBR_YT");
    if (e) return atoi(e) == 2 ? 2 : 1;
    return ytiles >= 65536 ? 2 : 1;
}

template <class R, int YT>
static void mbr_order(const uint32_t *gmin, uint32_t ngroups, const MbrYSet &ys, uint32_t *lpt, uint32_t *err,
                      hipStream_t st) {
    const uint32_t nyu = (ys.ntiles + YT - 1) / YT;
    k_mbr_cost<typename R::Pair, YT><<<(nyu + kThreads - 1) / kThreads, kThreads, 0, st>>>(gmin, ngroups, ys, lpt);
    // the queue sized for ys.ntiles units holds the fewer units' items too
    k_mbr_order<<<1, 1024, 0, st>>>(nyu, mbr_qcap(ys.ntiles), lpt, err);
}

template <class R, int D>
static void mbr_launch_t(const MbrArgs &a, hipStream_t st, hipError_t *lerr) {
    const uint32_t mr = a.mr;
    const uint32_t ntiles = (uint32_t)mbr_tiles(mr);
    const unsigned gb = (unsigned)((mr + kThreads - 1) / kThreads);
    const uint32_t *perm = mbr_build<R, D>((const uint32_t *)a.rows, a.rep_key, mr, a.mm, a.code, a.code_alt, a.idx,
                                           a.idx_alt, a.radix_scratch, a.err, a.trows, a.tpart, a.tmin, a.tmax,
                                           a.tprange, a.tsub, a.gmin, a.gprange, st, lerr);
    const unsigned gp = mbr_pair_waves(ntiles);
    const MbrYSet ys{a.trows, a.tpart, a.tmax, a.tprange, mr, ntiles};
#define SKY_MBR_PAIRS(F, G, Y)                                                                               \
    k_mbr_pairs<typename R::Pair, F, G, Y><<<gp, kMbrPairThreads, 0, st>>>(a.trows, a.tpart, a.tmin, a.tprange,   \
                                                                         a.tsub, a.gmin, a.gprange, mr, ntiles, ys, \
                                                                         a.dbg, a.domf, a.pairs, a.lpt, a.trace)
#define SKY_MBR_RUN(Y)                                                                                        \
    do {                                                                                                      \
        mbr_order<R, Y>(a.gmin, (uint32_t)mbr_groups(mr), ys, a.lpt, a.err, st);                              \
        if (a.full) {                                                                                         \
            if (a.gmerge) SKY_MBR_PAIRS(true, true, Y);                                                       \
            else SKY_MBR_PAIRS(true, false, Y);                                                               \
        } else {                                                                                              \
            if (a.gmerge) SKY_MBR_PAIRS(false, true, Y);                                                      \
            else SKY_MBR_PAIRS(false, false, Y);                                                              \
        }                                                                                                     \
    } while (0)
    if (mbr_yt(ntiles) == 2) SKY_MBR_RUN(2);
    else SKY_MBR_RUN(1);
#undef SKY_MBR_RUN
#undef SKY_MBR_PAIRS
    k_mbr_finish<<<gb, kThreads, 0, st>>>(perm, a.domf, mr, a.gmerge ? 1 : 0, a.alive_l, a.alive_g);
}

// own rows (y) against the union (x): flags[own row] = inL | inG << 1, and this rank's shares of
// |L_k| / survivors_k from the own rows' multiplicities
__global__ __launch_bounds__(kThreads) void k_mbr_union_finish(const uint32_t *__restrict__ perm,
                                                               const uint32_t *__restrict__ domf, uint32_t mr,
                                                               const uint64_t *__restrict__ ykey,
                                                               const int64_t *__restrict__ ymult, int K,
                                                               uint8_t *__restrict__ flags,
                                                               unsigned long long *__restrict__ lsz,
                                                               unsigned long long *__restrict__ surv) {
    // the stat shares summed per workgroup in LDS first: one global atomic per (workgroup, key)
    // (a global atomic per own row onto K words serialised: 11.8 ms for 1.2M rows, 16 keys)
    __shared__ unsigned long long s_l[kMaxK], s_g[kMaxK];
    const int Ke = K < kMaxK ? K : kMaxK;          // keys are the sort key's top byte
    for (int q = threadIdx.x; q < Ke; q += kThreads) { s_l[q] = 0; s_g[q] = 0; }
    __syncthreads();
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j < mr) {
        const uint32_t f = domf[j], r = perm[j];
        const bool in_l = !(f & 1u), in_g = !(f & 2u);
        flags[r] = (uint8_t)((in_l ? 1u : 0u) | (in_g ? 2u : 0u));
        const int k = (int)(ykey[r] >> 56);
        if (k < Ke) {
            const unsigned long long m = (unsigned long long)ymult[r];
            if (in_l) atomicAdd(&s_l[k], m);
            if (in_g) atomicAdd(&s_g[k], m);
        }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < Ke; q += kThreads) {
        if (s_l[q]) atomicAdd(&lsz[q], s_l[q]);
        if (s_g[q]) atomicAdd(&surv[q], s_g[q]);
    }
}

template <class R, int D>
static void mbr_union_t(const MbrUnionArgs &a, hipStream_t st, hipError_t *lerr) {
    const MbrArgs &x = a.x, &y = a.y;
    mbr_build<R, D>((const uint32_t *)x.rows, x.rep_key, x.mr, x.mm, x.code, x.code_alt, x.idx, x.idx_alt,
                    x.radix_scratch, x.err, x.trows, x.tpart, x.tmin, x.tmax, x.tprange, x.tsub, x.gmin, x.gprange, st,
                    lerr);
    const uint32_t *perm = mbr_build<R, D>((const uint32_t *)y.rows, y.rep_key, y.mr, y.mm, y.code, y.code_alt, y.idx,
                                           y.idx_alt, y.radix_scratch, y.err, y.trows, y.tpart, y.tmin, y.tmax,
                                           y.tprange, y.tsub, nullptr, nullptr, st, lerr);
    const uint32_t nyt = (uint32_t)mbr_tiles(y.mr);
    const unsigned gp = mbr_pair_waves(nyt);
    const MbrYSet ys{y.trows, y.tpart, y.tmax, y.tprange, y.mr, nyt};
    if (mbr_yt(nyt) == 2) {
        mbr_order<R, 2>(x.gmin, (uint32_t)mbr_groups(x.mr), ys, y.lpt, y.err, st);
        k_mbr_pairs<typename R::Pair, true, true, 2><<<gp, kMbrPairThreads, 0, st>>>(
            x.trows, x.tpart, x.tmin, x.tprange, x.tsub, x.gmin, x.gprange, x.mr, (uint32_t)mbr_tiles(x.mr), ys, x.dbg,
            y.domf, x.pairs, y.lpt, nullptr);
    } else {
    mbr_order<R, 1>(x.gmin, (uint32_t)mbr_groups(x.mr), ys, y.lpt, y.err, st);
    k_mbr_pairs<typename R::Pair, true, true, 1><<<gp, kMbrPairThreads, 0, st>>>(x.trows, x.tpart, x.tmin, x.tprange, x.tsub, x.gmin,
                                                        x.gprange, x.mr, (uint32_t)mbr_tiles(x.mr), ys, x.dbg,
                                                        y.domf, x.pairs, y.lpt, nullptr);
    }
    k_mbr_union_finish<<<(y.mr + kThreads - 1) / kThreads, kThreads, 0, st>>>(perm, y.domf, y.mr, y.rep_key, a.ymult,
                                                                             a.K, a.flags, a.lsz, a.surv);
}

hipError_t launch_mbr_union(const MbrUnionArgs &a, hipStream_t st) {
    if (!a.y.mr || !a.x.mr) return hipSuccess;
    hipError_t lerr = hipSuccess;
    if (a.x.fmt == 0) {
        if (a.x.D <= 8) {
            SKY_DISPATCH_D(a.x.D, (mbr_union_t<RowU16<DD, 4>, DD>(a, st, &lerr)));
        } else {
            SKY_DISPATCH_D(a.x.D, (mbr_union_t<RowU16<DD, 8>, DD>(a, st, &lerr)));
        }
    } else if (a.x.fmt == 1) {
        SKY_DISPATCH_D(a.x.D, (mbr_union_t<RowF32<DD>, DD>(a, st, &lerr)));
    } else {
        SKY_DISPATCH_D(a.x.D, (mbr_union_t<RowF64<DD>, DD>(a, st, &lerr)));
    }
    if (lerr != hipSuccess) return lerr;
    return hipGetLastError();
}

hipError_t launch_mbr(const MbrArgs &a, hipStream_t st) {
    if (!a.mr) return hipSuccess;
    hipError_t lerr = hipSuccess;
    if (a.fmt == 0) {
        if (a.D <= 8) {
            SKY_DISPATCH_D(a.D, (mbr_launch_t<RowU16<DD, 4>, DD>(a, st, &lerr)));
        } else {
            SKY_DISPATCH_D(a.D, (mbr_launch_t<RowU16<DD, 8>, DD>(a, st, &lerr)));
        }
    } else if (a.fmt == 1) {
        SKY_DISPATCH_D(a.D, (mbr_launch_t<RowF32<DD>, DD>(a, st, &lerr)));
    } else {
        SKY_DISPATCH_D(a.D, (mbr_launch_t<RowF64<DD>, DD>(a, st, &lerr)));
    }
    if (lerr != hipSuccess) return lerr;
    return hipGetLastError();
}

}  // namespace sky
