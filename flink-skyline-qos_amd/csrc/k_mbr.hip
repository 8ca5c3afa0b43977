// k_mbr.hip — both skyline levels of a LARGE representative set in one all-pairs pass
// with bounding-box pruning: no SFS rounds, no host round trips.
//
// Representatives (distinct candidate vectors, FlinkSkyline.java:417-444 / :548-566 as a
// set computation): y is in L_k iff no rep of its partition dominates it, and in G iff no
// rep at all dominates it (a dominator outside the union of the L_k is itself dominated
// by a member of it: transitivity), the same rule as the small-set brute path (k_sfs.hip).
//
//   k_mbr_minmax   per-dimension min / max of an order-preserving u32 image of the values
//   k_mbr_code     sort key = partition << (b*D) | Morton code of the values quantised to
//                  b bits per dimension (nearby vectors -> nearby positions)
//   radix sort     (k_radix.hip) of the keys, rep index as value
//   k_mbr_tiles    one wave per tile of 64 consecutive positions: rows gathered into tile
//                  order, the tile's bounding box (per-dimension min and max) and partition
//                  range
//   k_mbr_pairs    one wave per y tile (lane = y).  The x tiles are scanned 64 at a time
//                  (lane = x tile): an x tile can hold a dominator of some y of the y tile
//                  only if its min corner <= the y tile's max corner.  A candidate tile is
//                  then tested per lane (min corner <= y), and only if some live lane passes
//                  are its 64 rows compared (scalar row loads, y in VGPRs).  A lane is done
//                  once a rep of its own partition dominates it.
//   k_mbr_finish   alive_l / alive_g per rep
//
// The order only decides how much is pruned, never the result: any bounding box contains
// its rows, so a skipped tile holds no dominator.  On the labelled std-anti 8D stream about
// 2 % of the tile pairs survive the box test (tools/mbr_sim note in DESIGN.md §2.2).
#include "sky_internal.h"

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
__device__ __forceinline__ uint32_t ord_f32(float f) {       // order-preserving image (no NaN here)
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// ---- row formats: NW 32-bit words per row ------------------------------------------
// packed u16 pairs (k_dom16.hip layout): x <= y everywhere  <=>  OR_w sat(x_w - y_w) == 0
template <int D, int W>
struct RowU16 {
    static constexpr int NW = W;
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
#pragma unroll
    for (int d = 0; d < D; d++) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            lo[d] = min(lo[d], (uint32_t)__shfl_xor((int)lo[d], o, 64));
            hi[d] = max(hi[d], (uint32_t)__shfl_xor((int)hi[d], o, 64));
        }
    }
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int d = 0; d < D; d++) {
            atomicMin(&mm[d], lo[d]);
            atomicMax(&mm[D + d], hi[d]);
        }
    }
}

template <class R, int D>
__global__ __launch_bounds__(kThreads) void k_mbr_code(const uint32_t *__restrict__ rows,
                                                       const uint64_t *__restrict__ rep_key, uint32_t mr, int bits,
                                                       const uint32_t *__restrict__ mm, uint64_t *__restrict__ code,
                                                       uint32_t *__restrict__ idx) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= mr) return;
    const uint32_t *r = rows + (size_t)j * R::NW;
    uint32_t q[D];
#pragma unroll
    for (int d = 0; d < D; d++) {
        const uint64_t span = (uint64_t)mm[D + d] - mm[d] + 1u;
        q[d] = (uint32_t)((((uint64_t)(R::ord(r, d) - mm[d])) << bits) / span);
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

template <class R>
__global__ __launch_bounds__(kThreads) void k_mbr_tiles(const uint32_t *__restrict__ rows,
                                                        const uint64_t *__restrict__ rep_key,
                                                        const uint32_t *__restrict__ perm, uint32_t mr,
                                                        uint32_t ntiles, uint32_t *__restrict__ trows,
                                                        uint32_t *__restrict__ tpart, uint32_t *__restrict__ tmin,
                                                        uint32_t *__restrict__ tmax, uint32_t *__restrict__ tprange) {
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
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
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

// ---- the pair pass -------------------------------------------------------------------
// FULL: the complete test (x <= y and not y <= x) — given partition keys may repeat a
// vector across partitions, and f32/f64 rows may hold -0.0 / +0.0 twins; otherwise the rows
// are distinct vectors and "x <= y, x at another position" is dominance.
// GM: the global level is wanted (bit 1); else only the same-partition bit matters.
template <class R, bool FULL, bool GM>
__global__ __launch_bounds__(kThreads) void k_mbr_pairs(const uint32_t *__restrict__ trows,
                                                        const uint32_t *__restrict__ tpart,
                                                        const uint32_t *__restrict__ tmin,
                                                        const uint32_t *__restrict__ tmax,
                                                        const uint32_t *__restrict__ tprange, uint32_t mr,
                                                        uint32_t ntiles, int row_min, uint32_t *__restrict__ domf,
                                                        unsigned long long *__restrict__ pairs) {
    constexpr int NW = R::NW;
    const uint32_t yt = __builtin_amdgcn_readfirstlane(blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6));
    if (yt >= ntiles) return;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t j = yt * kMbrT + lane;
    const bool valid = j < mr;
    uint32_t y[NW], ymax[NW];
#pragma unroll
    for (int w = 0; w < NW; w++) y[w] = valid ? trows[(size_t)j * NW + w] : 0u;
#pragma unroll
    for (int w = 0; w < NW; w++) ymax[w] = tmax[(size_t)w * ntiles + yt];
    const uint32_t yr = tprange[yt];
    const uint32_t ypl = yr & 0xffffu, yph = yr >> 16;
    const uint32_t py = valid ? tpart[j] : 0xffffffffu;
    uint32_t f = 0;
    uint64_t live = __ballot(valid);
    uint64_t npairs = 0;
    // the next 64 tiles' min corners are loaded while the current ones are processed
    uint32_t tn[NW];
#pragma unroll
    for (int w = 0; w < NW; w++) tn[w] = lane < ntiles ? tmin[(size_t)w * ntiles + lane] : 0u;
    for (uint32_t base = 0; base < ntiles && live; base += 64) {
        const uint32_t t = base + lane;
        uint32_t tm[NW];
#pragma unroll
        for (int w = 0; w < NW; w++) tm[w] = tn[w];
        if (base + 64 < ntiles) {
            const uint32_t t2 = t + 64;
#pragma unroll
            for (int w = 0; w < NW; w++) tn[w] = t2 < ntiles ? tmin[(size_t)w * ntiles + t2] : 0u;
        }
        // some live lane not yet dominated by any rep (global level only): every tile
        // counts; otherwise only tiles holding rows of the y tile's partitions do
        const uint64_t need_any = GM ? (live & __ballot(!(f & 2u))) : 0ull;
        bool cand = t < ntiles && R::le(tm, ymax);
        if (cand && !need_any) {
            const uint32_t r = tprange[t];
            cand = (r & 0xffffu) <= yph && (r >> 16) >= ypl;
        }
        uint64_t m = __ballot(cand);
        while (m) {
            const uint32_t b = (uint32_t)__builtin_ctzll(m);
            m &= m - 1;
            const uint32_t xt = base + b;
            uint32_t xm[NW];
#pragma unroll
            for (int w = 0; w < NW; w++) xm[w] = (uint32_t)__builtin_amdgcn_readlane((int)tm[w], (int)b);
            uint64_t lm = live & __ballot(R::le(xm, y));
            if (!lm) continue;
            const uint32_t x0 = xt * kMbrT;
            const uint32_t nx = mr - x0 < (uint32_t)kMbrT ? mr - x0 : (uint32_t)kMbrT;
            npairs += (uint64_t)nx * (uint64_t)__popcll(lm);
            if (__popcll(lm) >= row_min) {
                // many y lanes in reach: every x row (scalar loads) against every lane
                const uint32_t *xr = trows + (size_t)x0 * NW;
                const uint32_t *xp = tpart + x0;
                if (xt == yt && !FULL) {
                    for (uint32_t q = 0; q < nx; q++) {
                        uint32_t x[NW];
#pragma unroll
                        for (int w = 0; w < NW; w++) x[w] = xr[(size_t)q * NW + w];
                        const bool dom = R::le(x, y) && q != lane;
                        f |= dom ? (xp[q] == py ? 3u : 2u) : 0u;
                    }
                } else {
#pragma unroll 4
                    for (uint32_t q = 0; q < nx; q++) {
                        uint32_t x[NW];
#pragma unroll
                        for (int w = 0; w < NW; w++) x[w] = xr[(size_t)q * NW + w];
                        bool dom = R::le(x, y);
                        if constexpr (FULL) dom = dom && !R::le(y, x);
                        f |= dom ? (xp[q] == py ? 3u : 2u) : 0u;
                    }
                }
            } else {
                // few y lanes in reach: lane = x row (one vector load of the tile), the
                // reachable y broadcast one at a time
                const uint32_t xi = x0 + lane;
                const bool xvalid = lane < nx;
                uint32_t xv[NW];
#pragma unroll
                for (int w = 0; w < NW; w++) xv[w] = xvalid ? trows[(size_t)xi * NW + w] : 0u;
                const uint32_t px = xvalid ? tpart[xi] : 0xfffffffeu;
                while (lm) {
                    const uint32_t yb = (uint32_t)__builtin_ctzll(lm);
                    lm &= lm - 1;
                    uint32_t yw[NW];
#pragma unroll
                    for (int w = 0; w < NW; w++) yw[w] = (uint32_t)__builtin_amdgcn_readlane((int)y[w], (int)yb);
                    const uint32_t pyu = (uint32_t)__builtin_amdgcn_readlane((int)py, (int)yb);
                    bool dom = xvalid && R::le(xv, yw);
                    if constexpr (FULL) dom = dom && !R::le(yw, xv);
                    else dom = dom && !(xt == yt && lane == yb);
                    const uint64_t hit = __ballot(dom);
                    if (hit) {
                        const uint32_t bits = __ballot(dom && px == pyu) ? 3u : 2u;
                        f |= lane == yb ? bits : 0u;
                    }
                }
            }
            live &= __ballot(!(f & 1u));
            if (!live) break;
        }
    }
    if (valid) domf[j] = f;
    if (lane == 0 && pairs) atomicAdd(pairs, (unsigned long long)npairs);
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

static int mbr_bits(int D) {
    int b = 32 / D;
    return b < 2 ? 2 : (b > 16 ? 16 : b);
}

size_t mbr_tiles(uint32_t mr) { return (mr + kMbrT - 1) / kMbrT; }

template <class R, int D>
static void mbr_launch_t(const MbrArgs &a, hipStream_t st, hipError_t *lerr) {
    const uint32_t mr = a.mr;
    const uint32_t ntiles = (uint32_t)mbr_tiles(mr);
    const unsigned gb = (unsigned)((mr + kThreads - 1) / kThreads);
    const int bits = mbr_bits(D);
    k_mbr_minmax<R, D><<<gb < 1024 ? gb : 1024, kThreads, 0, st>>>((const uint32_t *)a.rows, mr, a.mm);
    k_mbr_code<R, D><<<gb, kThreads, 0, st>>>((const uint32_t *)a.rows, a.rep_key, mr, bits, a.mm, a.code, a.idx);
    const int tb = bits * D + 8;
    const uint64_t kor = tb >= 64 ? ~0ull : ((1ull << tb) - 1ull);
    const bool alt = radix_sort_pairs(a.code, a.idx, a.code_alt, a.idx_alt, mr, kor, 0ull, a.radix_scratch, a.err, st,
                                      lerr);
    const uint32_t *perm = alt ? a.idx_alt : a.idx;
    const unsigned gt = (ntiles + 3) / 4;
    k_mbr_tiles<R><<<gt, kThreads, 0, st>>>((const uint32_t *)a.rows, a.rep_key, perm, mr, ntiles, a.trows, a.tpart,
                                            a.tmin, a.tmax, a.tprange);
    if (a.full) {
        if (a.gmerge)
            k_mbr_pairs<R, true, true><<<gt, kThreads, 0, st>>>(a.trows, a.tpart, a.tmin, a.tmax, a.tprange, mr, ntiles,
                                                                a.row_min, a.domf, a.pairs);
        else
            k_mbr_pairs<R, true, false><<<gt, kThreads, 0, st>>>(a.trows, a.tpart, a.tmin, a.tmax, a.tprange, mr,
                                                                 ntiles, a.row_min, a.domf, a.pairs);
    } else {
        if (a.gmerge)
            k_mbr_pairs<R, false, true><<<gt, kThreads, 0, st>>>(a.trows, a.tpart, a.tmin, a.tmax, a.tprange, mr,
                                                                 ntiles, a.row_min, a.domf, a.pairs);
        else
            k_mbr_pairs<R, false, false><<<gt, kThreads, 0, st>>>(a.trows, a.tpart, a.tmin, a.tmax, a.tprange, mr,
                                                                  ntiles, a.row_min, a.domf, a.pairs);
    }
    k_mbr_finish<<<gb, kThreads, 0, st>>>(perm, a.domf, mr, a.gmerge ? 1 : 0, a.alive_l, a.alive_g);
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
