// k_csv.hip — bulk CSV -> SoA decode of the tuple stream on the device.
//
// Replaces the reference's per-record ingest parse:
//   ServiceTuple.fromString   java/org.main/ServiceTuple.java:89-104  (s.split(","), Double.parseDouble)
//   .filter(Objects::nonNull) java/org.main/FlinkSkyline.java:103
//   Long.parseLong(point.id)  java/org.main/FlinkSkyline.java:276
// Records are '\n'-separated "id,v1,...,vD" (one Kafka value each in the reference).
//
// Passes (all HBM-streaming byte work, no MFMA):
//   k_csv_nl_count  per 4 KB chunk: number of '\n' (16 B per lane, one vector load)
//   scan            chunk offsets (k_scan.hip)
//   k_csv_group_pos  positions of every R-th '\n' -> line_g[] (group boundaries, R records per
//                   parse workgroup; the fallback finds a group's records itself)
//   k_csv_parse     one lane per record; the workgroup's 256 records are first staged
//                   into LDS with coalesced dword loads, then each lane walks its record:
//                   split semantics, Java trim, the Double.parseDouble grammar, the value
//                   (exact fast path: <= 19 significant digits, w <= 2^53, |e| <= 22, one
//                   correctly rounded IEEE op; otherwise an exact big-integer comparison
//                   against the halfway points, __noinline__ and rare), Long.parseLong.
//   k_csv_compact   only if some record was rejected: stable compaction of the rows.
#include "sky_internal.h"
#include "knobs.h"
#include <algorithm>
#include <cstdlib>

namespace sky {

constexpr int kCsvThreads = 256;
constexpr int kCsvChunk = kCsvThreads * 16;   // bytes per workgroup in the newline passes
constexpr int kCsvCountBlk = 64 * 16;         // bytes per newline count (one per wave of the count pass)
constexpr int kCommaShards = 256;             // comma-count accumulators (one global atomic per workgroup)

// ---------------------------------------------------------------- newline index
__device__ __forceinline__ uint32_t nl_in_word(uint32_t w) {
    // bytes equal to '\n' (0x0a): classic zero-byte test on w ^ 0x0a0a0a0a, exact per byte
    const uint32_t x = w ^ 0x0a0a0a0au;
    const uint32_t t = ((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x;
    return (~t) & 0x80808080u;   // bit 7 of byte b set iff byte b == '\n'
}

__device__ __forceinline__ uint32_t byte_eq_mask(uint32_t w, uint32_t pat) {
    const uint32_t x = w ^ pat;
    const uint32_t t = ((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x;
    return (~t) & 0x80808080u;
}

__device__ __forceinline__ void load16(const uint8_t *__restrict__ text, int64_t nbytes, int64_t base, bool aligned,
                                       uint32_t w[4]) {
    if (aligned && base + 16 <= nbytes) {
        const uint4 v = *reinterpret_cast<const uint4 *>(text + base);
        w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
        return;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint32_t x = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const int64_t i = base + k * 4 + b;
            const uint32_t c = i < nbytes ? text[i] : 0u;
            x |= c << (8 * b);
        }
        w[k] = x;
    }
}

__global__ __launch_bounds__(kCsvThreads) void k_csv_nl_count(const uint8_t *__restrict__ text, int64_t nbytes,
                                                              bool aligned, uint32_t *__restrict__ blk_cnt,
                                                              uint32_t *__restrict__ cnt1k,
                                                              unsigned long long *__restrict__ ncomma) {
    __shared__ uint32_t s_w[kCsvThreads / 64], s_c[kCsvThreads / 64];
    const int64_t base = (int64_t)blockIdx.x * kCsvChunk + threadIdx.x * 16;
    uint32_t w[4];
    load16(text, nbytes, base, aligned, w);
    uint32_t c = 0, cm = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        c += __popc(nl_in_word(w[k]));
        cm += __popc(byte_eq_mask(w[k], 0x2c2c2c2cu));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { c += __shfl_xor(c, o, 64); cm += __shfl_xor(cm, o, 64); }
    if ((threadIdx.x & 63) == 0) {
        s_w[threadIdx.x >> 6] = c;
        s_c[threadIdx.x >> 6] = cm;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        static_assert(kCsvChunk / kCsvCountBlk == 4, "one 16-byte store of the four 1 KB counts");
        reinterpret_cast<uint4 *>(cnt1k)[blockIdx.x] = make_uint4(s_w[0], s_w[1], s_w[2], s_w[3]);   // unscanned
        blk_cnt[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
        const uint32_t t = s_c[0] + s_c[1] + s_c[2] + s_c[3];
        if (t) atomicAdd(&ncomma[blockIdx.x & (kCommaShards - 1)], (unsigned long long)t);   // sharded: no hot spot
    }
}


// Only the group boundaries: line_g[g] = the position of newline (g + 1) R - 1 (0-based, in the
// text), the last newline of group g (the parse workgroups need only their group's first and last
// byte).  Found from the count pass's prefixes instead of a second pass over the text: one wave
// per 4 KB block knows from two prefixes which group ends fall in it (usually none or one), picks
// the 1 KB quarter holding each by the quarter counts, and reads that 1 KB (16 bytes per lane, a
// popcount scan): ~1 KB of text per group instead of all of it.
__global__ __launch_bounds__(kCsvThreads) void k_csv_group_pos(const uint8_t *__restrict__ text, int64_t nbytes,
                                                               bool aligned, const uint32_t *__restrict__ blk_off,
                                                               const uint32_t *__restrict__ cnt1k, int64_t nb,
                                                               uint32_t nl, uint32_t R, int64_t ngb,
                                                               int64_t *__restrict__ line_g) {
    const int64_t b = (int64_t)blockIdx.x * (kCsvThreads / 64) + (threadIdx.x >> 6);
    if (b >= nb) return;                                   // wave-uniform
    const int lane = threadIdx.x & 63;
    const uint32_t o0 = blk_off[b], o1 = b + 1 < nb ? blk_off[b + 1] : nl;
    // group ends q = (g + 1) R - 1 with o0 <= q < o1
    for (uint64_t q = ((uint64_t)o0 / R + 1) * R - 1; q < o1; q += R) {
        const int64_t g = (int64_t)((q + 1) / R) - 1;
        if (g >= ngb) break;
        uint32_t r = (uint32_t)q - o0;                     // rank of the newline inside block b
        int j = 0;
        for (; j < 3; j++) {
            const uint32_t c = cnt1k[b * (kCsvChunk / kCsvCountBlk) + j];
            if (r < c) break;
            r -= c;
        }
        const int64_t base = b * kCsvChunk + (int64_t)j * kCsvCountBlk + 16 * lane;
        uint32_t w[4], m[4], c = 0;
        load16(text, nbytes, base, aligned, w);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            m[k] = nl_in_word(w[k]);
            c += __popc(m[k]);
        }
        uint32_t inc = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(inc, o, 64);
            if (lane >= o) inc += t;
        }
        const uint32_t ex = inc - c;
        if (r >= ex && r < inc) {                          // exactly one lane
            uint32_t t = r - ex;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t ck = __popc(m[k]);
                if (t < ck) {
                    uint32_t mk = m[k];
                    for (uint32_t u = 0; u < t; u++) mk &= mk - 1;
                    line_g[g] = base + k * 4 + ((__ffs(mk) - 1) >> 3);
                    break;
                }
                t -= ck;
            }
        }
    }
}

// byte sources: text position i lives at p[i - off] (LDS staging: off = first staged byte)
struct LdsSrc {
    const uint8_t *p;
    int64_t off;
    __device__ __forceinline__ uint32_t operator[](int64_t i) const { return p[(int32_t)(i - off)]; }
};
struct GlbSrc {
    const uint8_t *p;
    int64_t off;
    __device__ __forceinline__ uint32_t operator[](int64_t i) const { return p[i]; }
};

__constant__ double kP10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// 10^k for 0 <= k <= 22, exactly (every partial product is a power of ten <= 1e22, so each
// multiplication is exact); selects only, no memory access
__device__ __forceinline__ double exact_pow10(int k) {
    double p = (k & 1) ? 1e1 : 1.0;
    p *= (k & 2) ? 1e2 : 1.0;
    p *= (k & 4) ? 1e4 : 1.0;
    p *= (k & 8) ? 1e8 : 1.0;
    p *= (k & 16) ? 1e16 : 1.0;
    return p;
}

// ---------------------------------------------------------------- number conversion
constexpr int kBigLimbs = 112;     // 3584 bits: the exact comparison needs <= ~2700 (see slow path)
constexpr int kMaxDigits = 800;    // significant digits kept (+ one sticky digit): halfway points of
                                   // doubles have <= 767 significant decimal digits

struct Big {
    uint32_t w[kBigLimbs];
    int n;
};

__device__ static void big_set(Big &a, uint64_t v) {
    a.w[0] = (uint32_t)v;
    a.w[1] = (uint32_t)(v >> 32);
    a.n = a.w[1] ? 2 : (a.w[0] ? 1 : 0);
}
__device__ static void big_mul_add(Big &a, uint32_t m, uint32_t add) {
    uint64_t carry = add;
    for (int i = 0; i < a.n; i++) {
        const uint64_t t = (uint64_t)a.w[i] * m + carry;
        a.w[i] = (uint32_t)t;
        carry = t >> 32;
    }
    if (carry && a.n < kBigLimbs) a.w[a.n++] = (uint32_t)carry;
}
__device__ static void big_pow5(Big &a, int k) {   // a *= 5^k
    while (k >= 13) { big_mul_add(a, 1220703125u, 0); k -= 13; }
    uint32_t m = 1;
    while (k-- > 0) m *= 5u;
    if (m != 1) big_mul_add(a, m, 0);
}
__device__ static void big_shl(Big &a, int s) {
    if (a.n == 0 || s <= 0) return;
    const int ls = s >> 5, bs = s & 31;
    int n = a.n + ls + 1;
    if (n > kBigLimbs) n = kBigLimbs;
    for (int i = n - 1; i >= 0; i--) {
        const int j = i - ls;
        uint32_t hi = (j >= 0 && j < a.n) ? a.w[j] : 0u;
        uint32_t lo = (j - 1 >= 0 && j - 1 < a.n) ? a.w[j - 1] : 0u;
        a.w[i] = bs ? (hi << bs) | (lo >> (32 - bs)) : hi;
    }
    while (n > 0 && a.w[n - 1] == 0) n--;
    a.n = n;
}
__device__ static int big_cmp(const Big &a, const Big &b) {
    if (a.n != b.n) return a.n < b.n ? -1 : 1;
    for (int i = a.n - 1; i >= 0; i--)
        if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
    return 0;
}

// sign(D * 10^E - h(b)), h(b) = the halfway point between finite b >= 0 and its successor:
// b = M * 2^Q (M < 2^53)  ->  h = (2M + 1) * 2^(Q - 1)
__device__ static int cmp_halfway(const Big &Dm, int E, uint64_t bits, Big &L, Big &R) {
    const int be = (int)(bits >> 52);
    uint64_t M = bits & ((1ull << 52) - 1);
    int Q;
    if (be == 0) Q = -1074;
    else { M |= 1ull << 52; Q = be - 1075; }
    const int t = Q - 1;
    L = Dm;
    big_set(R, 2 * M + 1);
    if (E >= 0) {
        big_pow5(L, E);
        const int s = E - t;
        if (s >= 0) big_shl(L, s); else big_shl(R, -s);
    } else {
        big_pow5(R, -E);
        const int s = t - E;
        if (s >= 0) big_shl(R, s); else big_shl(L, -s);
    }
    return big_cmp(L, R);
}

__device__ static double approx_pow10(double x, int e) {
    while (e > 22) { x *= 1e22; e -= 22; }
    while (e < -22) { x /= 1e22; e += 22; }
    return e >= 0 ? x * kP10[e] : x / kP10[-e];
}

// Exact decimal -> double (round half even) for the strings the fast path does not take.
// [q, qe) is the significand text (digits and at most one '.'), exp10 the parsed exponent,
// (w, ew) the first 19 significant digits and their scale (the candidate's seed).
__device__ __noinline__ double decimal_slow(const uint8_t *bp, int64_t boff, int64_t q, int64_t qe, int exp10,
                                            uint64_t w, int ew) {
    Big Dm, L, R;
    Dm.n = 0;
    int nsig = 0, E = 0;
    bool point = false, sticky = false;
    for (int64_t i = q; i < qe; i++) {
        const uint32_t c = bp[i - boff];
        if (c == '.') { point = true; continue; }
        const uint32_t d = c - '0';
        if (nsig == 0 && d == 0) { if (point) E--; continue; }
        if (nsig < kMaxDigits) {
            big_mul_add(Dm, 10u, d);
            if (point) E--;
        } else {
            if (!point) E++;
            if (d) sticky = true;
        }
        nsig++;
    }
    if (nsig > kMaxDigits) nsig = kMaxDigits;
    if (sticky) { big_mul_add(Dm, 10u, 1u); E--; nsig++; }
    E += exp10;
    const int dexp = nsig + E;                 // value in [10^(dexp-1), 10^dexp)
    if (dexp > 310) return __longlong_as_double(0x7ff0000000000000ll);
    if (dexp < -324) return 0.0;
    double x = approx_pow10((double)w, ew);
    uint64_t bits = (uint64_t)__double_as_longlong(x);
    if (bits >= 0x7ff0000000000000ull) bits = 0x7fefffffffffffffull;   // start from DBL_MAX
    for (int it = 0; it < 4096; it++) {
        const int c = cmp_halfway(Dm, E, bits, L, R);
        if (c > 0) {
            if (bits == 0x7fefffffffffffffull) return __longlong_as_double(0x7ff0000000000000ll);
            bits++;
            continue;
        }
        if (c == 0) return __longlong_as_double((long long)((bits & 1) ? bits + 1 : bits));
        if (bits == 0) return 0.0;
        const int c2 = cmp_halfway(Dm, E, bits - 1, L, R);
        if (c2 > 0) return __longlong_as_double((long long)bits);
        if (c2 == 0) return __longlong_as_double((long long)((bits & 1) ? bits - 1 : bits));
        bits--;
    }
    return __longlong_as_double((long long)bits);
}

// round m * 2^e2 (+ a positive amount below one unit of m when sticky) to the nearest double, ties even
__device__ static double make_double(uint64_t m, int e2, bool sticky) {
    if (m == 0) return 0.0;
    const int lz = __clzll((long long)m);
    m <<= lz;
    int lead = 63 + e2 - lz;   // value in [2^lead, 2^(lead+1))
    if (lead > 1023) return __longlong_as_double(0x7ff0000000000000ll);
    int r = 11;                // bits dropped below a 53-bit significand
    if (lead < -1022) r = 11 + (-1022 - lead);
    if (r > 64) return 0.0;    // below half the smallest subnormal
    uint64_t keep, half, rest;
    if (r == 64) { keep = 0; half = m >> 63; rest = (m << 1) != 0; }
    else {
        keep = m >> r;
        half = (m >> (r - 1)) & 1;
        rest = (m & ((1ull << (r - 1)) - 1)) != 0;
    }
    rest |= sticky;
    if (half && (rest || (keep & 1))) keep++;
    if (lead < -1022) {        // subnormal (keep counts units of 2^-1074; may round up into the normals)
        return __longlong_as_double((long long)keep);
    }
    if (keep >> 53) { keep >>= 1; lead++; }
    if (lead > 1023) return __longlong_as_double(0x7ff0000000000000ll);
    const uint64_t bits = ((uint64_t)(lead + 1023) << 52) | (keep & ((1ull << 52) - 1));
    return __longlong_as_double((long long)bits);
}

__device__ __forceinline__ bool is_digit(uint32_t c) { return c - '0' < 10u; }
__device__ __forceinline__ int hex_val(uint32_t c) {
    if (c - '0' < 10u) return (int)(c - '0');
    if (c - 'a' < 6u) return (int)(c - 'a' + 10);
    if (c - 'A' < 6u) return (int)(c - 'A' + 10);
    return -1;
}

// Double.parseDouble on b[s, e) (JDK 11 FloatingDecimal.readJavaFormatString grammar).
// Returns 0 on a NumberFormatException, 1 with `out` set, or (kFull = false only) 2 when the
// string is valid but needs the exact big-integer path: the caller queues it for k_csv_slow,
// which keeps the scratch-using code out of the streaming kernel.
template <bool kFull, typename Src>
__device__ __forceinline__ int java_parse_double(const Src b, int64_t s, int64_t e, double &out) {
    while (s < e && b[s] <= ' ') s++;
    while (e > s && b[e - 1] <= ' ') e--;
    if (s == e) return false;
    bool neg = false;
    int64_t p = s;
    uint32_t c = b[p];
    if (c == '+' || c == '-') { neg = c == '-'; p++; }
    if (p == e) return false;
    c = b[p];
    if (c == 'N') {
        if (e - p != 3 || b[p + 1] != 'a' || b[p + 2] != 'N') return false;
        out = __longlong_as_double(0x7ff8000000000000ll);
        return true;
    }
    if (c == 'I') {
        if (e - p != 8) return false;
        const char *inf = "Infinity";
        for (int k = 1; k < 8; k++)
            if (b[p + k] != (uint8_t)inf[k]) return false;
        out = neg ? -__longlong_as_double(0x7ff0000000000000ll) : __longlong_as_double(0x7ff0000000000000ll);
        return true;
    }
    if (c == '0' && e - p > 1 && (b[p + 1] == 'x' || b[p + 1] == 'X')) {
        // 0[xX] (H+ .? | H* . H+) [pP] [+-]? D+ [fFdD]?
        int64_t q = p + 2;
        uint64_t m = 0;
        int nh = 0, e2 = 0;
        bool point = false, sticky = false, any = false;
        for (; q < e; q++) {
            const uint32_t ch = b[q];
            if (ch == '.') {
                if (point) break;
                point = true;
                continue;
            }
            const int h = hex_val(ch);
            if (h < 0) break;
            any = true;
            if (nh == 0 && h == 0) { if (point) e2 -= 4; continue; }
            if (nh < 15) {
                m = (m << 4) | (uint64_t)h;
                if (point) e2 -= 4;
            } else {
                if (!point) e2 += 4;
                if (h) sticky = true;
            }
            nh++;
        }
        if (!any || q == e || (b[q] != 'p' && b[q] != 'P')) return false;
        q++;
        int es = 1;
        if (q < e && (b[q] == '+' || b[q] == '-')) { es = b[q] == '-' ? -1 : 1; q++; }
        int ev = 0, ne = 0;
        for (; q < e && is_digit(b[q]); q++, ne++) ev = ev < 100000 ? ev * 10 + (int)(b[q] - '0') : ev;
        if (ne == 0) return false;
        if (q < e && (b[q] == 'f' || b[q] == 'F' || b[q] == 'd' || b[q] == 'D')) q++;
        if (q != e) return false;
        const double v = make_double(m, e2 + es * ev, sticky);
        out = neg ? -v : v;
        return true;
    }
    // decimal: D* (. D*)? with >= 1 digit, ([eE] [+-]? D+)?, [fFdD]?
    const int64_t q0 = p;
    uint64_t w = 0;
    int nsig = 0, nd = 0, E = 0;
    bool point = false, trunc = false;
    int64_t q = p;
    for (; q < e; q++) {
        const uint32_t ch = b[q];
        if (is_digit(ch)) {
            const uint32_t d = ch - '0';
            nd++;
            if (nsig == 0 && d == 0) { if (point) E--; continue; }
            if (nsig < 19) {
                w = w * 10u + d;
                if (point) E--;
            } else {
                if (!point) E++;
                if (d) trunc = true;
            }
            nsig++;
        } else if (ch == '.' && !point) {
            point = true;
        } else {
            break;
        }
    }
    if (nd == 0) return false;
    const int64_t qe = q;
    int ev = 0;
    if (q < e && (b[q] == 'e' || b[q] == 'E')) {
        q++;
        int es = 1;
        if (q < e && (b[q] == '+' || b[q] == '-')) { es = b[q] == '-' ? -1 : 1; q++; }
        int ne = 0;
        for (; q < e && is_digit(b[q]); q++, ne++) ev = ev < 100000 ? ev * 10 + (int)(b[q] - '0') : ev;
        if (ne == 0) return false;
        ev *= es;
    }
    if (q < e && (b[q] == 'f' || b[q] == 'F' || b[q] == 'd' || b[q] == 'D')) q++;
    if (q != e) return false;
    double v;
    if (nsig == 0) {
        v = 0.0;
    } else {
        const int ex = E + ev;
        if (!trunc && w <= (1ull << 53) && ex >= -22 && ex <= 22) {
            const double wd = (double)w;   // exact
            v = ex == 0 ? wd : (ex > 0 ? wd * exact_pow10(ex) : wd / exact_pow10(-ex));
        } else {
            if (!kFull) return 2;
            v = decimal_slow(b.p, b.off, q0, qe, ev, w, ex);
        }
    }
    out = neg ? -v : v;
    return true;
}

// Long.parseLong (radix 10): no trim, optional sign, >= 1 ASCII digit, range-checked
template <typename Src>
__device__ __forceinline__ bool java_parse_long(const Src b, int64_t s, int64_t e, int64_t &out) {
    if (s == e) return false;
    bool neg = false;
    const uint32_t c0 = b[s];
    if (c0 == '+' || c0 == '-') { neg = c0 == '-'; s++; }
    if (s == e) return false;
    const uint64_t lim = neg ? 0x8000000000000000ull : 0x7fffffffffffffffull;
    uint64_t v = 0;
    for (; s < e; s++) {
        const uint32_t c = b[s];
        if (!is_digit(c)) return false;
        const uint64_t d = c - '0';
        if (v > (lim - d) / 10u) return false;
        v = v * 10u + d;
    }
    out = neg ? (int64_t)(0ull - v) : (int64_t)v;
    return true;
}

// one record b[s, e) -> status; values are written to row[0..D) as they parse
template <typename Src>
__device__ __forceinline__ uint8_t parse_record(const Src b, int64_t s, int64_t e, int D, int64_t &id,
                                                double *__restrict__ row) {
    int64_t id_s = s, id_e = s;
    int field = 0, nvals = 0, pending_empty = 0;
    bool bad = false;
    int64_t fs = s;
    for (int64_t q = s;; q++) {
        const bool end = q == e;
        if (!end && b[q] != ',') continue;
        if (field == 0) {
            id_e = q;
        } else if (fs == q) {
            pending_empty++;   // empty field: fine only if every later field is empty too (split drops them)
        } else {
            double v;
            if (pending_empty > 0 || !java_parse_double<true>(b, fs, q, v)) bad = true;
            else if (nvals < D) row[nvals] = v;
            nvals++;
        }
        field++;
        fs = q + 1;
        if (end || bad) break;
    }
    if (bad || nvals == 0) return SKY_CSV_MALFORMED;   // ServiceTuple.java:93,101-103
    if (!java_parse_long(b, id_s, id_e, id)) return SKY_CSV_BAD_ID;   // FlinkSkyline.java:276
    if (nvals != D) return SKY_CSV_ARITY;
    return SKY_CSV_OK;
}


// ---- main pass: one workgroup = 256 consecutive records, one lane per FIELD.
// Lane-per-record parsing diverges (every lane reaches its commas at a different
// character); here all lanes run the same short field parse.  Steps:
//  1. stage the records' bytes in LDS (coalesced dword loads);
//  2. each lane scans a contiguous run of staged words for ',' / '\n' (zero-byte test),
//     a block scan numbers the delimiters, and their offsets (u16) + record (u8) go to LDS;
//  3. fields are parsed round-robin (field f = bytes after delimiter f-1 up to delimiter f):
//     column 0 -> Long.parseLong, others -> Double.parseDouble, values stored straight into
//     the row-major output (consecutive fields -> consecutive addresses);
//  4. per record: split's trailing-empty rule, fromString's null cases, arity -> status.
// A workgroup whose records exceed the LDS window or kFieldsMax fields is listed for
// k_csv_records (lane per record, reading HBM).
constexpr int kFieldsMax = 2048;
constexpr int kCsvFastDims = 8;           // lane-per-record fast path: records of D <= 8 values
constexpr int kFieldText = 10 * 1024;   // ~19 KB of LDS per workgroup in all: 8 workgroups (32 waves) per CU


// SWAR fast path (simdjson's eight-digit parse), branch-free: bytes [s, s+len) of the staged
// words, 1 <= len <= 16, all ASCII digits -> value.  Covers the producer's payload (plain
// non-negative integers).  Two 8-byte windows are always formed, padded with leading '0's,
// validated and converted with selects only, so a wave whose lanes hold ids and values of
// different lengths runs one straight-line sequence.
__device__ __forceinline__ uint64_t swar_pad(uint64_t x, int L) {   // L in 0..8, first char in the low byte
    const uint64_t z = 0x3030303030303030ull;
    const int l = L < 1 ? 1 : (L > 7 ? 7 : L);                      // keep both shifts in 8..56
    const uint64_t y = (x << (8 * (8 - l))) | (z >> (8 * l));
    return L == 0 ? z : (L == 8 ? x : y);
}
__device__ __forceinline__ bool swar_is_digits(uint64_t y) {
    return (y & 0xF0F0F0F0F0F0F0F0ull) == 0x3030303030303030ull &&
           ((y + 0x0606060606060606ull) & 0xF0F0F0F0F0F0F0F0ull) == 0x3030303030303030ull;
}
__device__ __forceinline__ uint32_t swar_value(uint64_t y) {
    y -= 0x3030303030303030ull;
    y = (y * 10u) + (y >> 8);
    y = (((y & 0x000000FF000000FFull) * 0x000F424000000064ull) +
         (((y >> 16) & 0x000000FF000000FFull) * 0x0000271000000001ull)) >> 32;
    return (uint32_t)y;
}
__device__ __forceinline__ bool swar_digits(const uint32_t *__restrict__ buf, int s, int len, uint64_t &v) {
    const int k = s >> 2, sh = (s & 3) * 8;
    const uint64_t A = (uint64_t)buf[k] | ((uint64_t)buf[k + 1] << 32);
    const uint64_t B = (uint64_t)buf[k + 2] | ((uint64_t)buf[k + 3] << 32);
    const uint64_t C = buf[k + 4];
    const int shr = sh ? 64 - sh : 32;                               // unused when sh == 0
    const uint64_t x0 = sh ? (A >> sh) | (B << shr) : A;
    const uint64_t x1 = sh ? (B >> sh) | (C << shr) : B;
    const int L0 = len < 8 ? len : 8, L1 = len > 8 ? len - 8 : 0;   // L1 <= 8 for len <= 16
    const uint64_t y0 = swar_pad(x0, L0), y1 = swar_pad(x1, L1 > 8 ? 8 : L1);
    const bool ok = len >= 1 && len <= 16 && swar_is_digits(y0) && swar_is_digits(y1);
    uint32_t p = (L1 & 1) ? 10u : 1u;
    p *= (L1 & 2) ? 100u : 1u;
    p *= (L1 & 4) ? 10000u : 1u;
    p = (L1 & 8) ? 100000000u : p;
    v = (uint64_t)swar_value(y0) * p + swar_value(y1);
    return ok;
}

// the same for len <= 8, in 32-bit operations only (the 64-bit shifts and multiplies of the
// general path issue at a fraction of the rate): the producer's ids (< 10^8 for 100M records)
// and values (<= 4 digits) all take it; chosen per wave, so the branch is uniform.  The
// window is the 8 bytes [e - 8, e) that END at the field's delimiter (two v_alignbyte from
// three LDS words; buf must be readable 8 bytes before its start), with the bytes before s
// replaced by '0' — right-aligned, so the digit weights are fixed.
__device__ __forceinline__ uint32_t swar4_value(uint32_t d) {      // 4 digit bytes (0..9), first = most significant
    // bytes 0 / 2 of 10 d + (d >> 8): two-digit values.  A 24-bit multiply-add (byte 3 of 10 d is
    // not needed); written out because the compiler otherwise picks v_mad_u64_u32 for it
    uint32_t t;
    asm("v_mad_u32_u24 %0, %1, 10, %2" : "=v"(t) : "v"(d), "v"(d >> 8));
    return (t & 0xffu) * 100u + ((t >> 16) & 0xffu);
}
__device__ __forceinline__ uint32_t swar4_bad(uint32_t w) {        // 0 iff every byte is an ASCII digit
    return ((w & 0xF0F0F0F0u) ^ 0x30303030u) | (((w + 0x06060606u) & 0xF0F0F0F0u) ^ 0x30303030u);
}
__device__ __forceinline__ bool swar_digits8(const uint32_t *__restrict__ buf, int s, int e, uint32_t &v) {
    const int b = e - 8;
    const int k = b >> 2;                                           // >= -2
    const uint32_t sh = (uint32_t)b & 3u;
    const uint32_t x0 = buf[k], x1 = buf[k + 1], x2 = buf[k + 2];
    const uint32_t len = (uint32_t)(e - s);
    const uint64_t m = (1ull << (8u * (8u - min(max(len, 1u), 8u)))) - 1ull;   // the bytes before s
    const uint32_t m0 = (uint32_t)m, m1 = (uint32_t)(m >> 32);
    const uint32_t w0 = (__builtin_amdgcn_alignbyte(x1, x0, sh) & ~m0) | (0x30303030u & m0);
    const uint32_t w1 = (__builtin_amdgcn_alignbyte(x2, x1, sh) & ~m1) | (0x30303030u & m1);
    v = swar4_value(w0 - 0x30303030u) * 10000u + swar4_value(w1 - 0x30303030u);
    return ((swar4_bad(w0) | swar4_bad(w1)) == 0u) & (len - 1u < 8u);   // no short circuit: no branch
}

// CHUNK = false: workgroup b parses records [b R, b R + R) (group boundaries from k_csv_group_pos).
// CHUNK = true (no group pass): workgroup c parses the records that START in the byte chunk
// [c C, c C + C): it stages the chunk plus a tail for its last record, finds its first record
// start and its last record's end itself, and takes its first record's index from the count
// pass's prefix at the 4 KB block holding byte c C - 1 plus its own count of the newlines between
// that block's start and c C - 1.  Chunks that do not fit (a record past the staged tail, > 256
// records, > kFieldsMax fields) are listed as spans for k_csv_records.
struct CsvChunkArgs {
    const uint32_t *blk_off;     // exclusive newline counts per 4 KB count chunk
    const uint32_t *cnt1k;       // newline counts per 1 KB
    longlong4 *spans;            // (start, end or -1, first record, records) of listed chunks
    int chunk;                   // C, bytes (multiple of 16)
    int tail;                    // bytes staged past the chunk (C + 16 + tail <= kFieldText)
};
template <bool CHUNK>
__global__ __launch_bounds__(kCsvThreads) void k_csv_fields(const uint8_t *__restrict__ text, int64_t nbytes,
                                                            const int64_t *__restrict__ line_g, int64_t nl,
                                                            int64_t nrec, int D, int64_t *__restrict__ ids,
                                                            double *__restrict__ vals, uint8_t *__restrict__ status,
                                                            unsigned long long *__restrict__ counts,
                                                            uint32_t *__restrict__ spill,
                                                            longlong3 *__restrict__ slow,
                                                            unsigned long long *__restrict__ slow_n,
                                                            unsigned long long slow_cap, int R, int stop,
                                                            CsvChunkArgs ca) {
    // s_buf[-4, 0): readable front pad for swar_digits8's window (masked bytes)
    __shared__ __attribute__((aligned(16))) uint32_t s_bufp[4 + kFieldText / 4 + 8];
    uint32_t *const s_buf = s_bufp + 4;
    // delimiter f: staged byte offset | record << 16; s_dl[-1] closes the field before the first
    __shared__ __attribute__((aligned(16))) uint32_t s_dlp[1 + kFieldsMax + kCsvThreads];   // + one dummy slot per lane
    static_assert(2 * 64 * (kCsvFastDims + 1) * 8 <= (1 + kFieldsMax + kCsvThreads) * 4 &&
                      2 * 64 * (kCsvFastDims + 1) * 8 <= kFieldText, "two waves' row images per array");
    uint32_t *const s_dl = s_dlp + 1;
    __shared__ uint16_t s_rfirst[kCsvThreads + 1 + kCsvThreads];   // + one dummy slot per lane
    __shared__ int s_fempty[kCsvThreads];
    __shared__ uint8_t s_bad[kCsvThreads], s_idok[kCsvThreads];
    __shared__ uint32_t s_w[8], s_cnt[4];
    const int tid = threadIdx.x;
    constexpr int kUnits = (kFieldText / 16 + kCsvThreads - 1) / kCsvThreads;   // 3
    const bool aligned = ((uintptr_t)text & 15) == 0;
    int64_t r0, a0;
    int nr, nq, lo, hi;
    bool tail_open;
    uint32_t dw[kUnits * 4];
    // stage the 16-byte units [a0 + 16 q, ...) for q < nq: lane tid owns [tid*per, tid*per + per)
    // (registers + LDS), and numbers its delimiters later without re-reading LDS
    auto stage = [&](int per) {
#pragma unroll
        for (int u = 0; u < kUnits; u++) {
            const int q = tid * per + u;
            uint4 x = make_uint4(0, 0, 0, 0);
            if (u < per && q < nq) {
                const int64_t o = a0 + 16 * (int64_t)q;
                if (aligned && o + 16 <= nbytes) {
                    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                    const u32x4 y = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(text + o));
                    x = make_uint4(y.x, y.y, y.z, y.w);
                } else {
                    uint32_t t[4] = {0, 0, 0, 0};
                    for (int k = 0; k < 16; k++)
                        if (o + k < nbytes) t[k >> 2] |= (uint32_t)text[o + k] << (8 * (k & 3));
                    x = make_uint4(t[0], t[1], t[2], t[3]);
                }
                reinterpret_cast<uint4 *>(s_buf)[q] = x;
            }
            dw[4 * u] = x.x; dw[4 * u + 1] = x.y; dw[4 * u + 2] = x.z; dw[4 * u + 3] = x.w;
        }
    };
    int per;
    uint64_t cm64 = 0, nl64 = 0;                            // CHUNK: the lane's ',' / '\n' bits, unclipped
    auto below = [](int b) -> uint64_t {                    // bits [0, b), b clamped to [0, 64]
        return b <= 0 ? 0ull : (b >= 64 ? ~0ull : (1ull << b) - 1ull);
    };
    if constexpr (!CHUNK) {
        r0 = (int64_t)blockIdx.x * R;                       // R <= 256 records per workgroup (host-chosen)
        nr = (int)(nrec - r0 < R ? nrec - r0 : R);
        const int64_t rl = r0 + nr - 1;
        // group boundaries (k_csv_group_pos): the last group ends at the end of the text (its last
        // record has no '\n', or its '\n' is the last byte)
        const int64_t span_s = r0 == 0 ? 0 : line_g[blockIdx.x - 1] + 1;
        tail_open = rl >= nl;                               // last record has no '\n'
        const int64_t span_e = tail_open || nr < R ? nbytes : line_g[blockIdx.x] + 1;   // includes the final '\n'
        a0 = span_s & ~15ll;
        if (span_e - a0 > kFieldText) {                     // uniform per block
            if (tid == 0) spill[1 + atomicAdd(&spill[0], 1u)] = blockIdx.x;
            return;
        }
        if (stop == 4) return;
        nq = (int)((span_e - a0 + 15) >> 4);
        per = (nq + kCsvThreads - 1) / kCsvThreads;
        lo = (int)(span_s - a0);
        hi = (int)(span_e - a0);                            // staged byte range of the records
        stage(per);
    } else {
        __shared__ int s_red[kCsvThreads / 64][4];          // per wave: newlines, first, end, prefix newlines
        const int64_t c = blockIdx.x;
        const int64_t cs = c * ca.chunk, ce = min(cs + ca.chunk, nbytes);
        a0 = c ? cs - 16 : 0;                               // byte cs - 1 tells whether a record starts at cs
        const int64_t wend = min(a0 + 16 + ca.chunk + ca.tail, nbytes);
        nq = (int)((wend - a0 + 15) >> 4);
        per = (nq + kCsvThreads - 1) / kCsvThreads;
        // the newlines in [b_s, cs - 1), b_s = the start of the count block holding byte cs - 1
        // (< 4 KB, one 16-byte load per lane; the previous chunk staged most of them: L2-hot).
        // Chunks of whole count blocks start at a block boundary: then only byte cs - 1 (staged
        // here) is between the block's prefix and cs - 1, and nothing is loaded
        const bool blk_aligned = (ca.chunk & (kCsvCountBlk - 1)) == 0;
        const int64_t blk0 = c ? (blk_aligned ? cs / kCsvCountBlk : (cs - 1) / kCsvChunk) : 0;
        uint32_t nlb = 0;
        if (c && blk_aligned && tid < (int)(blk0 & 3)) nlb = ca.cnt1k[(blk0 & ~3ll) + tid];   // the 4 KB block's earlier KBs
        if (c && !blk_aligned) {
            const int64_t bs = blk0 * kCsvChunk, base = bs + 16 * tid;
            if (base < cs - 1) {
                uint32_t w[4];
                load16(text, nbytes, base, aligned, w);
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int64_t v = min<int64_t>(max<int64_t>(cs - 1 - (base + 4 * k), 0), 4);   // bytes before cs - 1
                    const uint32_t keep = v >= 4 ? 0x80808080u : (0x80808080u & ((1u << (8 * v)) - 1u));
                    nlb += __popc(nl_in_word(w[k]) & keep);
                }
            }
        }
        stage(per);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) nlb += __shfl_xor(nlb, o, 64);
        // newlines in [wlo, whi) start this chunk's records; the first one at or after whi ends its last
        const int wlo = c ? (int)(cs - 1 - a0) : 0, whi = (int)(ce - 1 - a0);
        // the lane's newlines as one bit per staged byte (as in the delimiter pass below), then the
        // window's count / first and the first at or after whi by popcount / ctz, no bit loops
        // (the ',' masks too: the delimiter pass below only clips them to [lo, hi))
        const int L0 = 16 * (tid * per);
#pragma unroll
        for (int k = 0; k < kUnits * 4; k++) {
            const uint32_t mn = k < per * 4 ? byte_eq_mask(dw[k], 0x0a0a0a0au) : 0u;   // unstaged bytes are 0
            const uint32_t mc = k < per * 4 ? byte_eq_mask(dw[k], 0x2c2c2c2cu) : 0u;
            nl64 |= (uint64_t)((mn * 0x00204081u) >> 28) << (4 * k);
            cm64 |= (uint64_t)((mc * 0x00204081u) >> 28) << (4 * k);
        }
        const uint64_t nlm = nl64;
        const uint64_t inw = nlm & below(whi - L0) & ~below(wlo - L0), aft = nlm & ~below(whi - L0);
        uint32_t cnt = (uint32_t)__popcll(inw);
        int first = inw ? L0 + (int)__builtin_ctzll(inw) : 0x7fffffff;
        int endp = aft ? L0 + (int)__builtin_ctzll(aft) : 0x7fffffff;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            cnt += __shfl_xor(cnt, o, 64);
            first = min(first, __shfl_xor(first, o, 64));
            endp = min(endp, __shfl_xor(endp, o, 64));
        }
        if ((tid & 63) == 0) {
            s_red[tid >> 6][0] = (int)cnt;
            s_red[tid >> 6][1] = first;
            s_red[tid >> 6][2] = endp;
            s_red[tid >> 6][3] = (int)nlb;
        }
        __syncthreads();                                    // (also: the staged text)
        int s_nlw = 0, s_nlb = 0, s_first = 0x7fffffff, s_end = 0x7fffffff;
#pragma unroll
        for (int i = 0; i < kCsvThreads / 64; i++) {
            s_nlw += s_red[i][0];
            s_first = min(s_first, s_red[i][1]);
            s_end = min(s_end, s_red[i][2]);
            s_nlb += s_red[i][3];
        }
        nr = s_nlw + (c == 0 ? 1 : 0);
        if (nr == 0 || stop == 4) return;
        // records before the chunk: record 0 + one per newline in [0, cs - 1)
        r0 = c == 0 ? 0
                    : 1 + (int64_t)ca.blk_off[blk_aligned ? blk0 >> 2 : blk0] + (int64_t)s_nlb -
                          (blk_aligned && (s_buf[3] >> 24) == 0x0au ? 1 : 0);   // byte cs - 1 = staged byte 15
        lo = c ? s_first + 1 : 0;
        tail_open = false;
        if (s_end != 0x7fffffff) {
            hi = s_end + 1;
        } else if (wend == nbytes) {
            hi = (int)(nbytes - a0);                        // the text's last record, without '\n'
            tail_open = true;
        } else {
            hi = -1;                                        // the last record runs past the staged tail
        }
        if (hi < 0 || nr > kCsvThreads) {
            if (tid == 0)
                ca.spans[atomicAdd(&spill[0], 1u)] = make_longlong4(a0 + lo, hi < 0 ? -1ll : a0 + hi, r0, nr);
            return;
        }
    }
    if (stop == 1) { __syncthreads(); if (s_buf[tid] == 0x12345678u) status[0] = 9; return; }
    if (tid < 4) s_cnt[tid] = 0;
    for (int i = tid; i < kFieldText / 32 + 4; i += kCsvThreads) s_dlp[i] = 0;   // 2b's bitmap
    s_fempty[tid] = 0x7fffffff;
    s_bad[tid] = 0;
    s_idok[tid] = 1;                                       // cleared by a failed id parse
    // the lane's delimiters as bit masks over its <= 48 staged bytes (bit b = byte b of its
    // range, bytes 0-31 in md0 / mnl0, 32-47 in md1 / mnl1): ',' or '\n' in md, '\n' in mnl.
    // Each word's four 0x80 flags are gathered into a nibble by one multiply (bits 7 / 15 /
    // 23 / 31 -> 28..31, no carries)
    static_assert(kUnits * 16 <= 64, "two 32-bit masks per lane");
    uint32_t md0, mnl0, md1, mnl1;
    {
        if constexpr (!CHUNK) {                             // (CHUNK: the prologue's masks)
#pragma unroll
            for (int k = 0; k < kUnits * 4; k++) {          // unstaged words are 0: no flags
                const uint32_t mn = byte_eq_mask(dw[k], 0x0a0a0a0au), mc = byte_eq_mask(dw[k], 0x2c2c2c2cu);
                nl64 |= (uint64_t)((mn * 0x00204081u) >> 28) << (4 * k);
                cm64 |= (uint64_t)((mc * 0x00204081u) >> 28) << (4 * k);
            }
        }
        const int L0 = 16 * (tid * per);                    // clipped to [lo, hi)
        const uint64_t clip = below(hi - L0) & ~below(lo - L0);
        const uint64_t d = (cm64 | nl64) & clip, n = nl64 & clip;
        md0 = (uint32_t)d;
        md1 = (uint32_t)(d >> 32);
        mnl0 = (uint32_t)n;
        mnl1 = (uint32_t)(n >> 32);
    }
    const uint32_t nd = __popc(md0) + __popc(md1), nn = __popc(mnl0) + __popc(mnl1);
    // block exclusive scan of (nd, nn), packed in 16-bit halves (a workgroup stages <= 12 KB)
    const int lane = tid & 63, wv = tid >> 6;
    const uint32_t x0 = nd | (nn << 16);
    uint32_t x = x0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t a = __shfl_up(x, o, 64);
        if (lane >= o) x += a;
    }
    if (lane == 63) s_w[wv] = x;
    __syncthreads();
    uint32_t base = x - x0, tot = 0;
    for (int i = 0; i < 4; i++) {
        if (i < wv) base += s_w[i];
        tot += s_w[i];
    }
    const uint32_t fbase = base & 0xffffu, rbase = base >> 16, ftot = tot & 0xffffu;
    const int nf = (int)ftot + (tail_open ? 1 : 0);
    const int nnl = (int)(tot >> 16);
    // 2b. the producer's shape, one lane per RECORD: when the workgroup holds exactly D + 1 fields
    // per record (D <= 8), every lane walks its own record: the delimiter masks the lanes already
    // hold go to an LDS bitmap (one bit per staged byte, two ds_or per lane), a lane reads its
    // record's 64 bits of it (records < 64 bytes; inside a record every delimiter is a ','), and
    // each field is one ctz + the 32-bit SWAR conversion, values in registers.  Straight-line for
    // every lane (a field count fixed by D, no grammar branches), so the divergence that sank
    // lane-per-record parsing in round 1 (the general grammar, from HBM) does not arise, and only
    // the newlines are numbered (~1 per lane, not every delimiter).  If ANY record of the
    // workgroup is not plain digit fields of 1..8 characters, nothing has been stored and the
    // workgroup takes the general path below on the same staged text.
    if (D <= kCsvFastDims && nf == nr * (D + 1) && nnl + (tail_open ? 1 : 0) == nr) {   // uniform per block
        uint16_t *const s_nl = s_rfirst;                    // newline k closes record k (rewritten below)
        uint32_t *const s_bits = s_dlp;                     // delimiter bitmap (zeroed above, rewritten below)
        {
            const uint32_t b0 = 16u * (uint32_t)(tid * per);
            const uint64_t x = ((uint64_t)md0 | ((uint64_t)md1 << 32)) << (b0 & 31u);   // <= 48 bits, shift 0 / 16
            if ((uint32_t)x) atomicOr(&s_bits[b0 >> 5], (uint32_t)x);
            if ((uint32_t)(x >> 32)) atomicOr(&s_bits[(b0 >> 5) + 1], (uint32_t)(x >> 32));
            uint64_t m = (uint64_t)mnl0 | ((uint64_t)mnl1 << 32);
            uint32_t r = rbase;
            while (m) {
                s_nl[r++] = (uint16_t)(b0 + (uint32_t)__builtin_ctzll(m));
                m &= m - 1ull;
            }
        }
        if (tail_open && tid == 0) s_nl[nr - 1] = (uint16_t)hi;   // the tail record ends at the text's end
        __syncthreads();
        if (stop == 6) { if (s_nl[tid] == 0x1234u) status[0] = 9; return; }
        bool ok = true;
        uint32_t idv = 0;
        double v[kCsvFastDims];
        if (tid < nr) {
            const int e = s_nl[tid];
            const int s0 = tid ? (int)s_nl[tid - 1] + 1 : lo;
            const int len = e - s0;
            int p = s0;
            const uint32_t w = (uint32_t)s0 >> 5, o = (uint32_t)s0 & 31u;
            const uint32_t y0 = s_bits[w], y1 = s_bits[w + 1], y2 = s_bits[w + 2];
            uint64_t m = (uint64_t)__builtin_amdgcn_alignbit(y1, y0, o) | ((uint64_t)__builtin_amdgcn_alignbit(y2, y1, o) << 32);
            m &= (1ull << (len & 63)) - 1ull;               // the record's bytes [p, e): its ','s
            ok = (len < 64) & (__popcll(m) == D);
#pragma unroll
            for (int f = 0; f <= kCsvFastDims; f++) {
                if (f > D) continue;                        // uniform
                const int end = f < D ? min(s0 + (int)__builtin_ctzll(m | (1ull << 63)), e) : e;
                m &= m - 1ull;
                uint32_t u;
                ok &= swar_digits8(s_buf, p, end, u);       // 1..8 digits
                if (f == 0) idv = u;
                else v[f - 1] = (double)u;
                p = end + 1;
            }
        }
        const int all_ok = __syncthreads_and(ok ? 1 : 0);
        if (stop == 5) { if (!all_ok && tid == 0) atomicAdd(&counts[0], 1ull); if (idv == 0x12345u) status[0] = (uint8_t)v[0]; return; }
        if (all_ok) {
            // each wave's <= 64 rows through its own LDS image (row stride D + 1 doubles: 2-way
            // banks at most), then D lane-contiguous 8-byte stores per wave; the text and the
            // bitmap are dead now (the barrier above)
            const int w = tid >> 6, l = tid & 63;
            double *const img = reinterpret_cast<double *>(w < 2 ? reinterpret_cast<uint32_t *>(s_buf) : s_dlp) +
                                (w & 1) * 64 * (kCsvFastDims + 1);
            const int nw = min(max(nr - 64 * w, 0), 64);
#pragma unroll
            for (int c = 0; c < kCsvFastDims; c++)
                if (c < D) img[l * (D + 1) + c] = v[c];
            __builtin_amdgcn_wave_barrier();
            double *const out = vals + (r0 + 64 * w) * D;
            const uint32_t mD = (65536u + (uint32_t)D - 1u) / (uint32_t)D;   // i / D = (i mD) >> 16 for i < 512
#pragma unroll
            for (int k = 0; k < kCsvFastDims; k++) {
                const uint32_t i = (uint32_t)(k * 64 + l), row = (i * mD) >> 16;
                if (k < D && (int)i < nw * D) out[i] = img[row * (D + 1) + (i - row * D)];
            }
            if (tid < nr) {
                ids[r0 + tid] = (int64_t)idv;
                status[r0 + tid] = SKY_CSV_OK;
            }
            return;
        }
    }
    if (nf > kFieldsMax) {                                 // uniform per block
        if (tid == 0) {
            if constexpr (CHUNK) ca.spans[atomicAdd(&spill[0], 1u)] = make_longlong4(a0 + lo, a0 + hi, r0, nr);
            else spill[1 + atomicAdd(&spill[0], 1u)] = blockIdx.x;
        }
        return;
    }
    if (tid == 0) {
        s_rfirst[0] = 0;
        s_dl[-1] = (uint32_t)(lo - 1) & 0xffffu;           // field 0 starts at lo
        if (tail_open) {                                   // virtual delimiter closing the tail record
            s_dl[nf - 1] = (uint32_t)hi | ((uint32_t)(nr - 1) << 16);
            s_rfirst[nr] = (uint16_t)nf;
        }
    }
    {
        // per half, one pass over the lane's set bits, as many steps as the wave's busiest lane
        // has delimiters there; the stores of a lane that has run out (or of a ',') go to its
        // own dummy slot instead of being branched around
        uint32_t f = fbase, rec = rbase;
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const uint32_t b0 = 16u * (uint32_t)(tid * per) + 32u * h;
            uint32_t m = h ? md1 : md0;
            const uint32_t mnl = h ? mnl1 : mnl0;
            while (__ballot(m != 0u)) {
                const bool has = m != 0u;
                const uint32_t low = m & (0u - m);
                const uint32_t bit = __builtin_ctz(m | 0x80000000u);   // 31 past the last: unused
                m ^= low;
                const uint32_t isn = (mnl & low) ? 1u : 0u;
                s_dl[has ? f : (uint32_t)(kFieldsMax + tid)] = (b0 + bit) | (rec << 16);
                rec += isn;
                s_rfirst[isn ? rec : (uint32_t)(kCsvThreads + 1 + tid)] = (uint16_t)(f + 1);
                f += has ? 1u : 0u;
            }
        }
    }
    __syncthreads();
    if (stop == 2) { if (s_dl[tid] == 0x1234u) status[0] = 9; return; }
    // 3. fields.  Common case, straight-line: a plain digit field (the SWAR path) that is an
    // id or an in-range value of <= 15 digits -> one 8-byte store, its address and bits
    // selected (ids and values interleave in every wave; exec-masked branches per kind cost
    // more than the selects).  Everything else (empty, signs, decimals, exponents, NaN /
    // Infinity, long digit strings, extra fields) takes the full grammar below.
    const LdsSrc src{reinterpret_cast<const uint8_t *>(s_buf), 0};
    int64_t *const ids_b = ids + r0;
    double *const vals_b = vals + r0 * D - 1;              // + j * D + col, col >= 1
    for (int f = tid; f < nf; f += kCsvThreads) {
        const uint32_t dp = s_dl[f - 1], dl = s_dl[f];
        const int s = (int)(((dp & 0xffffu) + 1u) & 0xffffu);
        const int e = (int)(dl & 0xffffu);
        const int j = (int)(dl >> 16);
        const int col = f - (int)s_rfirst[j];
        const bool is_id = col == 0;
        uint64_t u = 0;
        double v;
        bool fast;
        if (__ballot(e - s > 8) == 0ull) {
            uint32_t u32;
            fast = swar_digits8(s_buf, s, e, u32);
            u = u32;
            v = (double)u32;
        } else {
            fast = swar_digits(s_buf, s, e - s, u);
            v = (double)u;                                 // exact when len <= 15
        }
        if (fast & (is_id | ((e - s <= 15) & (col <= D)))) {
            const uint32_t off = is_id ? (uint32_t)j : __umul24((uint32_t)j, (uint32_t)D) + (uint32_t)col;
            int64_t *const p = (is_id ? ids_b : reinterpret_cast<int64_t *>(vals_b)) + off;
            *p = is_id ? (int64_t)u : __double_as_longlong(v);   // id < 10^16
            continue;
        }
        const bool empty = s == e;
        int64_t idv = (int64_t)u;
        bool idok = fast;
        int pr = 1;
        if (!(fast && (is_id || e - s <= 15)) && !empty) {   // rare: the full Java grammar
            if (is_id) idok = java_parse_long(src, s, e, idv);
            else pr = java_parse_double<false>(src, s, e, v);
        }
        if (is_id) {
            ids_b[j] = idv;
            s_idok[j] = idok;
        } else if (empty) {
            atomicMin(&s_fempty[j], col);
        } else {
            if (pr == 0) {
                s_bad[j] = 1;
            } else if (col <= D) {
                const int64_t o = (r0 + j) * D + col - 1;
                if (pr == 1) {
                    vals[o] = v;
                } else {                                   // exact path, in k_csv_slow
                    const unsigned long long k = atomicAdd(slow_n, 1ull);
                    if (k < slow_cap) slow[k] = make_longlong3(a0 + s, a0 + e, o);
                }
            }
        }
    }
    __syncthreads();
    if (stop == 3) return;
    // 4. records.  The last non-empty column: the record's field count - 1 unless it has an empty
    // field (rare: then its fields are walked here) — no per-field LDS atomic (the lanes of one
    // record all hit the same word)
    if (tid < nr) {
        const int f0 = s_rfirst[tid], f1 = s_rfirst[tid + 1];   // delimiters [f0, f1) close its fields
        int last = f1 - f0 - 1;
        if (s_fempty[tid] != 0x7fffffff) {
            last = 0;
            for (int f = f0 + 1; f < f1; f++) {
                const int fs = (int)(s_dl[f - 1] & 0xffffu) + 1, fe = (int)(s_dl[f] & 0xffffu);
                if (fe > fs) last = f - f0;
            }
        }
        uint8_t st;
        if (s_bad[tid] || last == 0 || s_fempty[tid] < last) st = SKY_CSV_MALFORMED;   // ServiceTuple.java:93,101
        else if (!s_idok[tid]) st = SKY_CSV_BAD_ID;                                      // FlinkSkyline.java:276
        else if (last != D) st = SKY_CSV_ARITY;
        else st = SKY_CSV_OK;
        status[r0 + tid] = st;
        if (st != SKY_CSV_OK) atomicAdd(&s_cnt[st], 1u);
    }
    __syncthreads();
    if (tid >= 1 && tid < 4 && s_cnt[tid]) atomicAdd(&counts[tid], (unsigned long long)s_cnt[tid]);
}

// ---- the queued exact conversions (long significands, exponents beyond the fast path)
__global__ __launch_bounds__(kCsvThreads) void k_csv_slow(const uint8_t *__restrict__ text,
                                                          const longlong3 *__restrict__ slow,
                                                          const unsigned long long *__restrict__ slow_n,
                                                          unsigned long long slow_cap, double *__restrict__ vals) {
    const unsigned long long n = *slow_n < slow_cap ? *slow_n : slow_cap;
    for (unsigned long long i = (unsigned long long)blockIdx.x * kCsvThreads + threadIdx.x; i < n;
         i += (unsigned long long)gridDim.x * kCsvThreads) {
        const longlong3 it = slow[i];
        double v = 0.0;
        java_parse_double<true>(GlbSrc{text, 0}, it.x, it.y, v);
        vals[it.z] = v;
    }
}

// ---- fallback: the workgroups k_csv_fields listed (very long records), lane per record from HBM.
// The group's records are found here: the workgroup scans its span (group boundaries from
// k_csv_group_pos, or a listed chunk's span: its first record, and its end when known) 4 KB at
// a time for newlines, numbering them by a block scan; a chunk's records go in rounds of 256.
__global__ __launch_bounds__(kCsvThreads) void k_csv_records(const uint8_t *__restrict__ text, int64_t nbytes,
                                                             const int64_t *__restrict__ line_g, int64_t nl,
                                                             int64_t nrec, int D, int64_t *__restrict__ ids,
                                                             double *__restrict__ vals, uint8_t *__restrict__ status,
                                                             unsigned long long *__restrict__ counts,
                                                             const uint32_t *__restrict__ spill, int64_t all_blocks,
                                                             int R, const longlong4 *__restrict__ spans) {
    __shared__ int64_t s_end[kCsvThreads];                 // record j of the group ends at s_end[j] ('\n')
    __shared__ uint32_t s_w[kCsvThreads / 64];
    const int64_t nlist = all_blocks ? all_blocks : (int64_t)spill[0];
    const bool aligned = ((uintptr_t)text & 15) == 0;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int64_t li = blockIdx.x; li < nlist; li += gridDim.x) {
      int64_t r0, span_s, span_e, left;
      if (spans) {
          const longlong4 sp = spans[li];
          span_s = sp.x;
          span_e = sp.y < 0 ? nbytes : sp.y;
          r0 = sp.z;
          left = sp.w;
      } else {
          const int64_t b = all_blocks ? li : (int64_t)spill[1 + li];
          r0 = b * R;
          left = nrec - r0 < R ? nrec - r0 : R;
          span_s = r0 == 0 ? 0 : line_g[b - 1] + 1;
          const bool tail_open = r0 + left - 1 >= nl;
          span_e = tail_open || left < R ? nbytes : line_g[b] + 1;
      }
      while (left > 0) {                                   // workgroup-uniform
        const int nr = (int)(left < kCsvThreads ? left : kCsvThreads);
        uint32_t found = 0;                                // workgroup-uniform
        for (int64_t a = span_s & ~15ll; a < span_e && found < (uint32_t)nr; a += kCsvChunk) {
            const int64_t base = a + threadIdx.x * 16;
            uint32_t w[4], m[4], c = 0;
            load16(text, nbytes, base, aligned, w);
#pragma unroll
            for (int k = 0; k < 4; k++) {
                m[k] = nl_in_word(w[k]);
                for (int t = 0; t < 4; t++) {              // only the span's bytes
                    const int64_t p = base + 4 * k + t;
                    if (p < span_s || p >= span_e) m[k] &= ~(0x80u << (8 * t));
                }
                c += __popc(m[k]);
            }
            uint32_t inc = c;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t t = __shfl_up(inc, o, 64);
                if (lane >= o) inc += t;
            }
            if (lane == 63) s_w[wv] = inc;
            __syncthreads();
            uint32_t idx = found + inc - c, tot = 0;
            for (int i = 0; i < kCsvThreads / 64; i++) {
                if (i < wv) idx += s_w[i];
                tot += s_w[i];
            }
#pragma unroll
            for (int k = 0; k < 4; k++) {
                uint32_t mk = m[k];
                while (mk) {
                    const int bit = __ffs(mk) - 1;
                    mk &= mk - 1;
                    if (idx < (uint32_t)nr) s_end[idx] = base + k * 4 + (bit >> 3);
                    idx++;
                }
            }
            found += tot;
            __syncthreads();                               // s_w reused by the next step
        }
        if ((int)threadIdx.x < nr) {
            const int j = threadIdx.x;
            const int64_t r = r0 + j;
            const int64_t s = j == 0 ? span_s : s_end[j - 1] + 1;
            const int64_t e = (uint32_t)j < found ? s_end[j] : nbytes;   // the tail record has no '\n'
            int64_t id = 0;
            const uint8_t st = parse_record(GlbSrc{text, 0}, s, e, D, id, vals + r * D);
            ids[r] = id;
            status[r] = st;
            if (st != SKY_CSV_OK) atomicAdd(&counts[st], 1ull);
        }
        const int64_t next = nr <= (int)found ? s_end[nr - 1] + 1 : nbytes;
        __syncthreads();                                   // s_end reused by the next round / group
        r0 += nr;
        left -= nr;
        span_s = next;
      }
    }
}

__global__ void k_csv_keep(const uint8_t *__restrict__ status, int64_t n, uint32_t *__restrict__ keep) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) keep[i] = status[i] == SKY_CSV_OK;
}

__global__ void k_csv_compact(const uint8_t *__restrict__ status, const uint32_t *__restrict__ pos, int64_t n, int D,
                              const int64_t *__restrict__ ids_in, const double *__restrict__ vals_in,
                              int64_t *__restrict__ ids_out, double *__restrict__ vals_out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || status[i] != SKY_CSV_OK) return;
    const int64_t o = pos[i];
    ids_out[o] = ids_in[i];
    for (int j = 0; j < D; j++) vals_out[o * D + j] = vals_in[i * D + j];
}

// ---------------------------------------------------------------- synthetic payload (producer format)
// "id,v1,...,vD\n" with integral values printed like Python's str(int) (python/unified_producer.py:174)
__device__ __forceinline__ int dec_len(uint64_t v) {
    int n = 1;
    while (v >= 10u) { v /= 10u; n++; }
    return n;
}
__device__ __forceinline__ bool int_field(double v, int64_t &iv, bool &neg) {
    if (!(v == v) || fabs(v) >= 9007199254740992.0 || v != trunc(v)) return false;
    iv = (int64_t)v;
    neg = __double_as_longlong(v) < 0;   // keeps -0.0 as "-0"
    return true;
}
__device__ __forceinline__ int field_len(int64_t iv, bool neg) {
    return (neg ? 1 : 0) + dec_len(iv < 0 ? (uint64_t)(-iv) : (uint64_t)iv);
}
__device__ __forceinline__ uint8_t *put_dec(uint8_t *o, int64_t iv, bool neg) {
    if (neg) *o++ = '-';
    uint64_t u = iv < 0 ? (uint64_t)(-iv) : (uint64_t)iv;
    const int n = dec_len(u);
    for (int k = n - 1; k >= 0; k--) { o[k] = (uint8_t)('0' + u % 10u); u /= 10u; }
    return o + n;
}

__global__ void k_csv_fmt_len(const int64_t *__restrict__ ids, const double *__restrict__ vals, int64_t n, int D,
                              uint32_t *__restrict__ len, unsigned long long *__restrict__ tot_err) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t L = 0, bad = 0;
    if (i < n) {
        const int64_t id = ids[i];
        L = field_len(id, id < 0) + 1 + D;   // id, D commas / newline
        for (int j = 0; j < D; j++) {
            int64_t iv;
            bool neg;
            if (!int_field(vals[i * D + j], iv, neg)) { bad = 1; iv = 0; neg = false; }
            L += field_len(iv, neg);
        }
        len[i] = L;
    }
    unsigned long long t = L;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { t += __shfl_xor(t, o, 64); bad |= __shfl_xor(bad, o, 64); }
    if ((threadIdx.x & 63) == 0) {
        if (t) atomicAdd(&tot_err[0], t);
        if (bad) atomicOr(&tot_err[1], 1ull);
    }
}

__global__ void k_csv_fmt_write(const int64_t *__restrict__ ids, const double *__restrict__ vals, int64_t n, int D,
                                const uint32_t *__restrict__ off, uint8_t *__restrict__ text) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint8_t *o = text + off[i];
    const int64_t id = ids[i];
    o = put_dec(o, id, id < 0);
    for (int j = 0; j < D; j++) {
        int64_t iv;
        bool neg;
        if (!int_field(vals[i * D + j], iv, neg)) { iv = 0; neg = false; }
        *o++ = ',';
        o = put_dec(o, iv, neg);
    }
    *o = '\n';
}

// ---------------------------------------------------------------- host launchers
void launch_csv_fmt_len(const int64_t *ids, const double *vals, int64_t n, int D, uint32_t *len,
                        unsigned long long *tot_err, hipStream_t st) {
    if (n == 0) return;
    k_csv_fmt_len<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(ids, vals, n, D, len, tot_err);
}
void launch_csv_fmt_write(const int64_t *ids, const double *vals, int64_t n, int D, const uint32_t *off,
                          uint8_t *text, hipStream_t st) {
    if (n == 0) return;
    k_csv_fmt_write<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(ids, vals, n, D, off, text);
}

int64_t csv_chunks(int64_t nbytes) { return (nbytes + kCsvChunk - 1) / kCsvChunk; }
int64_t csv_count_blocks(int64_t nbytes) { return csv_chunks(nbytes) * (kCsvChunk / kCsvCountBlk); }

void launch_csv_nl_count(const uint8_t *text, int64_t nbytes, uint32_t *blk_cnt, uint32_t *cnt1k,
                         unsigned long long *ncomma, hipStream_t st) {
    const int64_t nb = csv_chunks(nbytes);
    if (nb == 0) return;
    const bool aligned = ((uintptr_t)text & 15) == 0;
    k_csv_nl_count<<<(unsigned)nb, kCsvThreads, 0, st>>>(text, nbytes, aligned, blk_cnt, cnt1k, ncomma);
}
void launch_csv_nl_groups(const uint8_t *text, int64_t nbytes, const uint32_t *blk_off, const uint32_t *cnt1k,
                          int64_t nl, int R, int64_t *line_g, hipStream_t st) {
    const int64_t nb = csv_chunks(nbytes), ngb = nl / R;
    if (nb == 0 || ngb == 0) return;
    const bool aligned = ((uintptr_t)text & 15) == 0;
    k_csv_group_pos<<<(unsigned)((nb + kCsvThreads / 64 - 1) / (kCsvThreads / 64)), kCsvThreads, 0, st>>>(
        text, nbytes, aligned, blk_off, cnt1k, nb, (uint32_t)nl, (uint32_t)R, ngb, line_g);
}
static int csv_stop() {
    const char *e = SKY_MEASURE_ENV("SKY_CSV_STOP");
    return e ? atoi(e) : 0;
}
// spill: device u32 [1 + blocks], spill[0] zeroed by the caller; slow: queue of exact
// conversions (slow_n zeroed by the caller).  If *slow_n ends above slow_cap the caller
// re-parses everything with launch_csv_parse_exact.
void launch_csv_parse(const uint8_t *text, int64_t nbytes, const int64_t *line_g, int64_t nl, int64_t nrec, int D,
                      int64_t *ids, double *vals, uint8_t *status, unsigned long long *counts, uint32_t *spill,
                      longlong3 *slow, unsigned long long *slow_n, unsigned long long slow_cap, int R,
                      hipStream_t st) {
    if (nrec == 0) return;
    const int64_t nb = (nrec + R - 1) / R;
    k_csv_fields<false><<<(unsigned)nb, kCsvThreads, 0, st>>>(text, nbytes, line_g, nl, nrec, D, ids, vals, status,
                                                             counts, spill, slow, slow_n, slow_cap, R, csv_stop(),
                                                             CsvChunkArgs{});
    const unsigned g = (unsigned)(nb < 1024 ? nb : 1024);
    k_csv_records<<<g, kCsvThreads, 0, st>>>(text, nbytes, line_g, nl, nrec, D, ids, vals, status, counts, spill, 0,
                                             R, nullptr);
    k_csv_slow<<<1024, kCsvThreads, 0, st>>>(text, slow, slow_n, slow_cap, vals);
}
// Chunk mode: bytes per chunk from the average record length and field count, so that a chunk's
// records fit one workgroup (<= 0.8 x 256 records, 0.8 x kFieldsMax fields), and the staged tail
// past it (*tail: >= 256 bytes and 4 average records); 0 when the chunk would be under 512 bytes
// The producer's shape (every record D + 1 fields, D <= 8: the lane-per-record path, which has no
// field limit) packs 0.9 x 256 records per workgroup; anything else keeps the general path's margins.
static bool csv_fast_shape(int64_t nrec, int64_t nfields, int D) {
    return D >= 1 && D <= kCsvFastDims && nfields == nrec * (D + 1);
}
int csv_chunk_bytes(int64_t nbytes, int64_t nrec, int64_t nfields, int D, int *tail) {
    if (nrec <= 0 || nbytes <= 0) return 0;
    const double len = (double)nbytes / (double)nrec, nf = (double)nfields / (double)nrec;
    const double fit = csv_fast_shape(nrec, nfields, D)
                           ? 0.9 * kCsvThreads * len
                           : std::min(0.8 * kCsvThreads * len, 0.8 * kFieldsMax / std::max(nf, 1.0) * len);
    const int t = ((int)std::min(std::max(256.0, 4.0 * len), (double)kFieldText / 2) + 15) & ~15;
    int64_t cb = std::min<int64_t>((int64_t)fit, kFieldText - 16 - t) & ~15ll;
    // whole 1 KB count blocks (no newline scan per chunk for its first record's index), and a
    // staged window of <= 8 KB (two 16-byte units per lane: a third of the mask work less) when
    // that keeps >= 3/4 of the records per workgroup
    const int64_t c2 = (int64_t)(8192 - 16 - t) & ~(int64_t)(kCsvCountBlk - 1);
    if (cb >= kCsvCountBlk) cb = (cb >= c2 && 4 * c2 >= 3 * cb) ? c2 : (cb & ~(int64_t)(kCsvCountBlk - 1));
    if (const char *e = SKY_MEASURE_ENV("SKY_CSV_CHUNK_BYTES")) cb = atoi(e) & ~15;   // A/B
    *tail = t;
    return cb >= 512 ? (int)cb : 0;
}
int64_t csv_chunk_count(int64_t nbytes, int chunk) { return (nbytes + chunk - 1) / chunk; }
// blk_off: the count pass's exclusive newline counts per 1 KB; spill[0] zeroed (listed spans:
// spans[0 .. spill[0])), slow_n zeroed
void launch_csv_parse_chunks(const uint8_t *text, int64_t nbytes, int chunk, int tail, const uint32_t *blk_off,
                             const uint32_t *cnt1k, int D,
                             int64_t *ids, double *vals, uint8_t *status, unsigned long long *counts, uint32_t *spill,
                             longlong4 *spans, longlong3 *slow, unsigned long long *slow_n,
                             unsigned long long slow_cap, hipStream_t st) {
    const int64_t nc = csv_chunk_count(nbytes, chunk);
    if (nc == 0) return;
    CsvChunkArgs ca;
    ca.blk_off = blk_off;
    ca.cnt1k = cnt1k;
    ca.spans = spans;
    ca.chunk = chunk;
    ca.tail = tail;
    k_csv_fields<true><<<(unsigned)nc, kCsvThreads, 0, st>>>(text, nbytes, nullptr, 0, 0, D, ids, vals, status, counts,
                                                            spill, slow, slow_n, slow_cap, 0, csv_stop(), ca);
    const unsigned g = (unsigned)(nc < 1024 ? nc : 1024);
    k_csv_records<<<g, kCsvThreads, 0, st>>>(text, nbytes, nullptr, 0, 0, D, ids, vals, status, counts, spill, 0, 0,
                                             spans);
    k_csv_slow<<<1024, kCsvThreads, 0, st>>>(text, slow, slow_n, slow_cap, vals);
}
void launch_csv_parse_exact(const uint8_t *text, int64_t nbytes, const int64_t *line_g, int64_t nl, int64_t nrec,
                            int D, int64_t *ids, double *vals, uint8_t *status, unsigned long long *counts,
                            hipStream_t st) {
    if (nrec == 0) return;
    const int64_t nb = (nrec + kCsvThreads - 1) / kCsvThreads;
    const unsigned g = (unsigned)(nb < 4096 ? nb : 4096);
    k_csv_records<<<g, kCsvThreads, 0, st>>>(text, nbytes, line_g, nl, nrec, D, ids, vals, status, counts, nullptr,
                                             nb, kCsvThreads, nullptr);
}
// records per k_csv_fields workgroup: as many as fit the LDS windows at the stream's average
// record length and field count (outliers spill to k_csv_records)
int csv_records_per_block(int64_t nbytes, int64_t nrec, int64_t nfields, int D) {
    if (nrec <= 0) return kCsvThreads;
    const double len = (double)nbytes / (double)nrec, nf = (double)nfields / (double)nrec;
    const bool fast = csv_fast_shape(nrec, nfields, D);
    int R = kCsvThreads;
    R = std::min<int>(R, (int)((fast ? 0.9 : 0.8) * kFieldText / std::max(len, 1.0)));
    if (!fast) R = std::min<int>(R, (int)(0.8 * kFieldsMax / std::max(nf, 1.0)));
    return std::max(R, 8);
}
void launch_csv_keep(const uint8_t *status, int64_t n, uint32_t *keep, hipStream_t st) {
    if (n == 0) return;
    k_csv_keep<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(status, n, keep);
}
void launch_csv_compact(const uint8_t *status, const uint32_t *pos, int64_t n, int D, const int64_t *ids_in,
                        const double *vals_in, int64_t *ids_out, double *vals_out, hipStream_t st) {
    if (n == 0) return;
    k_csv_compact<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(status, pos, n, D, ids_in, vals_in, ids_out, vals_out);
}

}  // namespace sky
