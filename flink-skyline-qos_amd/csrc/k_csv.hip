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
//   k_csv_nl_write  positions of every '\n' -> line_end[] (record boundaries)
//   k_csv_parse     one lane per record; the workgroup's 256 records are first staged
//                   into LDS with coalesced dword loads, then each lane walks its record:
//                   split semantics, Java trim, the Double.parseDouble grammar, the value
//                   (exact fast path: <= 19 significant digits, w <= 2^53, |e| <= 22, one
//                   correctly rounded IEEE op; otherwise an exact big-integer comparison
//                   against the halfway points, __noinline__ and rare), Long.parseLong.
//   k_csv_compact   only if some record was rejected: stable compaction of the rows.
#include "sky_internal.h"

namespace sky {

constexpr int kCsvThreads = 256;
constexpr int kCsvChunk = kCsvThreads * 16;   // bytes per workgroup in the newline passes
constexpr int kCsvLds = 28 * 1024;            // staged record bytes per workgroup (else read from HBM)

// ---------------------------------------------------------------- newline index
__device__ __forceinline__ uint32_t nl_in_word(uint32_t w) {
    // bytes equal to '\n' (0x0a): classic zero-byte test on w ^ 0x0a0a0a0a, exact per byte
    const uint32_t x = w ^ 0x0a0a0a0au;
    const uint32_t t = ((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x;
    return (~t) & 0x80808080u;   // bit 7 of byte b set iff byte b == '\n'
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
                                                              bool aligned, uint32_t *__restrict__ blk_cnt) {
    __shared__ uint32_t s_w[kCsvThreads / 64];
    const int64_t base = (int64_t)blockIdx.x * kCsvChunk + threadIdx.x * 16;
    uint32_t w[4];
    load16(text, nbytes, base, aligned, w);
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) c += __popc(nl_in_word(w[k]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) blk_cnt[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

__global__ __launch_bounds__(kCsvThreads) void k_csv_nl_write(const uint8_t *__restrict__ text, int64_t nbytes,
                                                              bool aligned, const uint32_t *__restrict__ blk_off,
                                                              int64_t *__restrict__ line_end) {
    __shared__ uint32_t s_w[kCsvThreads / 64];
    const int64_t base = (int64_t)blockIdx.x * kCsvChunk + threadIdx.x * 16;
    uint32_t w[4], m[4];
    load16(text, nbytes, base, aligned, w);
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) { m[k] = nl_in_word(w[k]); c += __popc(m[k]); }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t inc = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
    }
    if (lane == 63) s_w[wv] = inc;
    __syncthreads();
    uint32_t off = blk_off[blockIdx.x] + inc - c;
    for (int i = 0; i < wv; i++) off += s_w[i];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint32_t mk = m[k];
        while (mk) {
            const int bit = __ffs(mk) - 1;
            mk &= mk - 1;
            line_end[off++] = base + k * 4 + (bit >> 3);
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
// Returns false on a NumberFormatException.
template <typename Src>
__device__ __forceinline__ bool java_parse_double(const Src b, int64_t s, int64_t e, double &out) {
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
            v = ex >= 0 ? wd * kP10[ex] : wd / kP10[-ex];
        } else {
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
            if (pending_empty > 0 || !java_parse_double(b, fs, q, v)) bad = true;
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


__global__ __launch_bounds__(kCsvThreads) void k_csv_parse(const uint8_t *__restrict__ text, int64_t nbytes,
                                                           const int64_t *__restrict__ line_end, int64_t nl,
                                                           int64_t nrec, int D, int64_t *__restrict__ ids,
                                                           double *__restrict__ vals, uint8_t *__restrict__ status,
                                                           unsigned long long *__restrict__ counts) {
    __shared__ uint32_t s_buf[kCsvLds / 4];
    __shared__ uint32_t s_cnt[4];
    const int64_t r0 = (int64_t)blockIdx.x * kCsvThreads;
    const int64_t rl = r0 + kCsvThreads - 1 < nrec ? r0 + kCsvThreads - 1 : nrec - 1;
    const int64_t span_s = r0 == 0 ? 0 : line_end[r0 - 1] + 1;
    const int64_t span_e = rl < nl ? line_end[rl] : nbytes;
    const int64_t a0 = span_s & ~3ll;
    const bool staged = span_e - a0 <= kCsvLds;
    if (threadIdx.x < 4) s_cnt[threadIdx.x] = 0;
    if (staged) {
        const int nw = (int)((span_e - a0 + 3) >> 2);
        const bool aligned = ((uintptr_t)text & 3) == 0;
        for (int i = threadIdx.x; i < nw; i += kCsvThreads) {
            const int64_t o = a0 + 4 * (int64_t)i;
            uint32_t x;
            if (aligned && o + 4 <= nbytes) {
                x = *reinterpret_cast<const uint32_t *>(text + o);
            } else {
                x = 0;
                for (int k = 0; k < 4; k++)
                    if (o + k < nbytes) x |= (uint32_t)text[o + k] << (8 * k);
            }
            s_buf[i] = x;
        }
    }
    __syncthreads();
    const int64_t r = r0 + threadIdx.x;
    uint8_t st = SKY_CSV_OK;
    if (r < nrec) {
        const int64_t s = r == 0 ? 0 : line_end[r - 1] + 1;
        const int64_t e = r < nl ? line_end[r] : nbytes;
        int64_t id = 0;
        double *row = vals + r * D;
        if (staged) st = parse_record(LdsSrc{reinterpret_cast<const uint8_t *>(s_buf), a0}, s, e, D, id, row);
        else st = parse_record(GlbSrc{text, 0}, s, e, D, id, row);
        ids[r] = id;
        status[r] = st;
        if (st != SKY_CSV_OK) atomicAdd(&s_cnt[st], 1u);
    }
    __syncthreads();
    if (threadIdx.x >= 1 && threadIdx.x < 4 && s_cnt[threadIdx.x])
        atomicAdd(&counts[threadIdx.x], (unsigned long long)s_cnt[threadIdx.x]);
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

void launch_csv_nl_count(const uint8_t *text, int64_t nbytes, uint32_t *blk_cnt, hipStream_t st) {
    const int64_t nb = csv_chunks(nbytes);
    if (nb == 0) return;
    const bool aligned = ((uintptr_t)text & 15) == 0;
    k_csv_nl_count<<<(unsigned)nb, kCsvThreads, 0, st>>>(text, nbytes, aligned, blk_cnt);
}
void launch_csv_nl_write(const uint8_t *text, int64_t nbytes, const uint32_t *blk_off, int64_t *line_end,
                         hipStream_t st) {
    const int64_t nb = csv_chunks(nbytes);
    if (nb == 0) return;
    const bool aligned = ((uintptr_t)text & 15) == 0;
    k_csv_nl_write<<<(unsigned)nb, kCsvThreads, 0, st>>>(text, nbytes, aligned, blk_off, line_end);
}
void launch_csv_parse(const uint8_t *text, int64_t nbytes, const int64_t *line_end, int64_t nl, int64_t nrec, int D,
                      int64_t *ids, double *vals, uint8_t *status, unsigned long long *counts, hipStream_t st) {
    if (nrec == 0) return;
    const int64_t nb = (nrec + kCsvThreads - 1) / kCsvThreads;
    k_csv_parse<<<(unsigned)nb, kCsvThreads, 0, st>>>(text, nbytes, line_end, nl, nrec, D, ids, vals, status, counts);
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
