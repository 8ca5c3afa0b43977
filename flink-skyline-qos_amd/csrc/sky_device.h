// sky_device.h — device-side building blocks shared by the gfx950 kernels.
//
// * Java narrowing (int) of a double (JLS 5.1.3)
// * fdlibm 5.3 atan / atan2 (what java.lang.Math.atan2 delegates to in JDK 11)
// * the three partitioner key functions, bit-exact with
//   /root/reference/java/org.main/FlinkSkyline.java (Dim :707-712, Grid :774-789,
//   Angle :827-875).  Built with -ffp-contract=off: Java never fuses a*b+c.
// * dominance (ServiceTuple.java:67-77)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "sky_common.h"

namespace sky {

__device__ __forceinline__ int32_t java_d2i(double x) {
    if (x != x) return 0;
    if (x >= 2147483647.0) return 2147483647;
    if (x <= -2147483648.0) return INT32_MIN;
    return (int32_t)x;
}

// ---- fdlibm s_atan.c / e_atan2.c ------------------------------------------
__device__ __forceinline__ double fd_atan(double x) {
    constexpr double hi0 = 4.63647609000806093515e-01, hi1 = 7.85398163397448278999e-01,
                     hi2 = 9.82793723247329054082e-01, hi3 = 1.57079632679489655800e+00;
    constexpr double lo0 = 2.26987774529616870924e-17, lo1 = 3.06161699786838301793e-17,
                     lo2 = 1.39033110312309984516e-17, lo3 = 6.12323399573676603587e-17;
    constexpr double a0 = 3.33333333333329318027e-01, a1 = -1.99999999998764832476e-01,
                     a2 = 1.42857142725034663711e-01, a3 = -1.11111104054623557880e-01,
                     a4 = 9.09088713343650656196e-02, a5 = -7.69187620504482999495e-02,
                     a6 = 6.66107313738753120669e-02, a7 = -5.83357013379057348645e-02,
                     a8 = 4.97687799461593236017e-02, a9 = -3.65315727442169155270e-02,
                     a10 = 1.62858201153657823623e-02;
    const int32_t hx = __double2hiint(x);
    const int32_t ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x44100000) {                              // |x| >= 2^66
        if (ix > 0x7ff00000 || (ix == 0x7ff00000 && __double2loint(x) != 0)) return x + x;
        return hx > 0 ? hi3 + lo3 : -hi3 - lo3;
    }
    if (ix < 0x3fdc0000) {                               // |x| < 0.4375
        if (ix < 0x3e200000) return x;                   // |x| < 2^-29 (inexact flag ignored)
        id = -1;
    } else {
        x = fabs(x);
        if (ix < 0x3ff30000) {
            if (ix < 0x3fe60000) { id = 0; x = (2.0 * x - 1.0) / (2.0 + x); }
            else                 { id = 1; x = (x - 1.0) / (x + 1.0); }
        } else {
            if (ix < 0x40038000) { id = 2; x = (x - 1.5) / (1.0 + 1.5 * x); }
            else                 { id = 3; x = -1.0 / x; }
        }
    }
    const double z = x * x;
    const double w = z * z;
    const double s1 = z * (a0 + w * (a2 + w * (a4 + w * (a6 + w * (a8 + w * a10)))));
    const double s2 = w * (a1 + w * (a3 + w * (a5 + w * (a7 + w * a9))));
    if (id < 0) return x - x * (s1 + s2);
    const double hi = id == 0 ? hi0 : id == 1 ? hi1 : id == 2 ? hi2 : hi3;
    const double lo = id == 0 ? lo0 : id == 1 ? lo1 : id == 2 ? lo2 : lo3;
    const double r = hi - ((x * (s1 + s2) - lo) - x);
    return hx < 0 ? -r : r;
}

__device__ __forceinline__ double fd_atan2(double y, double x) {
    constexpr double tiny = 1.0e-300;
    constexpr double pi_o_4 = 7.8539816339744827900E-01, pi_o_2 = 1.5707963267948965580E+00,
                     pi = 3.1415926535897931160E+00, pi_lo = 1.2246467991473531772E-16;
    const int32_t hx = __double2hiint(x), ix = hx & 0x7fffffff;
    const uint32_t lx = (uint32_t)__double2loint(x);
    const int32_t hy = __double2hiint(y), iy = hy & 0x7fffffff;
    const uint32_t ly = (uint32_t)__double2loint(y);
    if (((uint32_t)ix | ((lx | (0u - lx)) >> 31)) > 0x7ff00000u ||
        ((uint32_t)iy | ((ly | (0u - ly)) >> 31)) > 0x7ff00000u)
        return x + y;
    if (((hx - 0x3ff00000) | (int32_t)lx) == 0) return fd_atan(y);
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if ((iy | (int32_t)ly) == 0) {
        if (m <= 1) return y;
        return m == 2 ? pi + tiny : -pi - tiny;
    }
    if ((ix | (int32_t)lx) == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7ff00000) {
        if (iy == 0x7ff00000) {
            switch (m) {
                case 0: return pi_o_4 + tiny;
                case 1: return -pi_o_4 - tiny;
                case 2: return 3.0 * pi_o_4 + tiny;
                default: return -3.0 * pi_o_4 - tiny;
            }
        }
        switch (m) {
            case 0: return 0.0;
            case 1: return -0.0;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (iy == 0x7ff00000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int k = (iy - ix) >> 20;
    double z;
    if (k > 60) z = pi_o_2 + 0.5 * pi_lo;               // original fdlibm (JDK): no m &= 1
    else if (hx < 0 && k < -60) z = 0.0;
    else z = fd_atan(fabs(y / x));
    switch (m) {
        case 0: return z;
        case 1: return -z;
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

// ---- partition keys ----------------------------------------------------------
struct KeyParams {
    int algo;          // SKY_ALGO_*
    int P;             // partitions
    int K;             // queried key space: keys >= K are dropped (reference MR-Grid)
    double dim_width;  // maxVal / partitions  (:710)
    double grid_mid;   // maxVal / 2.0          (:756)
    double margin;     // MR-Angle fast path: distance of avg*P from an integer that is certain
    int grid_filter;   // MR-Grid dominance filter (FlinkSkyline.java:716-733, disabled in the reference):
                       // tuples with every value >= maxVal/2 get key -1 (removed before keyBy)
    // the fast path's f32 constants, converted once on the host (kernel arguments stay in
    // SGPRs; converted in the kernel they were VGPRs live across the whole stream loop)
    float ang_scale;   // (2/pi) / (D-1) * P
    float ang_lo, ang_hi;   // margin, 1 - margin
    // the special case's key for each exact normalized sum c in 0..2(D-1): byte c % 8 of
    // ang_special[c / 8] = clamp(d2i(c / (D-1) * P)), the reference's f64 ops done on the host
    uint64_t ang_special0, ang_special1, ang_special2, ang_special3;
};

// Error budget of the f32 estimate in t = avg*P (inputs with nonzero magnitudes in
// [1e-15, 1e15], so no f32 square over- or underflows):
//   * inputs and the f32 FMA sum of <= 15 squares: relative <= 1.1e-6; v_sqrt_f32
//     (1 ulp) -> hyp relative <= 7e-7; the ratio a = min/max via v_rcp_f32 (1 ulp)
//     -> relative <= 1e-6 -> angle error <= 1e-6 rad (d atan(a) <= da);
//   * atan on [0,1] by the 7-term odd polynomial atan_poly: <= 2.5e-7 rad, plus f32
//     evaluation and the pi/2 - r, pi - r reflections: <= 1e-6 rad;
//   so <= 2.2e-6 rad per angle; the f32 sum of <= 15 angles (each partial <= 15 pi)
//   adds <= 14 x 1.9e-6 rad; t = sum * (2/pi)/(D-1) * P then errs by <= 2.5e-6 * P
//   for every D in [2,16] (plus 1e-6 for the f32 scale).
// The margin 1e-5 + 8e-6*P keeps a >= 3x safety factor; the exact fdlibm fallback
// runs whenever t_est is closer than that to an integer.
inline double angle_margin(int P) { return 1e-5 + 8e-6 * (double)P; }

// atan(a) for a in [0,1]: a * poly(a^2), 7 terms, |error| <= 2.5e-7 (Lawson-refined
// least squares on Chebyshev nodes; the constants are what the bound was measured for)
__device__ __forceinline__ float atan_poly01(float a) {
    const float z = a * a;
    float p = 0.006811792604364258f;
    p = fmaf(p, z, -0.03360421913563544f);
    p = fmaf(p, z, 0.07962367186607752f);
    p = fmaf(p, z, -0.1323334216932318f);
    p = fmaf(p, z, 0.19807815630001427f);
    p = fmaf(p, z, -0.33317368071637243f);
    p = fmaf(p, z, 0.999996111561908f);
    return a * p;
}

// estimate of atan2(h, x) for h >= 0 (the reference's hyp): first-quadrant
// polynomial, then reflections; atan2(+0, -0) = pi and atan2(h>0, -0) = pi/2 as Java
__device__ __forceinline__ float atan2_est(float h, float x) {
    const float ax = fabsf(x);
    const float mn = fminf(h, ax), mx = fmaxf(h, ax);
    // mx == 0 means mn == 0: 0 * rcp(1e-30) = 0 without a compare/select (every mx > 0
    // the callers pass is >= 1e-15, so the max does not change it); rcp rounding can
    // push mn/mx past 1, clamped by one min (a is never NaN here)
    const float a = fminf(mn * __builtin_amdgcn_rcpf(fmaxf(mx, 1e-30f)), 1.0f);
    float r = atan_poly01(a);
    r = h > ax ? 1.57079632679489662f - r : r;
    return signbit(x) ? 3.14159265358979324f - r : r;
}

__device__ __forceinline__ int32_t clamp_key(int32_t p, int P) {
    p = p > P - 1 ? P - 1 : p;
    return p < 0 ? 0 : p;
}

// The reference's AnglePartitioner.getKey, operation for operation in f64.
template <int D>
__device__ __forceinline__ int32_t angle_key_exact(const double (&v)[D], int P) {
    constexpr double max_angle = 3.141592653589793 / 2.0;
    double normalized = 0.0;
    for (int i = 0; i < D - 1; i++) {
        double s = 0.0;
        for (int j = i + 1; j < D; j++) s = s + v[j] * v[j];   // ascending j, no FMA
        const double hyp = sqrt(s);
        normalized = normalized + fd_atan2(hyp, v[i]) / max_angle;
    }
    const double avg = normalized / (double)(D - 1);
    return clamp_key(java_d2i(avg * (double)P), P);
}

// MR-Angle key with a certified fast path (a "filtered predicate"):
//  1. exact special case: every angle is atan2(+0, x) or atan2(y>0, ±0), i.e. exactly
//     0, pi (x negative/-0) or pi/2 -> normalized 0, 2, 1 exactly; the remaining
//     f64 ops are replayed as the reference does them (all-zero tuples land here);
//  2. f32 estimate of sum(atan2/(pi/2)); if t = avg*P is farther than `margin`
//     (angle_margin) from an integer, floor(t) IS the exact key;
//  3. otherwise the exact fdlibm path (~1e-4 of the reference-formula tuples).

// kAngleUndecided: the fast path could not certify the key (non-ranged input or
// t within `margin` of an integer); the caller runs angle_key_exact.
constexpr int32_t kAngleUndecided = -1;
constexpr int32_t kKeyFiltered = -2;   // removed by the MR-Grid dominance filter (never queried)

template <int D>
__device__ __forceinline__ int32_t angle_key_fast(const double (&v)[D], const KeyParams &kp) {
    if (D < 2) return 0;
    // every value 0 or of magnitude in [1e-15, 1e15] (NaN and inf fail): then no
    // square underflows, so the reference's f64 s_i is 0 exactly when v_j == 0 for
    // every j > i, and f32 holds every s_i without overflow
    bool ranged = true;
    bool iz[D];                                            // v[i] == 0, one compare shared below
#pragma unroll
    for (int i = 0; i < D; i++) {
        const double a = fabs(v[i]);
        iz[i] = v[i] == 0.0;
        ranged &= iz[i] | ((a >= 1e-15) & (a <= 1e15));
    }
    if (ranged) {
        bool zero_after[D > 1 ? D - 1 : 1];
        bool z = true, special = true;
#pragma unroll
        for (int i = D - 2; i >= 0; i--) {
            z &= iz[i + 1];
            zero_after[i] = z;
            special &= z | iz[i];
        }
        if (special) {
            // normalized is the exact integer c = sum of the per-angle 0 / 1 / 2: the key of
            // each c was computed on the host (KeyParams::ang_special*)
            uint32_t c = 0;
#pragma unroll
            for (int i = 0; i < D - 1; i++) c += zero_after[i] ? (signbit(v[i]) ? 2u : 0u) : 1u;
            const uint64_t w = c < 8 ? kp.ang_special0 : c < 16 ? kp.ang_special1 : c < 24 ? kp.ang_special2
                                                                                         : kp.ang_special3;
            return (int32_t)((w >> ((c & 7u) * 8u)) & 0xffu);
        }
        float f[D];
#pragma unroll
        for (int i = 0; i < D; i++) f[i] = (float)v[i];
        float s = 0.0f, est = 0.0f;
#pragma unroll
        for (int i = D - 2; i >= 0; i--) {
            s = fmaf(f[i + 1], f[i + 1], s);
            est += atan2_est(__builtin_amdgcn_sqrtf(s), f[i]);
        }
        const float t = est * kp.ang_scale;
        const float fl = floorf(t);
        const float fr = t - fl;
        if (fr > kp.ang_lo && fr < kp.ang_hi) return clamp_key((int32_t)fl, kp.P);
    }
    return kAngleUndecided;
}

// Dim and Grid keys are exact; the Angle key may be kAngleUndecided.
template <int D>
__device__ __forceinline__ int32_t partition_key_fast(const double (&v)[D], const KeyParams &kp) {
    if (kp.algo == SKY_ALGO_DIM) return clamp_key(java_d2i(v[0] / kp.dim_width), kp.P);
    if (kp.algo == SKY_ALGO_GRID) {
        uint32_t mask = 0;
#pragma unroll
        for (int i = 0; i < D; i++)
            if (v[i] >= kp.grid_mid) mask |= (1u << (i & 31));
        if (kp.grid_filter && mask == (D >= 32 ? ~0u : (1u << D) - 1u)) return kKeyFiltered;
        return (int32_t)mask;
    }
    return angle_key_fast<D>(v, kp);
}

template <int D>
__device__ __forceinline__ int32_t partition_key(const double (&v)[D], const KeyParams &kp) {
    if (kp.algo == SKY_ALGO_DIM) return clamp_key(java_d2i(v[0] / kp.dim_width), kp.P);
    if (kp.algo == SKY_ALGO_GRID) {
        uint32_t mask = 0;
#pragma unroll
        for (int i = 0; i < D; i++)
            if (v[i] >= kp.grid_mid) mask |= (1u << (i & 31));
        if (kp.grid_filter && mask == (D >= 32 ? ~0u : (1u << D) - 1u)) return kKeyFiltered;
        return (int32_t)mask;
    }
    const int32_t k = angle_key_fast<D>(v, kp);
    return k != kAngleUndecided ? k : angle_key_exact<D>(v, kp.P);
}

template <int D>
__device__ __forceinline__ bool any_nan(const double (&v)[D]) {
    bool nan = false;
#pragma unroll
    for (int d = 0; d < D; d++) nan |= v[d] != v[d];
    return nan;
}

// ---- dominance ----------------------------------------------------------------
// a dominates b (ServiceTuple.java:67-77): all a<=b and some a<b.  With NaN-free
// rows the early-exit loop and this branch-free form agree.
template <int D, typename T>
__device__ __forceinline__ bool dominates_full(const T *a, const T *b) {
    bool le = true, lt = false;
#pragma unroll
    for (int d = 0; d < D; d++) { le &= a[d] <= b[d]; lt |= a[d] < b[d]; }
    return le && lt;
}
// For rows known to be DISTINCT vectors (representatives of one partition),
// "all a <= b" already implies some a < b: D compares per pair.
template <int D, typename T>
__device__ __forceinline__ bool dominates_distinct(const T *a, const T *b) {
    bool le = true;
#pragma unroll
    for (int d = 0; d < D; d++) le &= a[d] <= b[d];
    return le;
}
template <int D, typename T>
__device__ __forceinline__ bool rows_equal(const T *a, const T *b) {
    bool eq = true;
#pragma unroll
    for (int d = 0; d < D; d++) eq &= a[d] == b[d];
    return eq;
}

// order-preserving map f32 -> u32 (-0.0 canonicalised to +0.0)
__device__ __forceinline__ uint32_t f32_order_key(float f) {
    uint32_t u = __float_as_uint(f == 0.0f ? 0.0f : f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ uint32_t mix32(uint32_t h) {
    h ^= h >> 16; h *= 0x7feb352du; h ^= h >> 15; h *= 0x846ca68bu; h ^= h >> 16;
    return h;
}

}  // namespace sky
