// k_synth.hip — synthetic tuple streams generated directly in HBM.
//
// Restates the reference producer's three distributions
// (/root/reference/python/unified_producer.py:50-123) with a counter-based RNG
// (splitmix64 finaliser keyed by (seed, tuple id, draw)) in place of Python's
// unseeded Mersenne Twister, so any tuple can be generated independently by any
// thread and re-generated bit-identically by the host copy (sky_synth) and by the
// test oracle (oracle/skyline_oracle.c:orc_synth).  Two labelled extensions:
// SKY_DIST_STD_ANTI (a Borzsonyi-style anti-correlated band whose skyline has many
// distinct vectors) and SKY_DIST_MIXED (65536-tuple blocks cycling the three
// reference distributions, for the mixed-stream config).
#include "sky_internal.h"

namespace sky {

__host__ __device__ __forceinline__ uint64_t synth_mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ double synth_rnd(uint64_t seedmix, uint64_t i, uint32_t j) {
    const uint64_t h = synth_mix64(seedmix ^ (i * 0xD1B54A32D192ED03ull) ^ ((uint64_t)j * 0x8CB92BA72F3D8DD7ull));
    return (double)(h >> 11) * (1.0 / 9007199254740992.0);
}
__host__ __device__ __forceinline__ double synth_clamp_trunc(double v, int dmin, int dmax) {
    int64_t t = (int64_t)v;
    t = t > dmax ? dmax : t;
    t = t < dmin ? dmin : t;
    return (double)t;
}
__host__ __device__ __forceinline__ double synth_eps(int D) {
    if (D == 2) return 0.0005;
    if (D == 3) return 0.05;
    if (D == 4) return 0.9;
    return (double)D * 0.005 * 100;
}

template <int D>
__host__ __device__ __forceinline__ void synth_row(int dist, int dmin, int dmax, uint64_t sm, uint64_t i, double *v) {
    int dd = dist;
    if (dist == SKY_DIST_MIXED) dd = (int)((i >> 16) % 3);
    if (dd == SKY_DIST_UNIFORM) {
        const double range = (double)(dmax - dmin + 1);
        for (int d = 0; d < D; d++) v[d] = (double)(dmin + (int64_t)floor(synth_rnd(sm, i, d) * range));
    } else if (dd == SKY_DIST_CORRELATED) {
        const double a = (double)dmin, b = (double)dmax;
        const double base = a + (b - a) * synth_rnd(sm, i, 0);
        const double lo = -(1 - 0.9) * (double)(dmax - dmin);
        const double hi = +(1 - 0.9) * (double)(dmax - dmin);
        for (int d = 0; d < D; d++) {
            const double noise = lo + (hi - lo) * synth_rnd(sm, i, 1 + d);
            v[d] = synth_clamp_trunc(base + noise, dmin, dmax);
        }
    } else if (dd == SKY_DIST_ANTI) {
        const double eps = synth_eps(D);
        double total = 0.0;
        for (int d = 0; d < D; d++) { v[d] = synth_rnd(sm, i, d); total = total + v[d]; }
        const double mean = (double)(dmin + dmax) / 2.0 * D;
        const double slack = eps * (double)(dmax - dmin) * D;
        const double lo = mean - slack, hi = mean + slack;
        const double target = lo + (hi - lo) * synth_rnd(sm, i, 32);
        const double scale = total != 0 ? target / total : 1.0;
        for (int d = 0; d < D; d++) v[d] = synth_clamp_trunc(v[d] * scale, dmin, dmax);
    } else {
        const double c = 0.5 + 0.05 * ((synth_rnd(sm, i, 40) + synth_rnd(sm, i, 41) + synth_rnd(sm, i, 42) +
                                        synth_rnd(sm, i, 43)) - 2.0);
        bool ok = false;
        for (uint32_t att = 0; att < 8 && !ok; att++) {
            double mean = 0.0;
            for (int d = 0; d < D; d++) { v[d] = synth_rnd(sm, i, 64 + att * 32 + d); mean = mean + v[d]; }
            mean = mean / D;
            ok = true;
            for (int d = 0; d < D; d++) {
                v[d] = v[d] + (c - mean);
                if (v[d] < 0.0 || v[d] >= 1.0) ok = false;
            }
        }
        const double range = (double)(dmax - dmin);
        for (int d = 0; d < D; d++) {
            const double x = v[d] < 0.0 ? 0.0 : (v[d] >= 1.0 ? 0.9999999999999999 : v[d]);
            v[d] = (double)(dmin + (int64_t)floor(x * range));
        }
    }
}

template <int D>
__global__ __launch_bounds__(kThreads) void k_synth(int dist, int dmin, int dmax, uint64_t sm, int64_t id0,
                                                    int64_t n, double *__restrict__ vals,
                                                    int64_t *__restrict__ ids) {
    for (int64_t r = (int64_t)blockIdx.x * kThreads + threadIdx.x; r < n; r += (int64_t)gridDim.x * kThreads) {
        double v[D];
        synth_row<D>(dist, dmin, dmax, sm, (uint64_t)(id0 + r), v);
#pragma unroll
        for (int d = 0; d < D; d++) vals[r * D + d] = v[d];
        if (ids) ids[r] = id0 + r;
    }
}

void launch_synth(int dist, int D, int dmin, int dmax, uint64_t seed, int64_t id0, int64_t n, double *vals,
                  int64_t *ids, hipStream_t st) {
    if (n <= 0) return;
    const uint64_t sm = synth_mix64(seed);
    int64_t g = (n + kThreads - 1) / kThreads;
    if (g > 8192) g = 8192;
    SKY_DISPATCH_D(D, (k_synth<DD><<<(unsigned)g, kThreads, 0, st>>>(dist, dmin, dmax, sm, id0, n, vals, ids)));
}

void synth_host(int dist, int D, int dmin, int dmax, uint64_t seed, int64_t id0, int64_t n, double *vals,
                int64_t *ids) {
    const uint64_t sm = synth_mix64(seed);
    for (int64_t r = 0; r < n; r++) {
        SKY_DISPATCH_D(D, (synth_row<DD>(dist, dmin, dmax, sm, (uint64_t)(id0 + r), vals + r * D)));
        if (ids) ids[r] = id0 + r;
    }
}

}  // namespace sky
