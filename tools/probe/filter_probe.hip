// filter_probe.hip — does LDS-DMA prefetch (global_load_lds_dwordx4, several items deep) keep
// k_filter's 64-byte row stream busier than the one-row register prefetch, once each row also
// carries VALU work?  100M 8D f64 rows (6.4 GB), W dependent f64 ops per row (k_filter's key and
// pruner tests are ~100-200), one status word stored per row.
//   reg       one row per lane in flight in registers (k_filter's scheme)
//   lds<P>    P items in flight per wave through LDS (16 KB per item per 256-thread workgroup)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

constexpr int kThreads = 256, kItems = 24;   // a multiple of 3 and of 4

__device__ __forceinline__ uint16_t work(const double (&v)[8], int W) {
    double a = v[0], b = v[1];
#pragma unroll 1
    for (int i = 0; i < W; i++) {
        a = a * 1.0000001 + v[i & 7];
        b = b * 0.9999999 - a;
    }
    return (uint16_t)(a + b > 1e300 ? 1 : 0) | (uint16_t)(v[2] + v[3] + v[4] + v[5] + v[6] + v[7] > 1e300 ? 2 : 0);
}

__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(6))) void k_reg(const double *__restrict__ p, uint32_t n, int W,
                                                               uint16_t *__restrict__ st) {
    const uint32_t nl = n - 1;
    double vn[8];
    auto fetch = [&](uint32_t i) {
        const double2 *q = reinterpret_cast<const double2 *>(p + (size_t)min(i, nl) * 8);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const double2 x = q[k];
            vn[2 * k] = x.x;
            vn[2 * k + 1] = x.y;
        }
    };
    const uint32_t base = blockIdx.x * kThreads * kItems;
    fetch(base + threadIdx.x);
#pragma unroll 1
    for (int r = 0; r < kItems; r++) {
        const uint32_t i = base + r * kThreads + threadIdx.x;
        double v[8];
#pragma unroll
        for (int d = 0; d < 8; d++) v[d] = vn[d];
        fetch(i + kThreads);
        const uint16_t s = work(v, W);
        if (i < n) st[i] = s;
    }
}

// reg, but the status words of 8 items staged per wave in LDS and written as one 16-byte store
// per lane every 8 items (gfx9 counts stores in vmcnt: a short store per item sits in front of
// the next prefetch's wait)
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(6))) void k_reg_st8(const double *__restrict__ p, uint32_t n, int W,
                                                                   uint16_t *__restrict__ st) {
    __shared__ uint16_t s_st[kThreads / 64][8][64];
    const uint32_t nl = n - 1;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double vn[8];
    auto fetch = [&](uint32_t i) {
        const double2 *q = reinterpret_cast<const double2 *>(p + (size_t)min(i, nl) * 8);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const double2 x = q[k];
            vn[2 * k] = x.x;
            vn[2 * k + 1] = x.y;
        }
    };
    const uint32_t base = blockIdx.x * kThreads * kItems;
    fetch(base + threadIdx.x);
#pragma unroll 1
    for (int r0 = 0; r0 < kItems; r0 += 8) {
#pragma unroll
        for (int r = r0; r < r0 + 8; r++) {
            const uint32_t i = base + r * kThreads + threadIdx.x;
            double v[8];
#pragma unroll
            for (int d = 0; d < 8; d++) v[d] = vn[d];
            fetch(i + kThreads);
            s_st[w][r - r0][lane] = work(v, W);
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);        // lgkmcnt(0)
        __builtin_amdgcn_wave_barrier();
        // segment g = item r0 + g: rows base + (r0 + g) * 256 + 64 w .. + 64, 128 bytes
        const int g = lane >> 3, part = lane & 7;
        const uint4 x = reinterpret_cast<const uint4 *>(&s_st[w][g][0])[part];
        const uint32_t row0 = base + (r0 + g) * kThreads + 64 * w + 8 * part;
        if (row0 + 8 <= n) *reinterpret_cast<uint4 *>(st + row0) = x;
        __builtin_amdgcn_wave_barrier();
    }
}

// the box's stream ceilings for the same bytes: rows read one per lane (no work, no store), and
// 16 B per lane lane-contiguous (1 KB per wave instruction)
__global__ __launch_bounds__(kThreads) void k_rows_only(const double *__restrict__ p, uint32_t n, double *out) {
    const uint32_t nl = n - 1;
    const uint32_t base = blockIdx.x * kThreads * kItems;
    double acc = 0;
#pragma unroll 4
    for (int r = 0; r < kItems; r++) {
        const double2 *q = reinterpret_cast<const double2 *>(p + (size_t)min(base + r * kThreads + threadIdx.x, nl) * 8);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const double2 x = q[k];
            acc += x.x + x.y;
        }
    }
    if (acc == 1234.5) out[0] = acc;
}
__global__ __launch_bounds__(kThreads) void k_coal_only(const double2 *__restrict__ p, uint32_t n, double *out) {
    const size_t base = (size_t)blockIdx.x * kThreads * kItems * 4;    // double2 units
    const size_t lim = (size_t)n * 4;
    double acc = 0;
#pragma unroll 4
    for (int r = 0; r < kItems * 4; r++) {
        const size_t j = min(base + (size_t)r * kThreads + threadIdx.x, lim - 1);
        const double2 a = p[j];
        acc += a.x + a.y;
    }
    if (acc == 1234.5) out[0] = acc;
}
// coalesced 1 KB wave loads (lane-contiguous 16 B), transposed through a swizzled LDS image into
// one row per lane, W work and the status store per row (a register-staged k_filter shape)
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(6))) void k_coal_lds(const double *__restrict__ p, uint32_t n, int W,
                                                                    uint16_t *__restrict__ st) {
    __shared__ double2 s[kThreads / 64][64 * 4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t base = blockIdx.x * kThreads * kItems;
    const size_t lim = (size_t)n * 4;
    const double2 *p2 = reinterpret_cast<const double2 *>(p);
    double2 c[4];
    auto fetch = [&](int r) {          // wave w's 64 rows of item r: rows base + r*256 + 64w ..
        const size_t row0 = (size_t)base + (size_t)r * kThreads + 64 * w;
#pragma unroll
        for (int k = 0; k < 4; k++) c[k] = p2[min(row0 * 4 + (size_t)k * 64 + lane, lim - 1)];
    };
    fetch(0);
#pragma unroll 1
    for (int r = 0; r < kItems; r++) {
        double2 *buf = s[w];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int e = k * 64 + lane, row = e >> 2, q = e & 3;
            buf[row * 4 + (q ^ ((row >> 2) & 3))] = c[k];
        }
        if (r + 1 < kItems) fetch(r + 1);
        __builtin_amdgcn_s_waitcnt(0xc07f);        // lgkmcnt(0)
        __builtin_amdgcn_wave_barrier();
        double v[8];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const double2 x = buf[lane * 4 + (q ^ ((lane >> 2) & 3))];
            v[2 * q] = x.x;
            v[2 * q + 1] = x.y;
        }
        __builtin_amdgcn_wave_barrier();
        const uint16_t sv = work(v, W);
        const uint32_t i = base + r * kThreads + 64 * w + lane;
        if (i < n) st[i] = sv;
    }
}

// waitcnt immediates (gfx9 encoding): vmcnt(N) only, N < 64
#define VMCNT(N) (0x3f70 | ((N) & 15) | (((N) >> 4) << 14))

// P items in flight: P separate LDS arrays used round-robin with the loop unrolled by P, so every
// access names its array statically (the compiler then keeps the explicit vmcnt(4 (P - 1)) instead
// of waiting for every LDS-DMA load before each LDS read)
template <int P>
__global__ __launch_bounds__(kThreads) void k_lds(const double *__restrict__ p, uint32_t n, int W, uint16_t *__restrict__ st) {
    __shared__ __attribute__((aligned(16))) double2 b0[4][kThreads], b1[4][kThreads], b2[4][kThreads], b3[4][kThreads];
    const uint32_t nl = n - 1;
    const int t = threadIdx.x;
    const uint32_t base = blockIdx.x * kThreads * kItems;
    auto issue = [&](double2 (*buf)[kThreads], int r) {
        const double *g = p + (size_t)min(base + min(r, kItems - 1) * kThreads + t, nl) * 8;
#pragma unroll
        for (int q = 0; q < 4; q++)
            __builtin_amdgcn_global_load_lds(g + 2 * q, (__attribute__((address_space(3))) void *)&buf[q][t & ~63], 16,
                                             0, 0);
    };
    auto use = [&](double2 (*buf)[kThreads], int r) {
        __builtin_amdgcn_s_waitcnt(VMCNT(4 * (P - 1)));
        double v[8];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const double2 x = buf[q][t];
            v[2 * q] = x.x;
            v[2 * q + 1] = x.y;
        }
        const uint16_t s = work(v, W);
        const uint32_t i = base + r * kThreads + t;
        if (r < kItems && i < n) st[i] = s;
    };
    if constexpr (P == 3) {
        issue(b0, 0);
        issue(b1, 1);
#pragma unroll 1
        for (int r = 0; r < kItems; r += 3) {
            issue(b2, r + 2); use(b0, r);
            issue(b0, r + 3); use(b1, r + 1);
            issue(b1, r + 4); use(b2, r + 2);
        }
    } else {
        issue(b0, 0);
        issue(b1, 1);
        issue(b2, 2);
#pragma unroll 1
        for (int r = 0; r < kItems; r += 4) {
            issue(b3, r + 3); use(b0, r);
            issue(b0, r + 4); use(b1, r + 1);
            issue(b1, r + 5); use(b2, r + 2);
            issue(b2, r + 6); use(b3, r + 3);
        }
    }
}

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atol(argv[1]) : 100000000u;
    double *p;
    uint16_t *st;
    hipMalloc(&p, (size_t)n * 64);
    hipMalloc(&st, (size_t)n * 2);
    hipMemset(p, 0, (size_t)n * 64);
    const unsigned g = (n + kThreads * kItems - 1) / (kThreads * kItems);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    double *out;
    hipMalloc(&out, 64);
    {
        auto run0 = [&](const char *name, auto launch, double bytes) {
            launch();
            hipEventRecord(a);
            for (int k = 0; k < 5; k++) launch();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            ms /= 5;
            printf("read-only %-10s %.3f ms  %.2f TB/s\n", name, ms, bytes / (ms * 1e-3) / 1e12);
        };
        run0("rows", [&] { k_rows_only<<<g, kThreads>>>(p, n, out); }, (double)n * 64);
        run0("coalesced", [&] { k_coal_only<<<g, kThreads>>>(reinterpret_cast<const double2 *>(p), n, out); },
             (double)n * 64);
    }
    for (int W : {0, 16, 48, 96}) {
        auto run = [&](const char *name, auto launch) {
            launch();
            hipEventRecord(a);
            for (int k = 0; k < 5; k++) launch();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            ms /= 5;
            printf("W=%3d %-6s %.3f ms  %.2f TB/s\n", W, name, ms, (double)n * 66 / (ms * 1e-3) / 1e12);
        };
        run("reg", [&] { k_reg<<<g, kThreads>>>(p, n, W, st); });
        run("reg+st8", [&] { k_reg_st8<<<g, kThreads>>>(p, n, W, st); });
        run("coal+lds", [&] { k_coal_lds<<<g, kThreads>>>(p, n, W, st); });
        run("lds3", [&] { k_lds<3><<<g, kThreads>>>(p, n, W, st); });
        run("lds4", [&] { k_lds<4><<<g, kThreads>>>(p, n, W, st); });
    }
    if (hipDeviceSynchronize() != hipSuccess) { printf("error\n"); return 1; }
    return 0;
}
