// stream_probe2.hip — HBM read rate of candidate load shapes for k_filter's 64-byte rows
// (100M 8D f64 rows, 6.4 GB), on the box at hand:
//   rows      one row per lane, 4 x 16 B loads at a 64 B lane stride (k_filter today),
//             next row in flight while the current one is consumed
//   coal      16 B per lane, lane-contiguous (1 KB per wave instruction), no row view
//   coal_lds  coalesced 16 B loads of a wave's 64 rows (4 KB), through a swizzled LDS
//             image, read back one row per lane (what a row-per-lane consumer needs)
// Each kernel folds what it loaded into a never-taken store so the loads stay live.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kThreads = 256, kItems = 8, kTile = kThreads * kItems;

__global__ __launch_bounds__(kThreads) void k_rows(const double2 *__restrict__ p, uint32_t n, double *out) {
    double acc = 0;
    const uint32_t base = blockIdx.x * kTile;
    const uint32_t nl = n - 1;
    double2 c[4];
    {
        const double2 *q = p + (size_t)min(base + threadIdx.x, nl) * 4;
        c[0] = q[0]; c[1] = q[1]; c[2] = q[2]; c[3] = q[3];
    }
#pragma unroll 1
    for (int r = 0; r < kItems; r++) {
        double2 v[4] = {c[0], c[1], c[2], c[3]};
        const uint32_t nx = min(base + (r + 1) * kThreads + threadIdx.x, nl);
        const double2 *q = p + (size_t)nx * 4;
        c[0] = q[0]; c[1] = q[1]; c[2] = q[2]; c[3] = q[3];
        acc += v[0].x + v[0].y + v[1].x + v[1].y + v[2].x + v[2].y + v[3].x + v[3].y;
    }
    if (acc == 1234.5) out[0] = acc;
}

__global__ __launch_bounds__(kThreads) void k_coal(const double2 *__restrict__ p, uint32_t n, double *out) {
    double acc = 0;
    const size_t base = (size_t)blockIdx.x * kTile * 4;    // double2 units
    const size_t lim = (size_t)n * 4;
#pragma unroll 4
    for (int r = 0; r < kItems * 4; r++) {
        const size_t j = base + (size_t)r * kThreads + threadIdx.x;
        if (j < lim) {
            const double2 a = p[j];
            acc += a.x + a.y;
        }
    }
    if (acc == 1234.5) out[0] = acc;
}

// wave w of the workgroup owns rows [base + 64 * (4 r + w), +64) in step r: four 1 KB
// lane-contiguous loads, written to LDS with the 16 B chunk index XOR-ed by (row / 4) % 4
// so the row-per-lane reads (64 B lane stride) spread over the banks
__global__ __launch_bounds__(kThreads) void k_coal_lds(const double2 *__restrict__ p, uint32_t n, double *out) {
    __shared__ double2 s[kThreads / 64][2][64 * 4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t base = blockIdx.x * kTile;
    const size_t lim = (size_t)n * 4;
    double acc = 0;
    double2 c[4];
    auto fetch = [&](int r) {
        const size_t row0 = (size_t)base + (size_t)64 * (4 * r + w);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const size_t j = row0 * 4 + (size_t)k * 64 + lane;
            c[k] = j < lim ? p[j] : make_double2(0, 0);
        }
    };
    fetch(0);
#pragma unroll 1
    for (int r = 0; r < kItems; r++) {
        double2 *buf = s[w][r & 1];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int e = k * 64 + lane;           // 16 B chunk e: row e / 4, quarter e % 4
            const int row = e >> 2, q = e & 3;
            buf[row * 4 + (q ^ ((row >> 2) & 3))] = c[k];
        }
        if (r + 1 < kItems) fetch(r + 1);
        __builtin_amdgcn_s_waitcnt(0xc07f);        // lgkmcnt(0): this wave's LDS writes done
        __builtin_amdgcn_wave_barrier();
        double2 v[4];
#pragma unroll
        for (int q = 0; q < 4; q++) v[q] = buf[lane * 4 + (q ^ ((lane >> 2) & 3))];
        acc += v[0].x + v[0].y + v[1].x + v[1].y + v[2].x + v[2].y + v[3].x + v[3].y;
    }
    if (acc == 1234.5) out[0] = acc;
}

int main() {
    const uint32_t n = 100000000;
    double2 *p;
    double *o;
    if (hipMalloc(&p, (size_t)n * 64) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) return 1;
    (void)hipMemset(p, 0, (size_t)n * 64);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const unsigned g = (n + kTile - 1) / kTile;
    const char *names[3] = {"rows", "coal", "coal_lds"};
    for (int rep = 0; rep < 2; rep++) {
        for (int v = 0; v < 3; v++) {
            for (int w = 0; w < 2; w++) {
                if (v == 0) k_rows<<<g, kThreads>>>(p, n, o);
                else if (v == 1) k_coal<<<g, kThreads>>>(p, n, o);
                else k_coal_lds<<<g, kThreads>>>(p, n, o);
            }
            (void)hipEventRecord(a);
            for (int w = 0; w < 10; w++) {
                if (v == 0) k_rows<<<g, kThreads>>>(p, n, o);
                else if (v == 1) k_coal<<<g, kThreads>>>(p, n, o);
                else k_coal_lds<<<g, kThreads>>>(p, n, o);
            }
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            ms /= 10;
            printf("%-9s %.4f ms  %.0f GB/s\n", names[v], ms, (double)n * 64 / ms / 1e6);
        }
    }
    return hipGetLastError() == hipSuccess ? 0 : 2;
}
