// stream_probe.hip — HBM read rate of the k_filter access pattern (row per lane,
// 4 x 16 B loads per 64 B row) vs fully coalesced 16 B-per-lane wave loads, over a
// 6.4 GB buffer (100M 8D f64 rows), to separate access-pattern cost from compute.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(256) void k_rows(const double2 *__restrict__ p, uint32_t n, double *out) {
    double acc = 0;
    const uint32_t base = blockIdx.x * 2048;
    for (int r = 0; r < 8; r++) {
        const uint32_t i = base + r * 256 + threadIdx.x;
        if (i < n) {
            const double2 *q = p + (size_t)i * 4;
            double2 a = q[0], b = q[1], c = q[2], d = q[3];
            acc += a.x + a.y + b.x + b.y + c.x + c.y + d.x + d.y;
        }
    }
    if (acc == 1234.5) out[0] = acc;
}

__global__ __launch_bounds__(256) void k_coal(const double2 *__restrict__ p, uint32_t n, double *out) {
    double acc = 0;
    const size_t base = (size_t)blockIdx.x * 2048 * 4;    // in double2 units
    for (int r = 0; r < 32; r++) {
        const size_t j = base + (size_t)r * 256 + threadIdx.x;
        if (j < (size_t)n * 4) {
            const double2 a = p[j];
            acc += a.x + a.y;
        }
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
    const unsigned g = (n + 2047) / 2048;
    for (int v = 0; v < 2; v++) {
        for (int w = 0; w < 2; w++) {
            if (v) k_coal<<<g, 256>>>(p, n, o);
            else k_rows<<<g, 256>>>(p, n, o);
        }
        (void)hipEventRecord(a);
        for (int it = 0; it < 5; it++) {
            if (v) k_coal<<<g, 256>>>(p, n, o);
            else k_rows<<<g, 256>>>(p, n, o);
        }
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        printf("%s: %.3f ms  %.0f GB/s\n", v ? "coalesced" : "row-per-lane", ms / 5,
               (double)n * 64 / (ms / 5 * 1e-3) / 1e9);
    }
    return 0;
}
