// valu_probe.hip — on-box microbenchmark of the VALU rates the dominance kernels
// are priced against (SURVEY §8d asks for the VALU compare peak to be measured).
//   k_fadd      : independent v_add_f32 chains                   -> 32-bit lane-ops/s
//   k_cmp_f32   : dominance pair tests, f32 rows, ballot masks    -> compares/s
//   k_cmp_u16   : dominance pair tests, packed u16 rows (saturating subtract + or)
// x rows are wave-uniform (scalar loads), y rows live in VGPRs (PPT per lane).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

constexpr int kIters = 4096;

__global__ __launch_bounds__(256) void k_fadd(float *out, float seed) {
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = seed + threadIdx.x + i;
    for (int it = 0; it < kIters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) a[i] = a[i] + 1.0001f;
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s += a[i];
    if (s == 12345.f) out[0] = s;
}

// independent v_pk_sub_u16 (clamp) chains: the packed 16-bit lane-op rate (2 compares per op is the
// packed-u16 compare peak's definition)
__global__ __launch_bounds__(256) void k_pksub(uint32_t *out, const uint32_t *__restrict__ subs, uint32_t seed) {
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    u16x2 a[8], b[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        a[i] = __builtin_bit_cast(u16x2, seed + threadIdx.x * 65537u + i);
        b[i] = __builtin_bit_cast(u16x2, subs[i]);            // runtime operands: no folding of the chain
    }
    for (int it = 0; it < kIters; it += 8) {
#pragma unroll
        for (int j = 0; j < 8; j++)
#pragma unroll
            for (int i = 0; i < 8; i++) a[i] = __builtin_elementwise_sub_sat(a[i], b[(i + j) & 7]);
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s ^= __builtin_bit_cast(uint32_t, a[i]);
    if (s == 12345u) out[0] = s;
}

template <int PPT>
__global__ __launch_bounds__(256) void k_cmp_f32(const float *__restrict__ xs, int nx, float *out) {
    float y[PPT][8];
#pragma unroll
    for (int p = 0; p < PPT; p++)
#pragma unroll
        for (int d = 0; d < 8; d++) y[p][d] = (float)((threadIdx.x * 7 + p * 13 + d * 3) % 1000);
    uint64_t dom[PPT];
#pragma unroll
    for (int p = 0; p < PPT; p++) dom[p] = 0;
    for (int rep = 0; rep < kIters / 512; rep++) {
        for (int i = 0; i < nx; i++) {
            const float *x = xs + i * 8;
#pragma unroll
            for (int p = 0; p < PPT; p++) {
                uint64_t m = ~0ull;
#pragma unroll
                for (int d = 0; d < 8; d++) m &= __ballot(x[d] <= y[p][d]);
                dom[p] |= m;
            }
        }
    }
    uint64_t t = 0;
#pragma unroll
    for (int p = 0; p < PPT; p++) t ^= dom[p];
    if (t == 0x1234567ull) out[0] = 1.0f;
}

template <int PPT>
__global__ __launch_bounds__(256) void k_cmp_u16(const uint32_t *__restrict__ xs, int nx, float *out) {
    uint32_t y[PPT][4];
#pragma unroll
    for (int p = 0; p < PPT; p++)
#pragma unroll
        for (int w = 0; w < 4; w++) {
            const uint32_t lo = (threadIdx.x * 7 + p * 13 + w * 6) % 1000, hi = (threadIdx.x * 5 + p * 11 + w * 6 + 3) % 1000;
            y[p][w] = lo | (hi << 16);
        }
    uint64_t dom[PPT];
#pragma unroll
    for (int p = 0; p < PPT; p++) dom[p] = 0;
    for (int rep = 0; rep < kIters / 512; rep++) {
        for (int i = 0; i < nx; i++) {
            const uint32_t *x = xs + i * 4;
#pragma unroll
            for (int p = 0; p < PPT; p++) {
                // x <= y in every u16 half  <=>  sat(x - y) == 0 in every half
                uint32_t r0;
                typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
                u16x2 a0 = __builtin_bit_cast(u16x2, x[0]), b0 = __builtin_bit_cast(u16x2, y[p][0]);
                u16x2 a1 = __builtin_bit_cast(u16x2, x[1]), b1 = __builtin_bit_cast(u16x2, y[p][1]);
                u16x2 a2 = __builtin_bit_cast(u16x2, x[2]), b2 = __builtin_bit_cast(u16x2, y[p][2]);
                u16x2 a3 = __builtin_bit_cast(u16x2, x[3]), b3 = __builtin_bit_cast(u16x2, y[p][3]);
                u16x2 s0 = __builtin_elementwise_sub_sat(a0, b0);
                u16x2 s1 = __builtin_elementwise_sub_sat(a1, b1);
                u16x2 s2 = __builtin_elementwise_sub_sat(a2, b2);
                u16x2 s3 = __builtin_elementwise_sub_sat(a3, b3);
                r0 = __builtin_bit_cast(uint32_t, s0) | __builtin_bit_cast(uint32_t, s1) |
                     __builtin_bit_cast(uint32_t, s2) | __builtin_bit_cast(uint32_t, s3);
                dom[p] |= __ballot(r0 == 0u);
            }
        }
    }
    uint64_t t = 0;
#pragma unroll
    for (int p = 0; p < PPT; p++) t ^= dom[p];
    if (t == 0x1234567ull) out[0] = 1.0f;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s\n", hipGetErrorString(e), #x); return 1; } } while (0)

template <typename F>
static double time_ms(F launch) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    launch();
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 5; r++) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / 5.0;
}

int main() {
    hipDeviceProp_t pr;
    CK(hipGetDeviceProperties(&pr, 0));
    const int cus = pr.multiProcessorCount;
    printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d", pr.gcnArchName, cus, pr.clockRate);
    float *out;
    CK(hipMalloc(&out, 64));
    const int blocks = cus * 8;               // 8 x 256 threads per CU = 32 waves
    // fadd
    double ms = time_ms([&] { k_fadd<<<blocks, 256>>>(out, 1.0f); });
    double ops = (double)blocks * 256 * kIters * 8;
    printf(", \"fadd_lane_ops_per_s\": %.4g", ops / (ms * 1e-3));
    uint32_t *subs;
    CK(hipMalloc(&subs, 64));
    CK(hipMemset(subs, 0, 64));                               // x - 0: the chain keeps its values
    ms = time_ms([&] { k_pksub<<<blocks, 256>>>((uint32_t *)out, subs, 0x03e803e8u); });
    printf(", \"pk_sub_u16_lane_ops_per_s\": %.4g", ops / (ms * 1e-3));
    const int nx = 512;
    std::vector<float> hx(nx * 8);
    std::vector<uint32_t> hu(nx * 4);
    for (int i = 0; i < nx * 8; i++) hx[i] = (float)((i * 37) % 1000 + 1000);   // never dominates
    for (int i = 0; i < nx * 4; i++) hu[i] = (uint32_t)(((i * 37) % 1000 + 1000) | (((i * 41) % 1000 + 1000) << 16));
    float *dx; uint32_t *du;
    CK(hipMalloc(&dx, nx * 8 * 4)); CK(hipMalloc(&du, nx * 4 * 4));
    CK(hipMemcpy(dx, hx.data(), nx * 32, hipMemcpyHostToDevice));
    CK(hipMemcpy(du, hu.data(), nx * 16, hipMemcpyHostToDevice));
    const double pairs_per_lane_ppt = (double)(kIters / 512) * nx;
#define RUN_F(P) { double t = time_ms([&] { k_cmp_f32<P><<<blocks, 256>>>(dx, nx, out); }); \
        double c = (double)blocks * 256 * pairs_per_lane_ppt * P * 8; printf(", \"f32_ppt%d_compares_per_s\": %.4g", P, c / (t * 1e-3)); }
#define RUN_U(P) { double t = time_ms([&] { k_cmp_u16<P><<<blocks, 256>>>(du, nx, out); }); \
        double c = (double)blocks * 256 * pairs_per_lane_ppt * P * 8; printf(", \"u16_ppt%d_compares_per_s\": %.4g", P, c / (t * 1e-3)); }
    RUN_F(4) RUN_F(8) RUN_U(4) RUN_U(8) RUN_U(16)
    printf("}\n");
    CK(hipGetLastError());
    return 0;
}
