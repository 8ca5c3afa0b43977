// radix_test.hip — stress test of sky::radix_sort_pairs (k_radix.hip) in isolation:
// random 64-bit keys with a chosen varying-bit mask, values = original indices; checks
// sortedness, that the values form a permutation and that every key matches its
// source index, over many sizes and repetitions.
//   hipcc -O3 --offload-arch=gfx950 -I../../include -I../../flink-skyline-qos_amd/csrc radix_test.hip \
//         ../../flink-skyline-qos_amd/build/k_radix.o -o radix_test
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include "sky_internal.h"

static uint64_t rng_state = 88172645463325252ull;
static uint64_t xr() { rng_state ^= rng_state << 13; rng_state ^= rng_state >> 7; rng_state ^= rng_state << 17; return rng_state; }

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    const uint64_t masks[] = {0x0701fff00000ffffull, 0x00000000ffffffffull, 0x07ffffffffffffffull, 0x00ff00ff00ff00ffull};
    const uint32_t sizes[] = {1000, 4096, 92223, 250000, 1 << 20};
    int fails = 0;
    for (uint64_t mask : masks)
        for (uint32_t m : sizes) {
            std::vector<uint64_t> k(m), ks(m);
            std::vector<uint32_t> v(m), vs(m);
            uint64_t *dk, *dka;
            uint32_t *dv, *dva, *scr, *err;
            (void)hipMalloc(&dk, m * 8); (void)hipMalloc(&dka, m * 8);
            (void)hipMalloc(&dv, m * 4); (void)hipMalloc(&dva, m * 4);
            (void)hipMalloc(&scr, sky::radix_scratch_words(m) * 4 * (getenv("GUARD2") ? 2 : 1) + 64);
            (void)hipMalloc(&err, 4);
            for (int r = 0; r < reps; r++) {
                const uint64_t base = xr() & ~mask;
                uint64_t o = 0, a = ~0ull;
                for (uint32_t i = 0; i < m; i++) {
                    k[i] = base | (xr() & mask & (r % 3 ? xr() : ~0ull));
                    v[i] = i;
                    o |= k[i]; a &= k[i];
                }
                (void)hipMemcpy(dk, k.data(), m * 8, hipMemcpyHostToDevice);
                (void)hipMemcpy(dv, v.data(), m * 4, hipMemcpyHostToDevice);
                (void)hipMemset(err, 0, 4);
                const bool alt = sky::radix_sort_pairs(dk, dv, dka, dva, m, o, a, scr, err, 0);
                (void)hipDeviceSynchronize();
                (void)hipMemcpy(ks.data(), alt ? dka : dk, m * 8, hipMemcpyDeviceToHost);
                (void)hipMemcpy(vs.data(), alt ? dva : dv, m * 4, hipMemcpyDeviceToHost);
                uint32_t e = 0;
                (void)hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
                int bad = 0;
                std::vector<char> seen(m, 0);
                for (uint32_t j = 0; j < m; j++) {
                    if (j && ks[j - 1] > ks[j]) bad |= 1;
                    if (vs[j] >= m) { bad |= 2; continue; }
                    if (k[vs[j]] != ks[j]) {
                        if (!(bad & 4))
                            printf("  j=%u got %016llx want %016llx (src %u) prev %016llx next %016llx\n", j,
                                   (unsigned long long)ks[j], (unsigned long long)k[vs[j]], vs[j],
                                   (unsigned long long)(j ? ks[j - 1] : 0), (unsigned long long)(j + 1 < m ? ks[j + 1] : 0));
                        bad |= 4;
                    }
                    if (seen[vs[j]]++) bad |= 8;
                    if (j && ks[j - 1] == ks[j] && vs[j - 1] > vs[j]) bad |= 16;   // stability
                }
                if (bad || e) {
                    fails++;
                    printf("FAIL mask=%016llx m=%u rep=%d bad=%d err=%u\n", (unsigned long long)mask, m, r, bad, e);
                }
            }
            (void)hipFree(dk); (void)hipFree(dka); (void)hipFree(dv); (void)hipFree(dva); (void)hipFree(scr);
            (void)hipFree(err);
        }
    printf("radix_test: %d failures\n", fails);
    return fails ? 1 : 0;
}
