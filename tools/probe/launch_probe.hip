// launch_probe.hip — the cost of a dependent kernel boundary on one stream (MI355X):
// K back-to-back launches of (a) an empty kernel, (b) a one-workgroup kernel that reads a word
// written by the previous launch and writes the next one, (c) 256 workgroups doing the same
// through an atomic; timed with HIP events.  Build: hipcc --offload-arch=gfx950 -O3 -o
// tools/probe/launch_probe tools/probe/launch_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty() {}
__global__ void k_chain(unsigned *w) {
    if (threadIdx.x == 0 && blockIdx.x == 0) w[1] = w[0] + 1, w[0] = w[1];
}
__global__ void k_chain_grid(unsigned *w) {
    __shared__ unsigned v;
    if (threadIdx.x == 0) v = w[0];
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(&w[2 + (blockIdx.x & 63)], v);
    if (threadIdx.x == 0 && blockIdx.x == 0) w[0] = v + 1;
}
// last-arriver: every workgroup increments a counter after a release fence; the last one
// does a tiny serial phase (the pattern that replaces a second launch)
__global__ void k_last_arriver(unsigned *w, unsigned *ctr) {
    __shared__ bool last;
    if (threadIdx.x == 0) {
        atomicAdd(&w[2 + (blockIdx.x & 63)], 1u);
        __threadfence();
        last = atomicAdd(ctr, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (last && threadIdx.x == 0) {
        __threadfence();
        unsigned s = 0;
        for (int i = 0; i < 64; i++) s += __hip_atomic_load(&w[2 + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        w[0] = s;
        *ctr = 0;
    }
}

int main() {
    unsigned *w, *ctr;
    hipMalloc(&w, 4096);
    hipMalloc(&ctr, 64);
    hipMemset(w, 0, 4096);
    hipMemset(ctr, 0, 64);
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int K = 200;
    for (int mode = 0; mode < 6; mode++) {
        for (int rep = 0; rep < 2; rep++) {
            hipEventRecord(a, st);
            for (int i = 0; i < K; i++) {
                if (mode == 0) k_empty<<<1, 64, 0, st>>>();
                else if (mode == 1) k_chain<<<1, 256, 0, st>>>(w);
                else if (mode == 2) k_chain_grid<<<256, 256, 0, st>>>(w);
                else if (mode == 3) k_chain_grid<<<2048, 256, 0, st>>>(w);
                else if (mode == 4) k_last_arriver<<<256, 256, 0, st>>>(w, ctr);
                else k_last_arriver<<<2048, 256, 0, st>>>(w, ctr);
            }
            hipEventRecord(b, st);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            if (rep) printf("mode %d (%s): %.2f us per launch\n", mode,
                            mode == 0 ? "empty 1 WG" : mode == 1 ? "chain 1 WG" : mode == 2 ? "chain 256 WG" :
                            mode == 3 ? "chain 2048 WG" : mode == 4 ? "last-arriver 256 WG" : "last-arriver 2048 WG",
                            ms * 1e3 / K);
        }
    }
    return 0;
}
