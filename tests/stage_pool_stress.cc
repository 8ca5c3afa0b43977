// Stress test of the insert staging pool (flink-skyline-qos_amd/csrc/stage_pool.h), built by
// tests/test_cpu_stage_pool.py with and without -fsanitize=thread.
//
// Thousands of back-to-back jobs of varying size (0 .. 300 items, many of them tiny so workers
// that wake late for job k meet job k+1).  Every job's items write into a vector owned by that
// job's stack frame: after run() returns each item must have run exactly once, and nothing may
// touch the vector afterwards (it is freed and reused by the next job: TSAN / ASAN see a late
// worker).  Some items yield or sleep, so workers are descheduled inside and between jobs.
#include "stage_pool.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <random>

int main(int argc, char **argv) {
    const int jobs = argc > 1 ? atoi(argv[1]) : 20000;
    const int threads = argc > 2 ? atoi(argv[2]) : 4;
    sky::StagePool pool(threads);
    std::mt19937 rng(12345);
    long long items = 0;
    for (int j = 0; j < jobs; j++) {
        const size_t n = (rng() % 8 == 0) ? rng() % 301 : rng() % 6;
        const int mode = (int)(rng() % 16);
        auto hits = std::make_unique<std::atomic<int>[]>(n + 1);
        for (size_t i = 0; i <= n; i++) hits[i].store(0);
        std::vector<int> payload(n + 1, j);
        pool.run(n, [&](size_t i) {
            if (mode == 0 && i % 7 == 0) std::this_thread::yield();
            if (mode == 1 && i == 0) std::this_thread::sleep_for(std::chrono::microseconds(50));
            payload[i] += 1;                       // plain write: a race if two threads run item i
            hits[i].fetch_add(1);
        });
        for (size_t i = 0; i < n; i++) {
            if (hits[i].load() != 1 || payload[i] != j + 1) {
                fprintf(stderr, "job %d (n=%zu): item %zu ran %d times\n", j, n, i, hits[i].load());
                return 1;
            }
        }
        if (hits[n].load() != 0) {
            fprintf(stderr, "job %d: an item past n ran\n", j);
            return 1;
        }
        items += (long long)n;
    }
    printf("ok jobs=%d items=%lld workers=%d\n", jobs, items, pool.workers());
    return 0;
}
