// stage_pool.h — the host thread pool that stages an insert call's batches into pinned memory
// (part.hip).  Plain C++ (no HIP), so tests/stage_pool_stress.cc builds it under
// -fsanitize=thread.
//
// One job at a time (run() holds call_m_).  A job is published under m_ with a generation
// number; a worker joins it only while it is open (fn_ != nullptr) and registers itself in
// active_ under the same lock, so a worker woken for an earlier job either joins the current job
// completely (reading its fn_ / n_ under the lock) or not at all.  run() closes the job only
// when every item is done AND no worker is inside work(): next_ / done_ are reset by the next
// run() with no worker left that could claim an index of the old job, and the job's function
// (the caller's lambda) is never used after run() returns.
#pragma once

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace sky {

class StagePool {
  public:
    // `threads` counts the caller: threads - 1 persistent workers
    explicit StagePool(int threads) {
        const int hw = std::max(1, (int)std::thread::hardware_concurrency());
        const int nt = std::max(1, std::min(threads, hw));
        for (int i = 0; i < nt - 1; i++) workers_.emplace_back([this] { loop(); });
    }
    StagePool(const StagePool &) = delete;
    StagePool &operator=(const StagePool &) = delete;
    ~StagePool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (std::thread &t : workers_) t.join();
    }
    int workers() const { return (int)workers_.size(); }

    // f(i) for every i < n, on the pool's threads and the caller; returns when all are done and
    // no worker still runs f
    void run(size_t n, const std::function<void(size_t)> &f) {
        if (workers_.empty() || n < 2) {
            for (size_t i = 0; i < n; i++) f(i);
            return;
        }
        std::lock_guard<std::mutex> call(call_m_);
        {
            std::lock_guard<std::mutex> lk(m_);
            fn_ = &f;
            n_ = n;
            next_.store(0, std::memory_order_relaxed);
            done_.store(0, std::memory_order_relaxed);
            active_++;                       // the caller
            gen_++;
        }
        cv_.notify_all();
        work(f, n);
        std::unique_lock<std::mutex> lk(m_);
        active_--;
        done_cv_.wait(lk, [&] { return active_ == 0 && done_.load(std::memory_order_acquire) == n_; });
        fn_ = nullptr;                       // closed: late wakers skip it
        n_ = 0;
    }

  private:
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(size_t)> *fn;
            size_t n;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                if (!fn_) continue;          // that job closed before this worker woke
                fn = fn_;
                n = n_;
                active_++;
            }
            work(*fn, n);
            {
                std::lock_guard<std::mutex> lk(m_);
                if (--active_ == 0) done_cv_.notify_all();
            }
        }
    }
    void work(const std::function<void(size_t)> &f, size_t n) {
        for (;;) {
            const size_t i = next_.fetch_add(1, std::memory_order_relaxed);
            if (i >= n) return;
            f(i);
            done_.fetch_add(1, std::memory_order_acq_rel);
        }
    }

    std::vector<std::thread> workers_;
    std::mutex m_, call_m_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(size_t)> *fn_ = nullptr;   // guarded by m_
    size_t n_ = 0;                                       // guarded by m_
    int active_ = 0;                                     // threads inside work(), guarded by m_
    uint64_t gen_ = 0;                                   // guarded by m_
    bool stop_ = false;                                  // guarded by m_
    std::atomic<size_t> next_{0}, done_{0};
};

}  // namespace sky
