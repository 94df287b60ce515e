// skm_pool.h -- a fixed pool of host threads (the host side of a one-shot build
// must not be one thread).  run(n, f) calls f(0..n-1) on the pool's threads and the caller's,
// parts taken from an atomic counter, and returns when every part is done.  One run at a time
// (one build handle is driven from one host thread, include/skm.h).
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace skm {

class HostPool {
public:
    // threads including the caller: SKM_HOST_THREADS, else min(16, hardware threads) -- the GPU
    // box's cgroup quota is 16 CPUs while nproc shows the whole machine
    static int default_threads() {
        if (const char* e = std::getenv("SKM_HOST_THREADS")) {
            const int v = std::atoi(e);
            if (v > 0) return std::min(v, 256);
        }
        const unsigned hw = std::thread::hardware_concurrency();
        return (int)std::max(1u, std::min(16u, hw ? hw : 1u));
    }
    explicit HostPool(int threads) {
        for (int i = 1; i < threads; ++i) th_.emplace_back([this] { loop(); });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
            stop_flag_.store(true);
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    HostPool(const HostPool&) = delete;
    HostPool& operator=(const HostPool&) = delete;
    int threads() const { return (int)th_.size() + 1; }

    void run(int n, std::function<void(int)> f) {
        if (th_.empty() || n <= 1) {
            for (int p = 0; p < n; ++p) f(p);
            return;
        }
        {
            std::unique_lock<std::mutex> l(m_);
            done_.wait(l, [&] { return active_ == 0; });  // a late waker of the last run has left
            job_ = std::move(f);
            parts_ = n;
            next_.store(0);
            done_parts_.store(0, std::memory_order_relaxed);
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        work();
        // every part done: return without a futex round trip (a worker still leaving work() only
        // finds the part counter exhausted; the next run waits for it under the lock above)
        const auto t0 = std::chrono::steady_clock::now();
        while (done_parts_.load(std::memory_order_acquire) < n &&
               std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(SPIN_US))
            __builtin_ia32_pause();
        if (done_parts_.load(std::memory_order_acquire) >= n) return;
        std::unique_lock<std::mutex> l(m_);
        done_.wait(l, [&] { return active_ == 0; });
    }

private:
    void work() {
        for (int p; (p = next_.fetch_add(1)) < parts_;) {
            job_(p);
            done_parts_.fetch_add(1, std::memory_order_release);
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            // a caller adding many small batches back to back (one per genome file) would pay a
            // futex wake-up per batch: spin a little for the next run before sleeping
            const auto t0 = std::chrono::steady_clock::now();
            while (gen_.load(std::memory_order_acquire) == seen && !stop_flag_.load(std::memory_order_relaxed) &&
                   std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(SPIN_US))
                __builtin_ia32_pause();
            std::unique_lock<std::mutex> l(m_);
            cv_.wait(l, [&] { return stop_ || gen_.load() != seen; });
            if (stop_) return;
            seen = gen_.load();
            ++active_;
            l.unlock();
            work();
            l.lock();
            if (--active_ == 0) done_.notify_all();
        }
    }
    static constexpr int SPIN_US = 200;
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    std::function<void(int)> job_;
    std::atomic<int> next_{0}, done_parts_{0};
    int parts_ = 0, active_ = 0;
    std::atomic<uint64_t> gen_{0};
    bool stop_ = false;
    std::atomic<bool> stop_flag_{false};  // stop_ for the spinning workers
};

}  // namespace skm
