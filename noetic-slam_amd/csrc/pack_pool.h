// pack_pool.h -- the host staging thread pool of libtsdf_hip (tsdf_capi.cpp), plain C++ so the CPU
// tests can build and stress it without a GPU (tests/test_pack_pool.py).
#pragma once
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace tsdf {

// Host staging of tsdf_integrate's PointCloud2 records (the node's per-scan call): the record ->
// packed-xyz loop of a large scan is split over a few persistent threads (the caller's thread takes
// the first chunk).  One context is used by one thread at a time, so one pool per context.
struct PackPool {
    std::vector<std::thread> th;
    std::mutex m;
    std::condition_variable go, done;
    std::function<void(int)> job;  // stable while busy > 0
    std::atomic<uint64_t> gen{0};
    std::atomic<int> busy{0};
    std::atomic<bool> stop{false};
    // a worker (and a waiting caller) spins this long before sleeping: scans arrive back to back,
    // and waking a sleeping thread costs tens of microseconds on a busy host
    static constexpr double SPIN_US = 100.0;

    static bool spin_until(const std::function<bool()>& ready) {
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0;; i++) {
            if (ready()) return true;
            if ((i & 63) == 63 &&
                std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0)
                        .count() > SPIN_US)
                return false;
#if defined(__x86_64__)
            __builtin_ia32_pause();
#endif
        }
    }

    explicit PackPool(int workers) {
        for (int w = 0; w < workers; w++)
            th.emplace_back([this, w] {
                uint64_t seen = 0;
                for (;;) {
                    auto fresh = [&] { return stop.load(std::memory_order_acquire) ||
                                              gen.load(std::memory_order_acquire) != seen; };
                    if (!spin_until(fresh)) {
                        std::unique_lock<std::mutex> l(m);
                        go.wait(l, fresh);
                    }
                    if (stop.load(std::memory_order_acquire)) return;
                    seen = gen.load(std::memory_order_acquire);
                    job(w + 1);
                    if (busy.fetch_sub(1, std::memory_order_acq_rel) == 1) {
                        std::lock_guard<std::mutex> l(m);
                        done.notify_one();
                    }
                }
            });
    }
    int parts() const { return (int)th.size() + 1; }
    // f(part) for part = 0 .. parts() - 1, part 0 on the calling thread
    void run(const std::function<void(int)>& f) {
        start(f, 0);
        f(0);
        wait();
    }
    // the workers run f(base + 1) .. f(base + workers) while the caller goes on; wait() joins
    void start(const std::function<void(int)>& f, int base) {
        job = base ? std::function<void(int)>([f, base](int part) { f(base + part); }) : f;
        busy.store((int)th.size(), std::memory_order_release);
        gen.fetch_add(1, std::memory_order_acq_rel);
        { std::lock_guard<std::mutex> l(m); }  // a worker between its check and its sleep sees gen
        go.notify_all();
    }
    void wait() {
        auto idle = [&] { return busy.load(std::memory_order_acquire) == 0; };
        if (spin_until(idle)) return;
        std::unique_lock<std::mutex> l(m);
        done.wait(l, idle);
    }
    ~PackPool() {
        stop.store(true, std::memory_order_release);
        { std::lock_guard<std::mutex> l(m); }
        go.notify_all();
        for (auto& t : th) t.join();
    }
};

}  // namespace tsdf
