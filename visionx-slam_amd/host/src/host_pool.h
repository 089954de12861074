// host_pool.h — a small persistent worker pool for the adapters' per-element host loops (the
// snapshot gather of LocalBA::Flatten and the result write-back into the Frame / Landmark objects).
// Internal to libvxslam_host.  One job at a time (jobs from several threads are serialised); the
// calling thread works on the job too.  $VX_HOST_THREADS sets the participants (default: up to 8,
// at most the CPUs this process may use); 1 runs every job inline.
#pragma once

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include <sched.h>

namespace visionx {
namespace vxhost {

class Pool {
public:
    static Pool& Get() {
        static Pool pool;
        return pool;
    }
    int Threads() const { return (int)workers_.size() + 1; }

    // fn(begin, end) over [0, n) in chunks of at least min_chunk items; returns when every chunk is done
    void For(size_t n, size_t min_chunk, const std::function<void(size_t, size_t)>& fn) {
        if (n == 0) return;
        const size_t parts = std::min<size_t>((size_t)Threads() * 4, (n + min_chunk - 1) / std::max<size_t>(min_chunk, 1));
        if (workers_.empty() || parts <= 1) {
            fn(0, n);
            return;
        }
        std::lock_guard<std::mutex> serial(submit_);
        {
            std::lock_guard<std::mutex> lk(m_);
            fn_ = &fn;
            n_ = n;
            chunk_ = (n + parts - 1) / parts;
            next_.store(0, std::memory_order_relaxed);
            busy_ = (int)workers_.size();
            ++gen_;
        }
        cv_.notify_all();
        Work();
        std::unique_lock<std::mutex> lk(m_);
        done_cv_.wait(lk, [&] { return busy_ == 0; });
        fn_ = nullptr;
    }

    Pool(const Pool&) = delete;
    Pool& operator=(const Pool&) = delete;

private:
    Pool() {
        int want = 8;
        cpu_set_t set;
        if (sched_getaffinity(0, sizeof(set), &set) == 0) want = std::min(want, CPU_COUNT(&set));
        if (const char* e = std::getenv("VX_HOST_THREADS")) want = std::max(1, std::atoi(e));
        for (int i = 1; i < want; ++i) workers_.emplace_back([this] { Loop(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
            ++gen_;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }
    void Work() {
        for (;;) {
            const size_t b = next_.fetch_add(chunk_, std::memory_order_relaxed);
            if (b >= n_) return;
            (*fn_)(b, std::min(n_, b + chunk_));
        }
    }
    void Loop() {
        unsigned long long seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                if (stop_) return;
            }
            Work();
            std::lock_guard<std::mutex> lk(m_);
            if (--busy_ == 0) done_cv_.notify_one();
        }
    }

    std::vector<std::thread> workers_;
    std::mutex submit_, m_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(size_t, size_t)>* fn_ = nullptr;
    size_t n_ = 0, chunk_ = 1;
    std::atomic<size_t> next_{0};
    int busy_ = 0;
    unsigned long long gen_ = 0;
    bool stop_ = false;
};

}  // namespace vxhost
}  // namespace visionx
