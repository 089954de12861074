// host_pool.h — a small persistent worker pool for the adapters' per-element host loops (the
// snapshot gather of LocalBA::Flatten and the result write-back into the Frame / Landmark objects).
// Internal to libvxslam_host.  One job at a time (jobs from several threads are serialised); the
// calling thread works on the job too.  $VX_HOST_THREADS sets the participants (default: up to 8,
// at most the CPUs this process may use); 1 runs every job inline.  The workers are bound to the
// CPUs that share the creating thread's last-level cache (its CCD on an EPYC host): on the GPU box
// (2 sockets, 16 L3 slices, affinity over all 256 CPUs) a free-floating worker lands on any slice,
// and every array a job hands over then crosses slices or sockets ($VX_HOST_PIN=0: unbound).
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <cstdlib>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include <cstdio>
#include <cstring>
#include <string>

#include <pthread.h>
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
        // each job has its own counters: a worker that arrives after the job is done only finds
        // next >= n (it never calls fn then), whatever job runs next
        auto job = std::make_shared<Job>();
        job->fn = &fn;
        job->n = n;
        job->chunk = (n + parts - 1) / parts;
        {
            std::lock_guard<std::mutex> lk(m_);
            cur_ = job;
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        Run(*job);
        while (job->done.load(std::memory_order_acquire) < n) Relax();
    }

    Pool(const Pool&) = delete;
    Pool& operator=(const Pool&) = delete;

private:
    struct Job {
        const std::function<void(size_t, size_t)>* fn = nullptr;
        size_t n = 0, chunk = 1;
        std::atomic<size_t> next{0}, done{0};
    };
    Pool() {
        // participants: 8, or with the workers bound to an L3 slice every CPU of that slice up to 16
        // (the GPU box's slices are 8 cores / 16 threads: 16 measured 4 % faster on the snapshot call,
        // 2 % on the resident one, r06s); never more than the CPUs this process may use
        // (a process confined to a few CPUs spread over slices leaves too few in the creating thread's
        // slice: then the workers stay unbound rather than share two or three CPUs)
        const char* pin = std::getenv("VX_HOST_PIN");
        cpu_set_t llc;
        const bool bind = !(pin && pin[0] == '0') && LlcCpus(&llc) && CPU_COUNT(&llc) >= 8;
        int want = bind ? std::min(16, CPU_COUNT(&llc)) : 8;
        cpu_set_t set;
        if (sched_getaffinity(0, sizeof(set), &set) == 0) want = std::min(want, CPU_COUNT(&set));
        if (const char* e = std::getenv("VX_HOST_THREADS")) want = std::max(1, std::atoi(e));
        if (const char* e = std::getenv("VX_HOST_SPIN_US")) spin_us_ = std::max(0, std::atoi(e));
        for (int i = 1; i < want; ++i) workers_.emplace_back([this] { Loop(); });
        if (bind)
            for (auto& t : workers_) (void)pthread_setaffinity_np(t.native_handle(), sizeof llc, &llc);
    }
    // the CPUs sharing the calling thread's last-level cache, within this process's affinity
    static bool LlcCpus(cpu_set_t* out) {
        const int cpu = sched_getcpu();
        if (cpu < 0) return false;
        char path[128];
        std::snprintf(path, sizeof path, "/sys/devices/system/cpu/cpu%d/cache/index3/shared_cpu_list", cpu);
        FILE* f = std::fopen(path, "r");
        if (!f) return false;
        char buf[512] = {0};
        const bool ok = std::fgets(buf, sizeof buf, f) != nullptr;
        std::fclose(f);
        if (!ok) return false;
        cpu_set_t allowed;
        if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return false;
        CPU_ZERO(out);
        for (char* tok = std::strtok(buf, ",\n"); tok; tok = std::strtok(nullptr, ",\n")) {
            int a = -1, b = -1;
            const int n = std::sscanf(tok, "%d-%d", &a, &b);
            if (n < 1) continue;
            if (n == 1) b = a;
            for (int i = a; i <= b && i < CPU_SETSIZE; ++i)
                if (i >= 0 && CPU_ISSET(i, &allowed)) CPU_SET(i, out);
        }
        return CPU_COUNT(out) >= 2;
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }
    static void Relax() { __builtin_ia32_pause(); }
    static void Run(Job& j) {
        for (;;) {
            const size_t b = j.next.fetch_add(j.chunk, std::memory_order_acq_rel);
            if (b >= j.n) return;
            const size_t e = std::min(j.n, b + j.chunk);
            (*j.fn)(b, e);
            j.done.fetch_add(e - b, std::memory_order_acq_rel);
        }
    }
    // A worker spins for spin_us_ ($VX_HOST_SPIN_US, default 0) after a job before it sleeps again.
    void Loop() {
        unsigned long long seen = 0;
        {
            std::lock_guard<std::mutex> lk(m_);
            seen = gen_.load(std::memory_order_relaxed);
        }
        for (;;) {
            bool job = false;
            const auto t0 = std::chrono::steady_clock::now();
            for (unsigned it = 0;; ++it) {
                if (gen_.load(std::memory_order_acquire) != seen) {
                    job = true;
                    break;
                }
                if ((it & 255) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us_)) break;
                Relax();
            }
            std::shared_ptr<Job> j;
            {
                std::unique_lock<std::mutex> lk(m_);
                if (!job) cv_.wait(lk, [&] { return gen_.load(std::memory_order_relaxed) != seen; });
                seen = gen_.load(std::memory_order_relaxed);
                if (stop_) return;
                j = cur_;
            }
            if (j) Run(*j);
        }
    }

    std::vector<std::thread> workers_;
    std::mutex submit_, m_;
    std::condition_variable cv_;
    std::shared_ptr<Job> cur_;
    std::atomic<unsigned long long> gen_{0};
    bool stop_ = false;
    int spin_us_ = 0;  // ($VX_HOST_SPIN_US: 300 measured slower on the GPU box, whose CPU quota a spinning
                       // worker eats into)
};

}  // namespace vxhost
}  // namespace visionx
