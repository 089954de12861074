// Landmark write-back loop (LocalBA::OptimizeResident) with and without software prefetch, on the
// host: g++ -O2 -std=c++17 -pthread -Ivisionx-slam_amd/host/include scripts/probe/writeback_prefetch.cpp
// -o /tmp/wb && /tmp/wb <distance>   (distance 0: no prefetch; caches evicted before each run)
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>
#include "visionx/frame.h"
#include "../../visionx-slam_amd/host/src/host_pool.h"
using namespace visionx;
int main(int argc, char** argv) {
    const int N = 20000, D = argc > 1 ? atoi(argv[1]) : 0;
    std::vector<Landmark::Ptr> lms;
    std::mt19937 rng(1);
    // allocate with interleaved garbage to scatter
    std::vector<std::unique_ptr<char[]>> junk;
    for (int i = 0; i < 200000; ++i) {
        lms.push_back(std::make_shared<Landmark>(i, Vec3d(1, 2, 3)));
        junk.emplace_back(new char[64 + rng() % 512]);
    }
    std::vector<int> rows(N);
    for (int i = 0; i < N; ++i) rows[i] = rng() % 200000;
    std::vector<double> pos(3 * N, 1.5);
    auto& pool = vxhost::Pool::Get();
    std::vector<char> flush(64 << 20, 1);
    double best = 1e9, sum = 0;
    for (int rep = 0; rep < 30; ++rep) {
        for (size_t i = 0; i < flush.size(); i += 64) flush[i]++;  // evict caches
        auto t0 = std::chrono::steady_clock::now();
        pool.For((size_t)N, 1024, [&](size_t a, size_t b) {
            for (size_t i = a; i < b; ++i) {
                if (D && i + D < b) {
                    const Landmark* p = lms[rows[i + D]].get();
                    __builtin_prefetch(p, 1);
                    __builtin_prefetch(reinterpret_cast<const char*>(p) + 64, 1);
                    __builtin_prefetch(reinterpret_cast<const char*>(p) + 128, 1);
                }
                if (D && i + 2 * D < b) __builtin_prefetch(&lms[rows[i + 2 * D]], 0);
                const auto& lm = lms[rows[i]];
                if (lm) lm->SetPosition(Vec3d(pos[3 * i], pos[3 * i + 1], pos[3 * i + 2]));
            }
        });
        double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        best = std::min(best, us);
        if (rep >= 10) sum += us;
    }
    printf("D=%d best %.1f us mean %.1f us (threads %d)\n", D, best, sum / 20, pool.Threads());
}
