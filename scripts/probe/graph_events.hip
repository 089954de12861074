// Host cost of event-wait / event-record nodes inside a graph (round 4): could a
// frame's cross-stream waits and records travel inside its graph launches instead of costing a
// hipStreamWaitEvent / hipEventRecord call each?  Prints host microseconds per launch for kernel-only
// graphs and the same graphs with event nodes, the frame pattern both ways, and an ordering check
// (a consumer graph that waits on an event recorded by a slow producer graph on another stream
// must see the producer's write).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                            \
    do {                                                                 \
        hipError_t e_ = (x);                                             \
        if (e_ != hipSuccess) {                                          \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));          \
            std::exit(1);                                                \
        }                                                                \
    } while (0)

__global__ void k_noop(int* p) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345) p[1] = 1;
}
// producer: ~20 us of waiting (bounded by the clock), then flag = i
__global__ void k_slow_write(int* flag, int* iter) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        const unsigned long long t0 = __builtin_readcyclecounter();
        while (__builtin_readcyclecounter() - t0 < 40000ull) __builtin_amdgcn_s_sleep(8);
        const int i = iter[0] + 1;
        iter[0] = i;
        flag[0] = i;
    }
}
// consumer: out[n++] = flag
__global__ void k_read(const int* flag, int* out, int* n) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        const int k = n[0];
        if (k < 4096) out[k] = flag[0];
        n[0] = k + 1;
    }
}

using clk = std::chrono::steady_clock;
static double us_since(clk::time_point t0) { return std::chrono::duration<double, std::micro>(clk::now() - t0).count(); }

// a linear graph: [wait ew] -> n kernel nodes -> [record er]
static hipGraphExec_t make_graph(void* fn, void** args, int n, hipEvent_t ew, hipEvent_t er) {
    hipGraph_t g;
    CK(hipGraphCreate(&g, 0));
    hipGraphNode_t prev = nullptr, node;
    if (ew) {
        CK(hipGraphAddEventWaitNode(&node, g, nullptr, 0, ew));
        prev = node;
    }
    for (int i = 0; i < n; ++i) {
        hipKernelNodeParams kp{};
        kp.func = fn;
        kp.gridDim = dim3(64);
        kp.blockDim = dim3(256);
        kp.kernelParams = args;
        CK(hipGraphAddKernelNode(&node, g, prev ? &prev : nullptr, prev ? 1 : 0, &kp));
        prev = node;
    }
    if (er) {
        CK(hipGraphAddEventRecordNode(&node, g, prev ? &prev : nullptr, prev ? 1 : 0, er));
        prev = node;
    }
    hipGraphExec_t x;
    CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
    CK(hipGraphDestroy(g));
    return x;
}

int main() {
    hipStream_t s, s2;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    int* d;
    CK(hipMalloc(&d, 64));
    CK(hipMemset(d, 0, 64));
    void* args[] = {&d};
    hipEvent_t e1, e2, e3;
    CK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&e2, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&e3, hipEventDisableTiming));
    CK(hipEventRecord(e1, s2));
    CK(hipEventRecord(e2, s2));
    CK(hipStreamSynchronize(s2));
    const int kRounds = 40, kPer = 16;
    auto time_graph = [&](const char* name, hipGraphExec_t x) {
        double tot = 0;
        for (int w = 0; w < 2; ++w) {
            tot = 0;
            for (int r = 0; r < kRounds; ++r) {
                auto t0 = clk::now();
                for (int i = 0; i < kPer; ++i) CK(hipGraphLaunch(x, s));
                tot += us_since(t0);
                CK(hipStreamSynchronize(s));
            }
        }
        std::printf("%-44s %7.2f us/launch\n", name, tot / (kRounds * kPer));
    };
    hipGraphExec_t g6 = make_graph((void*)k_noop, args, 6, nullptr, nullptr);
    hipGraphExec_t gw6 = make_graph((void*)k_noop, args, 6, e1, nullptr);
    hipGraphExec_t g6r = make_graph((void*)k_noop, args, 6, nullptr, e3);
    hipGraphExec_t gw6r = make_graph((void*)k_noop, args, 6, e1, e3);
    time_graph("6 kernel nodes", g6);
    time_graph("event wait + 6 kernel nodes", gw6);
    time_graph("6 kernel nodes + event record", g6r);
    time_graph("event wait + 6 kernel nodes + event record", gw6r);

    // frame pattern as calls (launch_cost.hip) and as graphs carrying their waits / records
    {
        hipGraphExec_t x4 = make_graph((void*)k_noop, args, 4, nullptr, nullptr);
        hipGraphExec_t x6 = make_graph((void*)k_noop, args, 6, nullptr, nullptr);
        hipGraphExec_t y4 = make_graph((void*)k_noop, args, 4, e2, e1);
        hipGraphExec_t y6 = make_graph((void*)k_noop, args, 6, e1, e2);
        for (int variant = 0; variant < 2; ++variant) {
            double tot = 0;
            for (int w = 0; w < 2; ++w) {
                tot = 0;
                for (int r = 0; r < kRounds; ++r) {
                    auto t0 = clk::now();
                    for (int i = 0; i < 12; ++i) {
                        if (variant == 0) {
                            CK(hipStreamWaitEvent(s, e2, 0));
                            CK(hipGraphLaunch(x4, s));
                            CK(hipEventRecord(e1, s));
                            CK(hipStreamWaitEvent(s2, e1, 0));
                            CK(hipGraphLaunch(x6, s2));
                            CK(hipEventRecord(e2, s2));
                        } else {
                            CK(hipGraphLaunch(y4, s));
                            CK(hipGraphLaunch(y6, s2));
                        }
                    }
                    tot += us_since(t0);
                    CK(hipStreamSynchronize(s));
                    CK(hipStreamSynchronize(s2));
                }
            }
            std::printf("frame pattern (4+6 nodes, 2 waits, 2 records) %s %7.2f us/frame\n",
                        variant == 0 ? "as calls      " : "inside graphs ", tot / (kRounds * 12));
        }
    }

    // event query (complete / pending) and the stream memory operations
    {
        hipEvent_t eq;
        CK(hipEventCreateWithFlags(&eq, hipEventDisableTiming));
        CK(hipEventRecord(eq, s2));
        CK(hipStreamSynchronize(s2));
        double tq = 0;
        for (int r = 0; r < kRounds; ++r) {
            auto t0 = clk::now();
            for (int i = 0; i < kPer; ++i) (void)hipEventQuery(eq);
            tq += us_since(t0);
        }
        std::printf("%-44s %7.2f us/call\n", "hipEventQuery (complete)", tq / (kRounds * kPer));
        int *fl, *it;
        CK(hipMalloc(&fl, 4));
        CK(hipMalloc(&it, 4));
        CK(hipMemset(fl, 0, 4));
        CK(hipMemset(it, 0, 4));
        CK(hipDeviceSynchronize());
        void* pa[] = {&fl, &it};
        hipGraphExec_t slow = make_graph((void*)k_slow_write, pa, 1, nullptr, eq);
        tq = 0;
        for (int r = 0; r < kRounds; ++r) {
            CK(hipGraphLaunch(slow, s2));
            auto t0 = clk::now();
            for (int i = 0; i < kPer; ++i) (void)hipEventQuery(eq);
            tq += us_since(t0);
            CK(hipStreamSynchronize(s2));
        }
        std::printf("%-44s %7.2f us/call\n", "hipEventQuery (pending)", tq / (kRounds * kPer));
        double tw = 0, tv = 0;
        for (int w = 0; w < 2; ++w) {
            tw = tv = 0;
            for (int r = 0; r < kRounds; ++r) {
                auto t0 = clk::now();
                for (int i = 0; i < kPer; ++i) CK(hipStreamWriteValue32(s2, fl, (uint32_t)(r * kPer + i), 0));
                tv += us_since(t0);
                t0 = clk::now();
                for (int i = 0; i < kPer; ++i) CK(hipStreamWaitValue32(s, fl, 0u, hipStreamWaitValueGte, 0xffffffffu));
                tw += us_since(t0);
                CK(hipStreamSynchronize(s));
                CK(hipStreamSynchronize(s2));
            }
        }
        std::printf("%-44s %7.2f us/call\n", "hipStreamWriteValue32", tv / (kRounds * kPer));
        std::printf("%-44s %7.2f us/call\n", "hipStreamWaitValue32 (satisfied)", tw / (kRounds * kPer));
    }

    // ordering: producer graph on s2 (slow write, record e3), consumer graph on s (wait e3, read)
    {
        int *flag, *iter, *out, *n;
        CK(hipMalloc(&flag, 4));
        CK(hipMalloc(&iter, 4));
        CK(hipMalloc(&out, 4096 * 4));
        CK(hipMalloc(&n, 4));
        CK(hipMemset(flag, 0, 4));
        CK(hipMemset(iter, 0, 4));
        CK(hipMemset(n, 0, 4));
        CK(hipMemset(out, 0xff, 4096 * 4));
        CK(hipDeviceSynchronize());
        void* pa[] = {&flag, &iter};
        void* ca[] = {&flag, &out, &n};
        hipGraphExec_t prod = make_graph((void*)k_slow_write, pa, 1, nullptr, e3);
        hipGraphExec_t cons = make_graph((void*)k_read, ca, 1, e3, nullptr);
        const int kN = 200;
        for (int i = 0; i < kN; ++i) {
            CK(hipGraphLaunch(prod, s2));
            CK(hipGraphLaunch(cons, s));
        }
        CK(hipDeviceSynchronize());
        std::vector<int> h(kN);
        CK(hipMemcpy(h.data(), out, kN * 4, hipMemcpyDeviceToHost));
        int bad = 0;
        for (int i = 0; i < kN; ++i) bad += h[i] < i + 1;  // (a later producer may already have run)
        std::printf("ordering: consumer saw its producer's write (or a later one) in %d of %d launches\n", kN - bad, kN);
    }
    return 0;
}
