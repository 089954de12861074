// Host cost of the HIP calls a pipelined step makes (round 4): hipGraphLaunch of
// captured graphs of N kernel nodes, a plain kernel launch, hipEventRecord and hipStreamWaitEvent —
// host microseconds per call, averaged over batches that stay below the queue depth.
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

struct Big {
    double* p[40];
    int v[32];
};  // ~450 bytes of kernel arguments, like k_ba_iter's BAArgs + FusedArgs
__global__ void k_big(Big b, int it) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && b.v[it & 31] == 12345) b.p[0][0] = 1.0;
}
extern __shared__ double dyn_lds[];
__global__ void k_lds(int* p) {
    dyn_lds[threadIdx.x] = 1.0;
    __syncthreads();
    if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345) p[1] = (int)dyn_lds[5];
}

using clk = std::chrono::steady_clock;
static double us_since(clk::time_point t0) { return std::chrono::duration<double, std::micro>(clk::now() - t0).count(); }

int main() {
    hipStream_t s, s2;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    int* d;
    CK(hipMalloc(&d, 64));
    CK(hipMemset(d, 0, 64));
    const int kBatch = 64, kRounds = 40;
    // plain launches
    for (int w = 0; w < 2; ++w) {
        double tot = 0;
        for (int r = 0; r < kRounds; ++r) {
            auto t0 = clk::now();
            for (int i = 0; i < kBatch; ++i) hipLaunchKernelGGL(k_noop, dim3(64), dim3(256), 0, s, d);
            tot += us_since(t0);
            CK(hipStreamSynchronize(s));
        }
        if (w) std::printf("kernel launch            %7.2f us/call\n", tot / (kRounds * kBatch));
    }
    // graphs of N nodes
    for (int n : {1, 2, 4, 8, 16, 32}) {
        hipGraph_t g;
        hipGraphExec_t x;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
        for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_noop, dim3(64), dim3(256), 0, s, d);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
        double tot = 0;
        for (int w = 0; w < 2; ++w) {
            tot = 0;
            for (int r = 0; r < kRounds; ++r) {
                auto t0 = clk::now();
                for (int i = 0; i < kBatch / 4; ++i) CK(hipGraphLaunch(x, s));
                tot += us_since(t0);
                CK(hipStreamSynchronize(s));
            }
        }
        std::printf("graph of %2d nodes        %7.2f us/launch  (%5.2f us/node)\n", n, tot / (kRounds * kBatch / 4),
                    tot / (kRounds * kBatch / 4) / n);
        CK(hipGraphExecDestroy(x));
        CK(hipGraphDestroy(g));
    }
    // graphs of 6 nodes with large kernel arguments / 96 KB of dynamic LDS
    {
        Big b{};
        b.p[0] = reinterpret_cast<double*>(d);
        CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_lds), hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
        for (int variant = 0; variant < 2; ++variant) {
            hipGraph_t g;
            hipGraphExec_t x;
            CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
            for (int i = 0; i < 6; ++i) {
                if (variant == 0) hipLaunchKernelGGL(k_big, dim3(129), dim3(512), 0, s, b, i);
                else hipLaunchKernelGGL(k_lds, dim3(129), dim3(512), 96 * 1024, s, d);
            }
            CK(hipStreamEndCapture(s, &g));
            CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
            double tot = 0;
            for (int w = 0; w < 2; ++w) {
                tot = 0;
                for (int r = 0; r < kRounds; ++r) {
                    auto t0 = clk::now();
                    for (int i = 0; i < kBatch / 4; ++i) CK(hipGraphLaunch(x, s));
                    tot += us_since(t0);
                    CK(hipStreamSynchronize(s));
                }
            }
            std::printf("graph of 6 nodes, %s %7.2f us/launch\n", variant == 0 ? "450 B args     " : "96 KB dyn LDS  ",
                        tot / (kRounds * kBatch / 4));
            CK(hipGraphExecDestroy(x));
            CK(hipGraphDestroy(g));
        }
    }
    // events
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    for (int w = 0; w < 2; ++w) {
        double tr = 0, tw = 0;
        for (int r = 0; r < kRounds; ++r) {
            auto t0 = clk::now();
            for (int i = 0; i < kBatch; ++i) CK(hipEventRecord(ev, s));
            tr += us_since(t0);
            t0 = clk::now();
            for (int i = 0; i < kBatch; ++i) CK(hipStreamWaitEvent(s2, ev, 0));
            tw += us_since(t0);
            CK(hipStreamSynchronize(s));
            CK(hipStreamSynchronize(s2));
        }
        if (w) {
            std::printf("hipEventRecord           %7.2f us/call\n", tr / (kRounds * kBatch));
            std::printf("hipStreamWaitEvent       %7.2f us/call\n", tw / (kRounds * kBatch));
        }
    }
    // the pattern of a frame: wait, graph(4), record on s; wait, graph(2), record on s2
    {
        hipGraph_t g4, g2;
        hipGraphExec_t x4, x2;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
        for (int i = 0; i < 4; ++i) hipLaunchKernelGGL(k_noop, dim3(64), dim3(256), 0, s, d);
        CK(hipStreamEndCapture(s, &g4));
        CK(hipGraphInstantiate(&x4, g4, nullptr, nullptr, 0));
        CK(hipStreamBeginCapture(s2, hipStreamCaptureModeRelaxed));
        for (int i = 0; i < 6; ++i) hipLaunchKernelGGL(k_noop, dim3(64), dim3(256), 0, s2, d);
        CK(hipStreamEndCapture(s2, &g2));
        CK(hipGraphInstantiate(&x2, g2, nullptr, nullptr, 0));
        hipEvent_t e1, e2;
        CK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&e2, hipEventDisableTiming));
        double tot = 0;
        for (int w = 0; w < 2; ++w) {
            tot = 0;
            for (int r = 0; r < kRounds; ++r) {
                auto t0 = clk::now();
                for (int i = 0; i < 12; ++i) {
                    CK(hipStreamWaitEvent(s, e2, 0));
                    CK(hipGraphLaunch(x4, s));
                    CK(hipEventRecord(e1, s));
                    CK(hipStreamWaitEvent(s2, e1, 0));
                    CK(hipGraphLaunch(x2, s2));
                    CK(hipEventRecord(e2, s2));
                }
                tot += us_since(t0);
                CK(hipStreamSynchronize(s));
                CK(hipStreamSynchronize(s2));
            }
        }
        std::printf("frame pattern (4+6 nodes, 2 waits, 2 records) %7.2f us/frame\n", tot / (kRounds * 12));
    }
    return 0;
}
