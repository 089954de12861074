// Does a captured multi-stream graph (fork / join through events) run its branches concurrently
// on this runtime, and what does its launch cost on the host?  Two / four branches of one ~50 us
// spinning kernel each, against the same kernels back to back; then a 4-branch graph of 150 small
// nodes with cross-branch edges (the shape of a 12-frame pipeline step).
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

// one workgroup spinning on the shader clock for `cycles` (s_memtime: a scalar read, no store)
__global__ void k_spin(long long cycles, int* p) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) {
    }
    if (threadIdx.x == 0 && p[0] == 12345) p[1] = 1;
}
__global__ void k_noop(int* p) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345) p[1] = 1;
}

using clk = std::chrono::steady_clock;
static double us_since(clk::time_point t0) { return std::chrono::duration<double, std::micro>(clk::now() - t0).count(); }

int main() {
    int* d;
    CK(hipMalloc(&d, 64));
    CK(hipMemset(d, 0, 64));
    std::vector<hipStream_t> st(4);
    for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<hipEvent_t> ev(8);
    for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    const long long cyc = 100000;  // ~50 us at ~2 GHz
    // reference: one spin kernel, and two back to back on one stream
    auto time_stream = [&](int n) {
        double best = 1e30;
        for (int r = 0; r < 20; ++r) {
            auto t0 = clk::now();
            for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, st[0], cyc, d);
            CK(hipStreamSynchronize(st[0]));
            best = std::min(best, us_since(t0));
        }
        return best;
    };
    std::printf("1 spin kernel, one stream          %8.1f us\n", time_stream(1));
    std::printf("2 spin kernels back to back        %8.1f us\n", time_stream(2));
    for (int nb : {2, 4}) {
        hipGraph_t g;
        hipGraphExec_t x;
        CK(hipStreamBeginCapture(st[0], hipStreamCaptureModeRelaxed));
        CK(hipEventRecord(ev[0], st[0]));
        for (int b = 1; b < nb; ++b) CK(hipStreamWaitEvent(st[b], ev[0], 0));
        for (int b = 0; b < nb; ++b) hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, st[b], cyc, d);
        for (int b = 1; b < nb; ++b) {
            CK(hipEventRecord(ev[b], st[b]));
            CK(hipStreamWaitEvent(st[0], ev[b], 0));
        }
        CK(hipStreamEndCapture(st[0], &g));
        CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
        double best = 1e30;
        for (int r = 0; r < 20; ++r) {
            auto t0 = clk::now();
            CK(hipGraphLaunch(x, st[0]));
            CK(hipStreamSynchronize(st[0]));
            best = std::min(best, us_since(t0));
        }
        std::printf("graph, %d branches of 1 spin kernel %8.1f us\n", nb, best);
        CK(hipGraphExecDestroy(x));
        CK(hipGraphDestroy(g));
    }
    // a 12-frame step: 3 extraction branches (4 nodes per frame) and one BA branch (6 nodes per
    // frame) with cross-branch edges per frame
    {
        hipGraph_t g;
        hipGraphExec_t x;
        std::vector<hipEvent_t> fe(12), fm(12);
        for (auto& e : fe) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        CK(hipStreamBeginCapture(st[0], hipStreamCaptureModeRelaxed));
        CK(hipEventRecord(ev[0], st[0]));
        for (int b = 1; b < 4; ++b) CK(hipStreamWaitEvent(st[b], ev[0], 0));
        for (int i = 0; i < 12; ++i) {
            hipStream_t se = st[i % 3];
            for (int k = 0; k < 4; ++k) hipLaunchKernelGGL(k_noop, dim3(64), dim3(256), 0, se, d);
            CK(hipEventRecord(fe[i], se));
            CK(hipStreamWaitEvent(st[3], fe[i], 0));
            for (int k = 0; k < 6; ++k) hipLaunchKernelGGL(k_noop, dim3(64), dim3(256), 0, st[3], d);
        }
        for (int b = 1; b < 4; ++b) {
            CK(hipEventRecord(ev[b], st[b]));
            CK(hipStreamWaitEvent(st[0], ev[b], 0));
        }
        CK(hipStreamEndCapture(st[0], &g));
        CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
        size_t nn = 0;
        CK(hipGraphGetNodes(g, nullptr, &nn));
        double host = 0, wall = 1e30;
        for (int r = 0; r < 30; ++r) {
            auto t0 = clk::now();
            CK(hipGraphLaunch(x, st[0]));
            const double h = us_since(t0);
            CK(hipStreamSynchronize(st[0]));
            if (r >= 10) host += h;
            wall = std::min(wall, us_since(t0));
        }
        std::printf("12-frame step graph (%zu nodes): host %.1f us per launch, launch-to-done %.1f us\n", nn,
                    host / 20, wall);
    }
    return 0;
}
