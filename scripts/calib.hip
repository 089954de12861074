// calib.hip — latency calibration probes for the MI355X (not part of the library).
//   empty kernel duration vs grid size; dependent global-load chain (L2-resident / HBM);
//   FP64 dependent FMA chain; LDS round trip.  Prints one line per probe (µs from hipEvents
//   over 200 back-to-back launches, so per-launch numbers include the launch boundary).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            return 1;                                                           \
        }                                                                       \
    } while (0)

__global__ void k_empty(int* p) {
    if (threadIdx.x == 0 && blockIdx.x == 0x7fffffff) p[0] = 1;
}

// one lane per block chases a pointer chain of n hops; the time per hop = dependent load latency
__global__ void k_chase(const unsigned* __restrict__ nxt, int n, unsigned* out) {
    if (threadIdx.x) return;
    unsigned i = blockIdx.x * 64;
    for (int k = 0; k < n; ++k) i = nxt[i];
    if (i == 0xffffffffu) out[0] = i;
}

__global__ void k_fma64(double* out, int n) {
    double x = threadIdx.x * 1e-3, y = 1.0000001;
    for (int k = 0; k < n; ++k) x = fma(x, y, 1e-9);
    if (x == 12345.0) out[0] = x;
}

__global__ void k_lds(int* out, int n) {
    __shared__ int s[1024];
    s[threadIdx.x] = threadIdx.x;
    __syncthreads();
    int i = threadIdx.x;
    for (int k = 0; k < n; ++k) i = s[(i * 7 + 1) & 1023];
    if (i == -1) out[0] = i;
}

__global__ void k_sync(int* out, int n) {
    __shared__ int s[1024];
    int v = threadIdx.x;
    for (int k = 0; k < n; ++k) {
        s[threadIdx.x] = v;
        __syncthreads();
        v += s[(threadIdx.x + 1) & (blockDim.x - 1)];
        __syncthreads();
    }
    if (v == -1) out[0] = v;
}

template <class F>
static float time_us(F launch, int reps = 200) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 10; ++i) launch();
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i) launch();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms * 1e3f / reps;
}

int main() {
    int* d_out;
    CK(hipMalloc(&d_out, 64));
    for (int g : {1, 64, 256, 1024, 4096})
        printf("empty       grid %5d x 256 : %7.2f us/launch\n", g,
               time_us([&] { hipLaunchKernelGGL(k_empty, dim3(g), dim3(256), 0, 0, d_out); }));
    // pointer chains: small (L2-resident, 256 KB) and large (1 GB, HBM) random cycles
    for (size_t n : {size_t(64) << 10, size_t(256) << 20}) {
        std::vector<unsigned> h(n);
        unsigned long long s = 88172645463325252ull;
        std::vector<unsigned> perm(n);
        for (size_t i = 0; i < n; ++i) perm[i] = (unsigned)i;
        for (size_t i = n - 1; i > 0; --i) {
            s ^= s << 13; s ^= s >> 7; s ^= s << 17;
            std::swap(perm[i], perm[s % (i + 1)]);
        }
        for (size_t i = 0; i < n; ++i) h[perm[i]] = perm[(i + 1) % n];
        unsigned* d;
        CK(hipMalloc(&d, n * 4));
        CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
        for (int hops : {1, 16, 64}) {
            const float t = time_us([&] { hipLaunchKernelGGL(k_chase, dim3(64), dim3(64), 0, 0, d, hops, (unsigned*)d_out); }, 50);
            printf("chase %6zu KB hops %3d   : %7.2f us/launch\n", n * 4 >> 10, hops, t);
        }
        CK(hipFree(d));
    }
    for (int n : {1, 256, 4096})
        printf("fma64 chain %5d          : %7.2f us/launch\n", n,
               time_us([&] { hipLaunchKernelGGL(k_fma64, dim3(256), dim3(256), 0, 0, (double*)d_out, n); }));
    for (int n : {1, 256, 4096})
        printf("lds chain %5d            : %7.2f us/launch\n", n,
               time_us([&] { hipLaunchKernelGGL(k_lds, dim3(256), dim3(1024), 0, 0, d_out, n); }));
    for (int n : {1, 64, 512})
        printf("syncthreads x2 %4d (1024): %7.2f us/launch\n", n,
               time_us([&] { hipLaunchKernelGGL(k_sync, dim3(256), dim3(1024), 0, 0, d_out, n); }));
    CK(hipDeviceSynchronize());
    return 0;
}
