// Probe: cost of a device-wide barrier among co-resident workgroups on gfx950 (atomic arrival
// counter + generation flag, agent-scope fences), against back-to-back dependent launches.
// Every spin is bounded (no hang possible): a timed-out wait sets an error flag.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/grid_barrier_probe.hip -o build/grid_barrier_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ bool grid_sync(unsigned* count, volatile unsigned* gen, unsigned nblocks, int* err) {
    __syncthreads();
    bool ok = true;
    if (threadIdx.x == 0) {
        const unsigned g = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __atomic_thread_fence(__ATOMIC_RELEASE);  // this block's writes before the arrival
        const unsigned arrived = __hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (arrived == nblocks - 1) {
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store((unsigned*)gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            long spins = 0;
            while (__hip_atomic_load((unsigned*)gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > 20000000) { atomicOr(err, 1); ok = false; break; }
            }
        }
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
    }
    __syncthreads();
    return ok;
}

__global__ void k_barriers(unsigned* count, unsigned* gen, int n, int* err, double* data) {
    for (int i = 0; i < n; ++i) {
        data[blockIdx.x * blockDim.x + threadIdx.x] += 1.0;
        if (!grid_sync(count, gen, gridDim.x, err)) return;
    }
}

__global__ void k_step(double* data) { data[blockIdx.x * blockDim.x + threadIdx.x] += 1.0; }

int main() {
    unsigned *count, *gen;
    int* err;
    double* data;
    hipMalloc(&count, 4); hipMalloc(&gen, 4); hipMalloc(&err, 4);
    hipMalloc(&data, 1024 * 1024 * 8);
    hipMemset(count, 0, 4); hipMemset(gen, 0, 4); hipMemset(err, 0, 4);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int blocks : {32, 128, 200, 256}) {
        const int n = 100;
        hipLaunchKernelGGL(k_barriers, dim3(blocks), dim3(512), 0, 0, count, gen, 10, err, data);
        hipEventRecord(a);
        hipLaunchKernelGGL(k_barriers, dim3(blocks), dim3(512), 0, 0, count, gen, n, err, data);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        int e = 0; hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
        // the same number of dependent steps as separate launches, captured in one graph
        hipStream_t s; hipStreamCreate(&s);
        hipGraph_t g; hipGraphExec_t ge;
        hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
        for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_step, dim3(blocks), dim3(512), 0, s, data);
        hipStreamEndCapture(s, &g);
        hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        hipGraphLaunch(ge, s); hipStreamSynchronize(s);
        hipEventRecord(a, s); hipGraphLaunch(ge, s); hipEventRecord(b, s); hipEventSynchronize(b);
        float ms2; hipEventElapsedTime(&ms2, a, b);
        printf("%4d workgroups x 512: grid barrier %.3f us each (err %d); dependent launch in a graph %.3f us each\n",
               blocks, 1e3 * ms / n, e, 1e3 * ms2 / n);
        hipGraphExecDestroy(ge); hipGraphDestroy(g); hipStreamDestroy(s);
    }
    return 0;
}
