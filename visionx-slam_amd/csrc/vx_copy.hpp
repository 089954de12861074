// vx_copy.hpp — several device-to-device copies in one launch.  A plan build's small table copies
// each cost a blit launch of ~3.5 us on the stream and ~7 us of host API time (rocprofv3,
// profiles/r04/sba_plan); one k_multi_copy replaces a list of them.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

namespace vx {
namespace {
constexpr int kMaxCopies = 16;
struct CopyList {
    const void* src[kMaxCopies];
    void* dst[kMaxCopies];
    unsigned long long bytes[kMaxCopies];  // multiples of 4; src / dst 4-byte aligned (16: vector copies)
    int n;
};

__global__ __launch_bounds__(256) void k_multi_copy(CopyList L) {
    const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x, nt = (size_t)gridDim.x * 256;
    for (int i = 0; i < L.n; ++i) {
        const bool v16 = ((reinterpret_cast<uintptr_t>(L.src[i]) | reinterpret_cast<uintptr_t>(L.dst[i])) & 15) == 0;
        const size_t q = v16 ? L.bytes[i] / 16 : 0;
        const uint4* s4 = static_cast<const uint4*>(L.src[i]);
        uint4* d4 = static_cast<uint4*>(L.dst[i]);
        for (size_t k = t; k < q; k += nt) d4[k] = s4[k];
        const size_t w0 = q * 4, w1 = L.bytes[i] / 4;
        const uint32_t* s = static_cast<const uint32_t*>(L.src[i]);
        uint32_t* d = static_cast<uint32_t*>(L.dst[i]);
        for (size_t k = w0 + t; k < w1; k += nt) d[k] = s[k];
    }
}

// builder: add() up to kMaxCopies copies (zero-byte ones skipped), then launch() on a stream
struct MultiCopy {
    CopyList L{};
    size_t total = 0;
    bool add(void* dst, const void* src, size_t bytes) {
        if (!bytes) return true;
        if (L.n >= kMaxCopies || (bytes & 3) || ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 3))
            return false;
        L.src[L.n] = src;
        L.dst[L.n] = dst;
        L.bytes[L.n] = bytes;
        ++L.n;
        total += bytes;
        return true;
    }
    hipError_t launch(hipStream_t s) const {
        if (!L.n) return hipSuccess;
        const unsigned blocks = (unsigned)std::min<size_t>(1024, std::max<size_t>(1, (total / 16 + 255) / 256));
        hipLaunchKernelGGL(k_multi_copy, dim3(blocks), dim3(256), 0, s, L);
        return hipGetLastError();
    }
};
}  // namespace
}  // namespace vx
