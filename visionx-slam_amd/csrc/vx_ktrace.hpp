// vx_ktrace.hpp — in-kernel phase timestamps for the trace build only (make trace ->
// lib/libvxslam_trace.so, -DVX_KTRACE).  VX_KT(slot) drains this wave's outstanding memory
// operations (s_waitcnt 0, so a phase's loads are charged to it), then lane 0 of workgroups
// < kKtBlocks records wall_clock64() (100 MHz) into the TU's trace table.  The product library
// compiles every VX_KT to nothing.
#pragma once

namespace vx {
constexpr int kKtBlocks = 256, kKtSlots = 16;
}

#ifdef VX_KTRACE
// table: [block][slot] wall_clock64, then [block][slot] s_memtime (shader clock cycles)
#define VX_KT_TABLE() __device__ long long g_ktrace[2 * vx::kKtBlocks * vx::kKtSlots]
#define VX_KT(slot)                                                                        \
    do {                                                                                   \
        __builtin_amdgcn_s_waitcnt(0);                                                     \
        const unsigned kt_b = blockIdx.x + blockIdx.y * gridDim.x; /* linear workgroup */  \
        if (threadIdx.x == 0 && kt_b < (unsigned)vx::kKtBlocks) {                          \
            g_ktrace[kt_b * vx::kKtSlots + (slot)] = (long long)wall_clock64();            \
            g_ktrace[(vx::kKtBlocks + kt_b) * vx::kKtSlots + (slot)] =                     \
                (long long)__builtin_amdgcn_s_memtime();                                   \
        }                                                                                  \
    } while (0)
// per wave: lane 0 of wave w records slot (base + w), for w < nw
#define VX_KTW(base, nw)                                                                   \
    do {                                                                                   \
        __builtin_amdgcn_s_waitcnt(0);                                                     \
        const unsigned kt_b = blockIdx.x + blockIdx.y * gridDim.x;                         \
        const unsigned kt_w = threadIdx.x >> 6;                                            \
        if ((threadIdx.x & 63) == 0 && kt_w < (unsigned)(nw) && kt_b < (unsigned)vx::kKtBlocks) \
            g_ktrace[kt_b * vx::kKtSlots + (base) + kt_w] = (long long)wall_clock64();     \
    } while (0)
#define VX_KT_EXPORT(name)                                                                 \
    extern "C" int name(long long* out) {                                                  \
        return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ktrace), sizeof(g_ktrace)) == hipSuccess ? 0 : -1; \
    }
// pass log (workgroup 0 only): entry i = (wall_clock64, tag); VX_KP_TABLE / VX_KP(tag) /
// VX_KP_EXPORT(name), entry 0 holds the count
#define VX_KP_TABLE() __device__ long long g_kpass[2 * 512]
#define VX_KP(tag)                                                                         \
    do {                                                                                   \
        __builtin_amdgcn_s_waitcnt(0);                                                     \
        if (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0) {   \
            const int kp_i = (int)g_kpass[0] + 1;                                          \
            if (kp_i < 512) {                                                              \
                g_kpass[2 * kp_i] = (long long)wall_clock64();                             \
                g_kpass[2 * kp_i + 1] = (long long)(tag);                                  \
                g_kpass[0] = kp_i;                                                         \
            }                                                                              \
        }                                                                                  \
    } while (0)
#define VX_KP_RESET()                                                                      \
    do {                                                                                   \
        if (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0) g_kpass[0] = 0; \
    } while (0)
#define VX_KP_EXPORT(name)                                                                 \
    extern "C" int name(long long* out) {                                                  \
        return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_kpass), sizeof(g_kpass)) == hipSuccess ? 0 : -1; \
    }
#else
#define VX_KP_TABLE() static_assert(true, "")
#define VX_KP(tag) \
    do {           \
    } while (0)
#define VX_KP_RESET() \
    do {              \
    } while (0)
#define VX_KP_EXPORT(name) static_assert(true, "")
#define VX_KT_TABLE() static_assert(true, "")
#define VX_KT(slot) \
    do {            \
    } while (0)
#define VX_KTW(base, nw) \
    do {                 \
    } while (0)
#define VX_KT_EXPORT(name) static_assert(true, "")
#endif
