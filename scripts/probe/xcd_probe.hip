// Which XCD (XCC_ID) and CU (HW_ID) the workgroups of a stream with a given CU mask run on: the
// mapping of hipExtStreamCreateWithCUMask bits to XCDs on this device (for keeping LocalBA's L2s free
// of the extraction streams).  Reads hardware registers with s_getreg only; results through vector
// stores.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>

__global__ void probe(unsigned* out) {
    if (threadIdx.x == 0) {
        const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
        out[2 * blockIdx.x] = xcc;
        out[2 * blockIdx.x + 1] = hw;
    }
    // keep the workgroup resident a little so the dispatcher spreads the grid
    for (volatile int i = 0; i < 2000; ++i) {
    }
}

static void run(const char* name, const std::vector<int>& cus, int ncu) {
    std::vector<uint32_t> mask((ncu + 31) / 32, 0);
    for (int c : cus) mask[c / 32] |= 1u << (c % 32);
    hipStream_t s;
    if (cus.empty()) {
        if (hipStreamCreate(&s) != hipSuccess) exit(1);
    } else if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
        exit(1);
    }
    const int nb = 2048;
    unsigned* d;
    if (hipMalloc(&d, nb * 8) != hipSuccess) exit(1);
    hipLaunchKernelGGL(probe, dim3(nb), dim3(64), 0, s, d);
    std::vector<unsigned> h(2 * nb);
    if (hipMemcpyAsync(h.data(), d, nb * 8, hipMemcpyDeviceToHost, s) != hipSuccess) exit(1);
    if (hipStreamSynchronize(s) != hipSuccess) exit(1);
    std::set<unsigned> xccs;
    std::set<std::pair<unsigned, unsigned>> units;  // (xcc, se/sh/cu bits)
    for (int b = 0; b < nb; ++b) {
        xccs.insert(h[2 * b] & 0xf);
        units.insert({h[2 * b] & 0xf, (h[2 * b + 1] >> 8) & 0xff});
    }
    printf("%-22s xcds {", name);
    for (unsigned x : xccs) printf(" %u", x);
    printf(" }  distinct (xcd, se/sh/cu) %zu\n", units.size());
    (void)hipFree(d);
    (void)hipStreamDestroy(s);
}

int main() {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 1;
    printf("CUs %d\n", ncu);
    run("all", {}, ncu);
    auto range = [](int a, int b, int st) {
        std::vector<int> v;
        for (int i = a; i < b; i += st) v.push_back(i);
        return v;
    };
    run("bits 0..31", range(0, 32, 1), ncu);
    run("bits 32..63", range(32, 64, 1), ncu);
    run("bits 0..7", range(0, 8, 1), ncu);
    run("every 8th from 0", range(0, ncu, 8), ncu);
    run("every 8th from 1", range(1, ncu, 8), ncu);
    run("bits 0..127", range(0, 128, 1), ncu);
    run("bits 128..255", range(128, ncu, 1), ncu);
    for (int x = 0; x < 8; ++x) {
        char nm[32];
        snprintf(nm, sizeof nm, "bit 8k+%d", x);
        run(nm, range(x, ncu, 8), ncu);
    }
    return 0;
}
