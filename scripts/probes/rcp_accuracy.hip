// v_rcp_f64 / v_rsq_f64 accuracy with 0, 1, 2 Newton steps, in ulps of the correctly rounded result
// (the BA kernels' frcp / frsq use two steps).  hipcc --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>
__global__ void k(const double* x, double* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double b = x[i];
    double r = __builtin_amdgcn_rcp(b);
    out[6 * i] = r;
    r = fma(fma(-b, r, 1.0), r, r);
    out[6 * i + 1] = r;
    r = fma(fma(-b, r, 1.0), r, r);
    out[6 * i + 2] = r;
    double s = __builtin_amdgcn_rsq(b);
    const double hx = 0.5 * b;
    out[6 * i + 3] = s;
    s = s * fma(-hx * s, s, 1.5);
    out[6 * i + 4] = s;
    s = s * fma(-hx * s, s, 1.5);
    out[6 * i + 5] = s;
}
int main() {
    const int n = 1 << 20;
    std::vector<double> x(n), o(6 * (size_t)n);
    std::mt19937_64 g(1);
    std::uniform_real_distribution<double> u(-30.0, 30.0);
    for (auto& v : x) v = std::exp2(u(g)) * (1.0 + 0.5 * std::generate_canonical<double, 53>(g));
    double *dx, *dout;
    hipMalloc(&dx, n * 8);
    hipMalloc(&dout, 6 * (size_t)n * 8);
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dx, dout, n);
    hipMemcpy(o.data(), dout, 6 * (size_t)n * 8, hipMemcpyDeviceToHost);
    double worst[6] = {0};
    for (int i = 0; i < n; ++i) {
        const double rr = 1.0 / x[i], rs = 1.0 / std::sqrt(x[i]);
        for (int j = 0; j < 6; ++j) {
            const double ref = j < 3 ? rr : rs;
            const double e = std::fabs(o[6 * (size_t)i + j] - ref) / (std::nextafter(std::fabs(ref), INFINITY) - std::fabs(ref));
            if (e > worst[j]) worst[j] = e;
        }
    }
    printf("rcp: 0 steps %.3g ulp, 1 step %.3g, 2 steps %.3g\n", worst[0], worst[1], worst[2]);
    printf("rsq: 0 steps %.3g ulp, 1 step %.3g, 2 steps %.3g\n", worst[3], worst[4], worst[5]);
    return 0;
}
