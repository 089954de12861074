// ransac.hip — PnP RANSAC for Tracking::TrackWithPnP.
//
// Replaces cv::solvePnPRansac(pts_3d, pts_2d, K, noArray(), rvec, tvec, false, iterations,
// max_reproj_error, 0.99, inliers) (core/frontend/tracking.cpp:414-423).  OpenCV's loop
// (RANSACPointSetRegistrator::run) draws one sample, solves, scores, maybe shrinks its iteration
// budget, repeats.  Here every hypothesis of the budget is drawn, solved and scored at once — one
// workgroup per (hypothesis, problem), the scoring pass reading the problem's correspondences
// (20 B each) from L2 — and the sequential loop is then replayed over the per-hypothesis inlier
// counts in hypothesis order (one thread, <= 4096 steps of integer compares and the
// RANSACUpdateNumIters formula), so the kept model and the reported iteration count are exactly
// those of a sequential run over the same hypothesis stream.  The kept model's inliers are then
// refined by Levenberg-Marquardt in one workgroup (solvePnPRansac's SOLVEPNP_ITERATIVE refit).
//
//   k_pnp_hyp     grid (H, problems)  sample 4 (splitmix64 counter stream), P3P (Grunert quartic,
//                                     real roots by derivative-isolated brackets + safeguarded
//                                     Newton), 4th-point choice, inlier count
//   k_pnp_refine  grid (problems)     sequential replay -> kept model, inlier mask, LM refit
//
// The hypothesis stage uses only + - * / and sqrt in a fixed order (-ffp-contract=off), so its
// models, counts, the kept hypothesis and the mask are bit-identical to the CPU restatement
// (oracle/ransac_oracle.cpp, the specification); the LM refit matches it to rounding.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "vx_internal.hpp"
#include "ba_common.hpp"

namespace vx {
namespace {

using namespace vx::ba;

constexpr int kThreads = 256;
constexpr int kMaxHyp = 4096;

struct HypRec {
    double R[9], t[3];
    int valid, count;
};

struct PnpArgs {
    const int* offsets;           // P + 1
    const double* intr;           // 4 per problem
    const vx_pnp_options* opt;    // per problem
    const float* obj;             // 3 per correspondence
    const float* img;             // 2 per correspondence
    HypRec* hyp;                  // [P][hmax]
    int hmax;
    vx_pnp_result* out;           // per problem
    uint8_t* mask;                // per correspondence
};

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

// ---------------------------------------------------------------- real polynomial roots (d <= 4)
// Degrees are template parameters and every small array is indexed by unrolled compile-time
// indices (get / put below), so coefficients, brackets and roots stay in VGPRs: with runtime
// degrees the arrays went to scratch and every Newton step paid a scratch round trip.
template <int N>
__device__ __forceinline__ double get(const double (&a)[N], int i) {
    double r = a[0];
#pragma unroll
    for (int k = 1; k < N; ++k)
        if (k == i) r = a[k];
    return r;
}
template <int N>
__device__ __forceinline__ void put(double (&a)[N], int i, double x) {
#pragma unroll
    for (int k = 0; k < N; ++k)
        if (k == i) a[k] = x;
}

template <int D>
__device__ __forceinline__ double peval(const double* c, double x) {
    double v = c[D];
#pragma unroll
    for (int k = D - 1; k >= 0; --k) v = v * x + c[k];
    return v;
}
template <int D>
__device__ __forceinline__ double pderiv(const double* c, double x) {
    double v = (double)D * c[D];
#pragma unroll
    for (int k = D - 1; k >= 1; --k) v = v * x + (double)k * c[k];
    return v;
}

// monotone bracket with a sign change, plo = p(lo) != 0: safeguarded Newton
template <int D>
__device__ double bracket_root(const double* c, double lo, double hi, double plo) {
    double x = 0.5 * (lo + hi);
    for (int it = 0; it < 100; ++it) {
        const double px = peval<D>(c, x);
        if (px == 0.0) return x;
        if ((px < 0.0) == (plo < 0.0)) lo = x;
        else hi = x;
        const double dp = pderiv<D>(c, x);
        double xn = x - px / dp;
        if (!(xn > lo && xn < hi)) xn = 0.5 * (lo + hi);
        if (fabs(xn - x) <= 4.440892098500626e-16 * fabs(xn)) return xn;
        x = xn;
    }
    return x;
}

// closed form for degree D <= 2 with c[D] != 0
template <int D>
__device__ __forceinline__ int roots_low(const double* c, double (&out)[4]) {
    if constexpr (D <= 0) {
        return 0;
    } else if constexpr (D == 1) {
        out[0] = -c[0] / c[1];
        return 1;
    } else {
        const double disc = c[1] * c[1] - 4.0 * c[2] * c[0];
        if (disc < 0.0) return 0;
        const double sq = sqrt(disc);
        const double q = -0.5 * (c[1] + (c[1] >= 0.0 ? sq : -sq));
        if (q == 0.0) {
            out[0] = 0.0;
            return 1;
        }
        double r1 = q / c[2], r2 = c[0] / q;
        if (r2 < r1) {
            const double tmp = r1;
            r1 = r2;
            r2 = tmp;
        }
        out[0] = r1;
        if (r2 == r1) return 1;
        out[1] = r2;
        return 2;
    }
}

template <int D>
__device__ int real_roots_t(const double* c, double (&out)[4], double (&crit_out)[4], int* n_crit);

// degree D (>= 3, c[D] != 0) roots from the ascending critical points crit[0..nc): intervals
// [-B, crit...(inside (-B, B)), B] with the Cauchy bound B, one bracketed root per sign change
template <int D>
__device__ int roots_from_crit(const double* c, const double (&crit)[4], int nc, double (&out)[4]) {
    double B = 0.0;
#pragma unroll
    for (int k = 0; k < D; ++k) B = fmax(B, fabs(c[k] / c[D]));
    B = 1.0 + B;
    int nr = 0;
    double a = -B;
    auto interval = [&](double b) {
        if (!(a < b)) return;
        const double pa = peval<D>(c, a), pb = peval<D>(c, b);
        if (pa == 0.0) {
            if (nr == 0 || get(out, nr - 1) != a) put(out, nr++, a);
        } else if (pb != 0.0 && ((pa < 0.0) != (pb < 0.0))) {
            put(out, nr++, bracket_root<D>(c, a, b, pa));
        }
    };
#pragma unroll
    for (int k = 0; k < D - 1; ++k) {
        if (k < nc && crit[k] > -B && crit[k] < B) {
            interval(crit[k]);
            a = crit[k];
        }
    }
    interval(B);
    return nr;
}

// real roots (ascending) of c[0] + ... + c[D] x^D, trailing zero coefficients dropped; for an
// effective degree >= 3 also its critical points (roots of p')
template <int D>
__device__ int real_roots_t(const double* c, double (&out)[4], double (&crit_out)[4], int* n_crit) {
    *n_crit = 0;
    if constexpr (D <= 0) {
        return 0;
    } else {
        if (c[D] == 0.0) return real_roots_t<D - 1>(c, out, crit_out, n_crit);
        if constexpr (D <= 2) {
            return roots_low<D>(c, out);
        } else {
            double dc[D];
#pragma unroll
            for (int k = 0; k < D; ++k) dc[k] = (double)(k + 1) * c[k + 1];
            double crit[4], unused[4];
            int nu;
            const int nc = real_roots_t<D - 1>(dc, crit, unused, &nu);
#pragma unroll
            for (int k = 0; k < 4; ++k) crit_out[k] = crit[k];
            *n_crit = nc;
            return roots_from_crit<D>(c, crit, nc, out);
        }
    }
}

// ---------------------------------------------------------------- P3P (Grunert)
__device__ __forceinline__ D3 sub3(D3 a, D3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ double dot3(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ D3 unit3(D3 a) {
    const double inv = 1.0 / sqrt(dot3(a, a));
    return {a.x * inv, a.y * inv, a.z * inv};
}
__device__ __forceinline__ D3 scl3(D3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }

struct Model {
    double R[9], t[3];
};

__device__ __forceinline__ D3 apply_model(const double* R, const double* t, D3 p) {
    return {R[0] * p.x + R[1] * p.y + R[2] * p.z + t[0], R[3] * p.x + R[4] * p.y + R[5] * p.z + t[1],
            R[6] * p.x + R[7] * p.y + R[8] * p.z + t[2]};
}

__device__ __forceinline__ bool reproj_sq(const double* R, const double* t, D3 p, double u, double v,
                                          const double* cam, double* err) {
    const D3 pc = apply_model(R, t, p);
    if (!(pc.z > 0.0)) return false;
    const double iz = 1.0 / pc.z;
    const double du = cam[0] * (pc.x * iz) + cam[2] - u;
    const double dv = cam[1] * (pc.y * iz) + cam[3] - v;
    *err = du * du + dv * dv;
    return true;
}

// candidate depth ratios v = s2 / s0 of Grunert's quartic: its real roots, then the local minima
// of |p| that stay off zero (a double root that measurement noise split into a complex pair)
template <int D>
__device__ int p3p_candidates(const double* A, double (&cand)[8]) {
    double roots[4], crit[4];
    int nc = 0;
    const int nr = real_roots_t<D>(A, roots, crit, &nc);
    int m = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (k < nr) put(cand, m++, roots[k]);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        if (k < nc) {
            const double pc = peval<D>(A, crit[k]);
            double d2 = 0.0;
#pragma unroll
            for (int j = D; j >= 2; --j) d2 = d2 * crit[k] + (double)(j * (j - 1)) * A[j];
            if (pc != 0.0 && ((pc > 0.0) == (d2 > 0.0)) && d2 != 0.0) put(cand, m++, crit[k]);
        }
    }
    return m;
}

// P3P on P[0..2] / unit bearings f[0..2]; among the solutions the one reprojecting (P3 -> uv3)
// best is kept (strictly smaller squared error, candidate order).  False when none qualifies.
__device__ bool p3p_best(const D3* P, const D3* f, D3 P3, double u3, double v3, const double* cam, Model* best) {
    const D3 d12 = sub3(P[1], P[2]), d02 = sub3(P[0], P[2]), d01 = sub3(P[0], P[1]);
    const double a2 = dot3(d12, d12), b2 = dot3(d02, d02), c2 = dot3(d01, d01);
    if (!(a2 > 0.0 && b2 > 0.0 && c2 > 0.0)) return false;
    const double ca = dot3(f[1], f[2]), cb = dot3(f[0], f[2]), cg = dot3(f[0], f[1]);
    const double amc = (a2 - c2) / b2, apc = (a2 + c2) / b2, c2b = c2 / b2, a2b = a2 / b2;
    const double bmc = (b2 - c2) / b2, bma = (b2 - a2) / b2;
    double A[5];
    A[4] = (amc - 1.0) * (amc - 1.0) - 4.0 * c2b * ca * ca;
    A[3] = 4.0 * (amc * (1.0 - amc) * cb - (1.0 - apc) * ca * cg + 2.0 * c2b * ca * ca * cb);
    A[2] = 2.0 * (amc * amc - 1.0 + 2.0 * amc * amc * cb * cb + 2.0 * bmc * ca * ca - 4.0 * apc * ca * cb * cg +
                  2.0 * bma * cg * cg);
    A[1] = 4.0 * (-amc * (1.0 + amc) * cb + 2.0 * a2b * cg * cg * cb - (1.0 - apc) * ca * cg);
    A[0] = (1.0 + amc) * (1.0 + amc) - 4.0 * a2b * cg * cg;
    double scale = 0.0;
#pragma unroll
    for (int k = 0; k < 5; ++k) scale = fmax(scale, fabs(A[k]));
    if (!(scale > 0.0)) return false;
    double cand[8];
    const int m = fabs(A[4]) <= 1e-12 * scale ? p3p_candidates<3>(A, cand) : p3p_candidates<4>(A, cand);
    const D3 we1 = unit3(sub3(P[1], P[0]));
    const D3 we3 = unit3(cross3(sub3(P[1], P[0]), sub3(P[2], P[0])));
    const D3 we2 = cross3(we3, we1);
    double best_err = INFINITY;
    bool found = false;
    for (int k = 0; k < m; ++k) {
        const double v = get(cand, k);
        if (!(v > 0.0)) continue;
        const double den = 2.0 * (cg - v * ca);
        if (den == 0.0) continue;
        const double u = ((amc - 1.0) * v * v - 2.0 * amc * cb * v + 1.0 + amc) / den;
        if (!(u > 0.0)) continue;
        const double s0sq = b2 / (1.0 + v * v - 2.0 * v * cb);
        if (!(s0sq > 0.0)) continue;
        const double s0 = sqrt(s0sq);
        const D3 C0 = scl3(f[0], s0), C1 = scl3(f[1], u * s0), C2 = scl3(f[2], v * s0);
        const D3 ce1 = unit3(sub3(C1, C0));
        const D3 ce3 = unit3(cross3(sub3(C1, C0), sub3(C2, C0)));
        const D3 ce2 = cross3(ce3, ce1);
        Model M;
        const double cw[3][3] = {{ce1.x, ce2.x, ce3.x}, {ce1.y, ce2.y, ce3.y}, {ce1.z, ce2.z, ce3.z}};
        const double ww[3][3] = {{we1.x, we2.x, we3.x}, {we1.y, we2.y, we3.y}, {we1.z, we2.z, we3.z}};
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int cc = 0; cc < 3; ++cc)
                M.R[3 * r + cc] = cw[r][0] * ww[cc][0] + cw[r][1] * ww[cc][1] + cw[r][2] * ww[cc][2];
        const D3 rp = {M.R[0] * P[0].x + M.R[1] * P[0].y + M.R[2] * P[0].z,
                       M.R[3] * P[0].x + M.R[4] * P[0].y + M.R[5] * P[0].z,
                       M.R[6] * P[0].x + M.R[7] * P[0].y + M.R[8] * P[0].z};
        M.t[0] = C0.x - rp.x;
        M.t[1] = C0.y - rp.y;
        M.t[2] = C0.z - rp.z;
        double e;
        if (!reproj_sq(M.R, M.t, P3, u3, v3, cam, &e)) continue;
        if (e < best_err) {
            best_err = e;
            *best = M;
            found = true;
        }
    }
    return found;
}

__device__ __forceinline__ D3 world_pt(const float* obj, int i) {
    return {(double)obj[3 * i], (double)obj[3 * i + 1], (double)obj[3 * i + 2]};
}

__device__ __forceinline__ D3 bearing(const float* img, int i, const double* cam) {
    const double x = ((double)img[2 * i] - cam[2]) / cam[0];
    const double y = ((double)img[2 * i + 1] - cam[3]) / cam[1];
    const double inv = 1.0 / sqrt(x * x + y * y + 1.0);
    return {x * inv, y * inv, inv};
}

// hypothesis h of a problem with n correspondences: sample 4 distinct, P3P, 4th-point choice
__device__ bool hypothesis(const float* obj, const float* img, int n, const double* cam, uint64_t seed, int h,
                           Model* best) {
    int i0 = -1, i1 = -1, i2 = -1, i3 = -1;
    int got = 0;
    for (int a = 0; a < 64 && got < 4; ++a) {
        const uint64_t x = mix64(seed + (uint64_t)h * 64u + (uint64_t)a);
        const int i = (int)(((x >> 32) * (uint64_t)n) >> 32);
        if (i == i0 || i == i1 || i == i2) continue;
        if (got == 0) i0 = i;
        else if (got == 1) i1 = i;
        else if (got == 2) i2 = i;
        else i3 = i;
        ++got;
    }
    if (got < 4) return false;
    const D3 P[3] = {world_pt(obj, i0), world_pt(obj, i1), world_pt(obj, i2)};
    const D3 f[3] = {bearing(img, i0, cam), bearing(img, i1, cam), bearing(img, i2, cam)};
    return p3p_best(P, f, world_pt(obj, i3), (double)img[2 * i3], (double)img[2 * i3 + 1], cam, best);
}

__device__ __forceinline__ bool is_inlier(const double* R, const double* t, const float* obj, const float* img, int i,
                                          const double* cam, double thr2) {
    double e;
    return reproj_sq(R, t, world_pt(obj, i), (double)img[2 * i], (double)img[2 * i + 1], cam, &e) && e <= thr2;
}

// block-wide integer sum of per-thread flags (ballot + popcount per wave, LDS atomics)
__device__ __forceinline__ void block_count(int flag, int* lds_cnt) {
    const uint64_t b = __ballot(flag);
    if ((threadIdx.x & 63) == 0) atomicAdd(lds_cnt, __popcll(b));
}

__global__ void __launch_bounds__(kThreads) k_pnp_hyp(PnpArgs a) {
    const int p = blockIdx.y, h = blockIdx.x;
    const vx_pnp_options o = a.opt[p];
    const int H = min(max(o.max_iterations, 0), kMaxHyp);
    if (h >= H) return;
    const int b = a.offsets[p], n = a.offsets[p + 1] - b;
    const float* obj = a.obj + 3 * (size_t)b;
    const float* img = a.img + 2 * (size_t)b;
    double cam[4] = {a.intr[4 * p], a.intr[4 * p + 1], a.intr[4 * p + 2], a.intr[4 * p + 3]};
    __shared__ double sR[9], st[3];
    __shared__ int svalid, scnt;
    if (threadIdx.x == 0) {
        Model M;
        const bool ok = n >= 4 && hypothesis(obj, img, n, cam, o.seed, h, &M);
        svalid = ok ? 1 : 0;
        scnt = 0;
        if (ok) {
            for (int k = 0; k < 9; ++k) sR[k] = M.R[k];
            for (int k = 0; k < 3; ++k) st[k] = M.t[k];
        }
    }
    __syncthreads();
    HypRec* rec = a.hyp + (size_t)p * a.hmax + h;
    if (!svalid) {
        if (threadIdx.x == 0) {
            rec->valid = 0;
            rec->count = 0;
        }
        return;
    }
    double R[9], t[3];
    for (int k = 0; k < 9; ++k) R[k] = sR[k];
    for (int k = 0; k < 3; ++k) t[k] = st[k];
    const double thr2 = o.reproj_error * o.reproj_error;
    for (int i0 = 0; i0 < n; i0 += kThreads) {
        const int i = i0 + threadIdx.x;
        block_count(i < n && is_inlier(R, t, obj, img, i, cam, thr2), &scnt);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 0; k < 9; ++k) rec->R[k] = R[k];
        for (int k = 0; k < 3; ++k) rec->t[k] = t[k];
        rec->valid = 1;
        rec->count = scnt;
    }
}

// RANSACUpdateNumIters for modelPoints = 4
__device__ int update_num_iters(double p, double ep, int max_iters) {
    p = fmax(p, 0.0);
    p = fmin(p, 1.0);
    ep = fmax(ep, 0.0);
    ep = fmin(ep, 1.0);
    double num = fmax(1.0 - p, DBL_MIN);
    const double x = 1.0 - ep;
    double denom = 1.0 - (x * x) * (x * x);
    if (denom < DBL_MIN) return 0;
    num = log(num);
    denom = log(denom);
    return denom >= 0.0 || -num >= (double)max_iters * -denom ? max_iters : (int)rint(num / denom);
}

__device__ void quat_of(const double* R, double* q) {
    const double tr = R[0] + R[4] + R[8];
    double x, y, z, w;
    if (tr > 0.0) {
        const double s = sqrt(tr + 1.0) * 2.0;
        w = 0.25 * s; x = (R[7] - R[5]) / s; y = (R[2] - R[6]) / s; z = (R[3] - R[1]) / s;
    } else if (R[0] > R[4] && R[0] > R[8]) {
        const double s = sqrt(1.0 + R[0] - R[4] - R[8]) * 2.0;
        w = (R[7] - R[5]) / s; x = 0.25 * s; y = (R[1] + R[3]) / s; z = (R[2] + R[6]) / s;
    } else if (R[4] > R[8]) {
        const double s = sqrt(1.0 + R[4] - R[0] - R[8]) * 2.0;
        w = (R[2] - R[6]) / s; x = (R[1] + R[3]) / s; y = 0.25 * s; z = (R[5] + R[7]) / s;
    } else {
        const double s = sqrt(1.0 + R[8] - R[0] - R[4]) * 2.0;
        w = (R[3] - R[1]) / s; x = (R[2] + R[6]) / s; y = (R[5] + R[7]) / s; z = 0.25 * s;
    }
    const double inv = 1.0 / sqrt(x * x + y * y + z * z + w * w);
    q[0] = x * inv; q[1] = y * inv; q[2] = z * inv; q[3] = w * inv;
}

constexpr int kAcc = 28;              // 21 upper-triangle H + 6 g + cost
constexpr int kRefineThreads = 512;   // 8 waves: <= 8 correspondences per thread at n = 4096

// sum over the block of kAcc per-thread values into red[0..kAcc) (fixed order: wave butterflies,
// then the wave partials in wave order)
__device__ void block_reduce(double* v, double* lds /* waves * kAcc */, double* red) {
    constexpr int kWaves = kRefineThreads / 64;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < kAcc; ++k) {
        double x = v[k];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off);
        if (lane == 0) lds[wave * kAcc + k] = x;
    }
    __syncthreads();
    if (threadIdx.x < kAcc) {
        double s = lds[threadIdx.x];
#pragma unroll
        for (int w = 1; w < kWaves; ++w) s += lds[w * kAcc + threadIdx.x];
        red[threadIdx.x] = s;
    }
    __syncthreads();
}

// per-thread partial {H, g, cost} of the masked correspondences at pose T (qx qy qz qw tx ty tz)
__device__ void accumulate(const double* T, const float* obj, const float* img, const uint8_t* mask, int n,
                           const double* cam, double* v) {
#pragma unroll
    for (int k = 0; k < kAcc; ++k) v[k] = 0.0;
    double Tl[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) Tl[k] = T[k];
    for (int i = threadIdx.x; i < n; i += kRefineThreads) {
        if (!mask[i]) continue;
        const D3 pc = se3_apply(Tl, world_pt(obj, i));
        if (pc.z <= 1e-6) continue;  // ProjectToPixel (projection.h:11-31)
        const double iz = 1.0 / pc.z;
        const double e0 = (double)img[2 * i] - (cam[0] * (pc.x * iz) + cam[2]);
        const double e1 = (double)img[2 * i + 1] - (cam[1] * (pc.y * iz) + cam[3]);
        // PoseJacobian (local_ba.cpp:26-33): Jp * [I | -hat(pc)]
        const double z2 = pc.z * pc.z;
        const double jx = cam[0] / pc.z, jxz = -cam[0] * pc.x / z2;
        const double jy = cam[1] / pc.z, jyz = -cam[1] * pc.y / z2;
        const double J0[6] = {jx, 0.0, jxz, jxz * pc.y, jx * pc.z - jxz * pc.x, -jx * pc.y};
        const double J1[6] = {0.0, jy, jyz, -jy * pc.z + jyz * pc.y, -jyz * pc.x, jy * pc.x};
        int k = 0;
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
            for (int c = r; c < 6; ++c) v[k++] += J0[r] * J0[c] + J1[r] * J1[c];
#pragma unroll
        for (int r = 0; r < 6; ++r) v[21 + r] += J0[r] * e0 + J1[r] * e1;
        v[27] += e0 * e0 + e1 * e1;
    }
}

// RANSACPointSetRegistrator::run's loop replayed by wave 0 over the hypothesis records, 64 at a
// time: a hypothesis can only be kept if its count beats every earlier count and 3 (an in-wave
// prefix max + ballot finds those "records"); the records are then walked in order, each shrinking
// the iteration budget, until one lies beyond the budget.  Returns {kept, hypotheses run, count}.
__device__ int3 replay(const HypRec* rec, int H, int n, double confidence) {
    const int lane = threadIdx.x & 63;
    int niters = n >= 4 ? H : 0, best = -1, good = 0;
    for (int base = 0; base < niters; base += 64) {
        const int h = base + lane;
        const int c = (h < niters && rec[h].valid) ? rec[h].count : -1;
        int incl = c;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(incl, off);
            if (lane >= off) incl = max(incl, y);
        }
        int excl = __shfl_up(incl, 1);
        if (lane == 0) excl = -1;
        uint64_t m = __ballot(c > max(max(excl, good), 3));
        bool stop = false;
        while (m) {
            const int k = __ffsll((unsigned long long)m) - 1;
            const int hk = base + k;
            if (hk >= niters) {
                stop = true;
                break;
            }
            const int ck = __shfl(c, k);
            best = hk;
            good = ck;
            niters = update_num_iters(confidence, (double)(n - ck) / (double)n, niters);
            m &= m - 1;
        }
        if (stop) break;
    }
    return make_int3(best, best >= 0 ? max(niters, best + 1) : niters, good);
}

__global__ void __launch_bounds__(kRefineThreads) k_pnp_refine(PnpArgs a) {
    const int p = blockIdx.x;
    const vx_pnp_options o = a.opt[p];
    const int H = min(max(o.max_iterations, 0), kMaxHyp);
    const int b = a.offsets[p], n = a.offsets[p + 1] - b;
    const float* obj = a.obj + 3 * (size_t)b;
    const float* img = a.img + 2 * (size_t)b;
    uint8_t* mask = a.mask + b;
    const double cam[4] = {a.intr[4 * p], a.intr[4 * p + 1], a.intr[4 * p + 2], a.intr[4 * p + 3]};
    const HypRec* rec = a.hyp + (size_t)p * a.hmax;
    // sfin (step finite, set before the trial pass) and sgo (continue, set after it) are separate
    // so a thread still reading one iteration's flag never sees thread 0's next write
    __shared__ int sbest, srun, sgood, sfin, sgo;
    __shared__ double sT[7], sT1[7], sacc[kAcc], lds[(kRefineThreads / 64) * kAcc], red[kAcc];
    if (threadIdx.x < 64) {
        const int3 r = replay(rec, H, n, o.confidence);
        if (threadIdx.x == 0) {
            sbest = r.x;
            srun = r.y;
            sgood = r.z;
        }
    }
    __syncthreads();
    const int best = sbest;
    vx_pnp_result* r = a.out + p;
    if (best < 0) {
        for (int i = threadIdx.x; i < n; i += kRefineThreads) mask[i] = 0;
        if (threadIdx.x == 0) {
            vx_pnp_result z{};
            z.best_hypothesis = -1;
            z.hypotheses_run = srun;
            z.pose[3] = 1.0;
            *r = z;
        }
        return;
    }
    double R[9], t[3];
#pragma unroll
    for (int k = 0; k < 9; ++k) R[k] = rec[best].R[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) t[k] = rec[best].t[k];
    const double thr2 = o.reproj_error * o.reproj_error;
    for (int i = threadIdx.x; i < n; i += kRefineThreads) mask[i] = is_inlier(R, t, obj, img, i, cam, thr2) ? 1 : 0;
    if (threadIdx.x == 0) {
        double q[4];
        quat_of(R, q);
        for (int k = 0; k < 4; ++k) sT[k] = q[k];
        for (int k = 0; k < 3; ++k) sT[4 + k] = t[k];
    }
    __syncthreads();  // mask + sT visible
    double v[kAcc];
    accumulate(sT, obj, img, mask, n, cam, v);
    block_reduce(v, lds, red);
    if (threadIdx.x < kAcc) sacc[threadIdx.x] = red[threadIdx.x];  // thread 0 owns the LM state below
    const double cost0 = red[27];
    double lambda = 1e-3;
    int iters = 0;
    __syncthreads();
    for (int it = 0; it < o.refine_iterations; ++it) {
        if (threadIdx.x == 0) {
            double A[36], g[6], dx[6];
            int k = 0;
            for (int rr = 0; rr < 6; ++rr)
                for (int c = rr; c < 6; ++c) {
                    A[6 * rr + c] = sacc[k];
                    A[6 * c + rr] = sacc[k];
                    ++k;
                }
            for (int d = 0; d < 6; ++d) A[7 * d] += lambda * A[7 * d];
            for (int d = 0; d < 6; ++d) g[d] = sacc[21 + d];
            ldlt_spd_solve<6>(A, g, dx);
            bool fin = true;
            for (int d = 0; d < 6; ++d) fin &= isfinite(dx[d]);
            double T1[8];
            for (int d = 0; d < 7; ++d) T1[d] = sT[d];
            if (fin) se3_left_update(dx, T1);
            for (int d = 0; d < 7; ++d) sT1[d] = T1[d];
            sfin = fin ? 1 : 0;
        }
        __syncthreads();
        iters = it + 1;
        if (!sfin) break;
        accumulate(sT1, obj, img, mask, n, cam, v);
        block_reduce(v, lds, red);
        if (threadIdx.x == 0) {
            int go = 1;
            if (red[27] < sacc[27]) {
                const double prev = sacc[27];
                for (int k = 0; k < kAcc; ++k) sacc[k] = red[k];
                for (int d = 0; d < 7; ++d) sT[d] = sT1[d];
                lambda = fmax(lambda * 0.1, 1e-12);
                if (prev - sacc[27] <= 1e-10 * prev) go = 0;
            } else {
                lambda *= 10.0;
                if (lambda > 1e8) go = 0;
            }
            sgo = go;
        }
        __syncthreads();
        if (!sgo) break;
    }
    if (threadIdx.x == 0) {
        vx_pnp_result z{};
        z.ok = 1;
        z.n_inliers = sgood;
        z.best_hypothesis = best;
        z.hypotheses_run = srun;
        z.refine_iterations = iters;
        double q[4] = {sT[0], sT[1], sT[2], sT[3]};
        if (q[3] < 0.0)
            for (int k = 0; k < 4; ++k) q[k] = -q[k];
        for (int k = 0; k < 4; ++k) z.pose[k] = q[k];
        for (int k = 0; k < 3; ++k) z.pose[4 + k] = sT[4 + k];
        const double s = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
        const double kk = s > 0.0 ? 2.0 * atan2(s, q[3]) / s : 2.0;
        for (int k = 0; k < 3; ++k) {
            z.rvec[k] = kk * q[k];
            z.tvec[k] = z.pose[4 + k];
        }
        z.cost0 = cost0;
        z.cost = sacc[27];
        *r = z;
    }
}

size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

}  // namespace
}  // namespace vx

using namespace vx;

extern "C" {

void vx_pnp_default_options(int n_points, vx_pnp_options* o) {
    if (!o) return;
    o->max_iterations = std::min(100, 2 * std::max(n_points, 0));  // tracking.cpp:420
    o->refine_iterations = 20;
    o->reproj_error = 2.0;  // Tracking::Options::max_reproj_error (tracking.h:29)
    o->confidence = 0.99;   // tracking.cpp:423
    o->seed = 0x5EEDull;
}

int vx_pnp_ransac_batch(vx_ctx* c, int P, const int32_t* offsets, const float* obj, const float* img,
                        const double* intr4, const vx_pnp_options* opt, uint8_t* inlier_mask, vx_pnp_result* out) {
    if (!c || P < 0 || (P > 0 && (!offsets || !intr4 || !opt || !out)))
        return c ? set_error(c, VX_ERR_INVALID, "vx_pnp_ransac_batch: bad arguments") : VX_ERR_INVALID;
    if (P == 0) return VX_OK;
    if (P > 65535) return set_error(c, VX_ERR_INVALID, "at most 65535 problems per batch");
    if (offsets[0] != 0) return set_error(c, VX_ERR_INVALID, "offsets[0] must be 0");
    int hmax = 1;
    for (int p = 0; p < P; ++p) {
        if (offsets[p + 1] < offsets[p]) return set_error(c, VX_ERR_INVALID, "offsets must be non-decreasing");
        if (opt[p].max_iterations > kMaxHyp)
            return set_error(c, VX_ERR_INVALID, "max_iterations %d > %d", opt[p].max_iterations, kMaxHyp);
        if (opt[p].refine_iterations < 0 || !(opt[p].reproj_error >= 0.0))
            return set_error(c, VX_ERR_INVALID, "bad options for problem %d", p);
        const double* k = intr4 + 4 * p;
        if (!(k[0] != 0.0 && k[1] != 0.0)) return set_error(c, VX_ERR_INVALID, "zero focal length (problem %d)", p);
        hmax = std::max(hmax, opt[p].max_iterations);
    }
    const int64_t N = offsets[P];
    if (N > 0 && (!obj || !img)) return set_error(c, VX_ERR_INVALID, "vx_pnp_ransac_batch: null points");
    if (N > INT32_MAX / 3) return set_error(c, VX_ERR_INVALID, "too many correspondences");
    VX_HIP(c, hipSetDevice(c->device));
    // one packed upload: offsets | intr | options | obj | img
    const size_t o_off = 0, o_intr = align16(o_off + (P + 1) * sizeof(int32_t)),
                 o_opt = align16(o_intr + (size_t)P * 4 * sizeof(double)),
                 o_obj = align16(o_opt + (size_t)P * sizeof(vx_pnp_options)),
                 o_img = align16(o_obj + (size_t)N * 3 * sizeof(float)),
                 in_bytes = align16(o_img + (size_t)N * 2 * sizeof(float));
    VX_HIP(c, c->rs_host.ensure(in_bytes));
    uint8_t* hs = static_cast<uint8_t*>(c->rs_host.p);
    std::memcpy(hs + o_off, offsets, (P + 1) * sizeof(int32_t));
    std::memcpy(hs + o_intr, intr4, (size_t)P * 4 * sizeof(double));
    std::memcpy(hs + o_opt, opt, (size_t)P * sizeof(vx_pnp_options));
    if (N) {
        std::memcpy(hs + o_obj, obj, (size_t)N * 3 * sizeof(float));
        std::memcpy(hs + o_img, img, (size_t)N * 2 * sizeof(float));
    }
    VX_HIP(c, c->rs_in.ensure(in_bytes));
    VX_HIP(c, hipMemcpyAsync(c->rs_in.p, hs, in_bytes, hipMemcpyHostToDevice, c->stream));
    VX_HIP(c, c->rs_hyp.ensure((size_t)P * hmax * sizeof(HypRec)));
    const size_t out_bytes = align16((size_t)P * sizeof(vx_pnp_result)) + (size_t)std::max<int64_t>(N, 1);
    VX_HIP(c, c->rs_out.ensure(out_bytes));
    uint8_t* din = c->rs_in.as<uint8_t>();
    PnpArgs a{};
    a.offsets = reinterpret_cast<const int*>(din + o_off);
    a.intr = reinterpret_cast<const double*>(din + o_intr);
    a.opt = reinterpret_cast<const vx_pnp_options*>(din + o_opt);
    a.obj = reinterpret_cast<const float*>(din + o_obj);
    a.img = reinterpret_cast<const float*>(din + o_img);
    a.hyp = c->rs_hyp.as<HypRec>();
    a.hmax = hmax;
    a.out = c->rs_out.as<vx_pnp_result>();
    a.mask = c->rs_out.as<uint8_t>() + align16((size_t)P * sizeof(vx_pnp_result));
    VX_HIP(c, launch(c, kStPnpHyp, k_pnp_hyp, dim3(hmax, P), dim3(kThreads), 0, c->stream, a));
    VX_HIP(c, launch(c, kStPnpRefine, k_pnp_refine, dim3(P), dim3(kRefineThreads), 0, c->stream, a));
    VX_HIP(c, c->rs_host_out.ensure(out_bytes));
    VX_HIP(c, hipMemcpyAsync(c->rs_host_out.p, c->rs_out.p, out_bytes, hipMemcpyDeviceToHost, c->stream));
    VX_HIP(c, hipStreamSynchronize(c->stream));
    const uint8_t* ho = static_cast<const uint8_t*>(c->rs_host_out.p);
    std::memcpy(out, ho, (size_t)P * sizeof(vx_pnp_result));
    if (inlier_mask && N) std::memcpy(inlier_mask, ho + align16((size_t)P * sizeof(vx_pnp_result)), (size_t)N);
    return VX_OK;
}

int vx_pnp_ransac(vx_ctx* c, const float* obj, const float* img, int n, const double* intr4,
                  const vx_pnp_options* opt, uint8_t* inlier_mask, vx_pnp_result* out) {
    if (!c || n < 0 || !intr4 || !opt || !out)
        return c ? set_error(c, VX_ERR_INVALID, "vx_pnp_ransac: bad arguments") : VX_ERR_INVALID;
    const int32_t offsets[2] = {0, n};
    return vx_pnp_ransac_batch(c, 1, offsets, obj, img, intr4, opt, inlier_mask, out);
}

}  // extern "C"

static_assert(sizeof(vx_pnp_options) == 32, "vx_pnp_options layout (python PNP_OPTIONS_DTYPE)");
static_assert(sizeof(vx_pnp_result) == 144, "vx_pnp_result layout (python PNP_RESULT_DTYPE)");
