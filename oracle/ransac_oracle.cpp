// ransac_oracle.cpp — CPU restatement of the PnP RANSAC the GPU runs for cv::solvePnPRansac in
// Tracking::TrackWithPnP (core/frontend/tracking.cpp:414-423).  TEST INFRASTRUCTURE ONLY.
//
// The reference's arithmetic lives in OpenCV (calib3d solvePnPRansac / RANSACPointSetRegistrator /
// PnPRansacCallback, vcpkg opencv4 at the baseline in vcpkg.json, not installed here), so this is
// the SPECIFICATION the build chose for the same contract, written independently of
// visionx-slam_amd/csrc/ransac.hip:
//   * hypothesis h samples 4 distinct correspondences from a splitmix64 counter stream;
//   * P3P (Grunert's quartic in the depth ratio v = s2 / s0) on the first 3, real roots by
//     derivative-isolated monotone brackets + safeguarded Newton (only + - * / sqrt, so the GPU
//     reproduces it bit for bit), camera points aligned to world points by orthonormal triads;
//     the 4th correspondence picks the solution with the smallest reprojection error;
//   * inlier = point in front of the camera and squared reprojection error <= thr^2;
//   * the sequential loop of RANSACPointSetRegistrator::run (strictly-better count than
//     max(best, modelPoints - 1), RANSACUpdateNumIters shrinking the iteration budget) replayed over
//     the hypothesis stream;
//   * Levenberg-Marquardt on the kept model's inliers (left SE(3) perturbation, PoseJacobian of
//     core/backend/local_ba.cpp:26-33).
// Pinned by tests/test_ransac_cpu.py: noise-free P3P recovers the true pose, RANSAC with outliers
// recovers ground truth, and the inlier mask / iteration budget re-derived in numpy agree.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "ba_math.h"
#include "oracle.h"

using namespace orc_ba;

namespace {

uint64_t mix64(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

// ---------------------------------------------------------------- real polynomial roots
double peval(const double* c, int d, double x) {
    double v = c[d];
    for (int k = d - 1; k >= 0; --k) v = v * x + c[k];
    return v;
}
double pderiv(const double* c, int d, double x) {
    double v = (double)d * c[d];
    for (int k = d - 1; k >= 1; --k) v = v * x + (double)k * c[k];
    return v;
}

// root of p in [lo, hi] where p is monotone and changes sign; plo = p(lo) != 0
double bracket_root(const double* c, int d, double lo, double hi, double plo) {
    double x = 0.5 * (lo + hi);
    for (int it = 0; it < 100; ++it) {
        const double px = peval(c, d, x);
        if (px == 0.0) return x;
        if ((px < 0.0) == (plo < 0.0)) lo = x;
        else hi = x;
        const double dp = pderiv(c, d, x);
        double xn = x - px / dp;
        if (!(xn > lo && xn < hi)) xn = 0.5 * (lo + hi);
        if (std::fabs(xn - x) <= 4.440892098500626e-16 * std::fabs(xn)) return xn;
        x = xn;
    }
    return x;
}

// real roots of c[0] + c[1] x + ... + c[d] x^d (d <= 4), ascending, distinct; the critical points
// (roots of p') found on the way go to crit_out / n_crit when given (d >= 3)
int real_roots(const double* c, int d, double* out, double* crit_out = nullptr, int* n_crit = nullptr) {
    if (n_crit) *n_crit = 0;
    while (d > 0 && c[d] == 0.0) --d;
    if (d <= 0) return 0;
    if (d == 1) {
        out[0] = -c[0] / c[1];
        return 1;
    }
    if (d == 2) {
        const double disc = c[1] * c[1] - 4.0 * c[2] * c[0];
        if (disc < 0.0) return 0;
        const double sq = std::sqrt(disc);
        const double q = -0.5 * (c[1] + (c[1] >= 0.0 ? sq : -sq));
        if (q == 0.0) {
            out[0] = 0.0;
            return 1;
        }
        double r1 = q / c[2], r2 = c[0] / q;
        if (r2 < r1) std::swap(r1, r2);
        out[0] = r1;
        if (r2 == r1) return 1;
        out[1] = r2;
        return 2;
    }
    double dc[4];
    for (int k = 0; k < d; ++k) dc[k] = (double)(k + 1) * c[k + 1];
    double crit[4];
    const int nc = real_roots(dc, d - 1, crit);
    if (crit_out) {
        for (int k = 0; k < nc; ++k) crit_out[k] = crit[k];
        *n_crit = nc;
    }
    double B = 0.0;
    for (int k = 0; k < d; ++k) B = std::max(B, std::fabs(c[k] / c[d]));
    B = 1.0 + B;
    double e[6];
    int ne = 0;
    e[ne++] = -B;
    for (int k = 0; k < nc; ++k)
        if (crit[k] > -B && crit[k] < B) e[ne++] = crit[k];
    e[ne++] = B;
    int nr = 0;
    for (int k = 0; k + 1 < ne; ++k) {
        const double a = e[k], b = e[k + 1];
        if (!(a < b)) continue;
        const double pa = peval(c, d, a), pb = peval(c, d, b);
        if (pa == 0.0) {
            if (nr == 0 || out[nr - 1] != a) out[nr++] = a;
        } else if (pb != 0.0 && ((pa < 0.0) != (pb < 0.0))) {
            out[nr++] = bracket_root(c, d, a, b, pa);
        }
    }
    return nr;
}

// ---------------------------------------------------------------- P3P
struct V3 { double x, y, z; };
V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V3 crs(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
V3 unit(V3 a) {
    const double inv = 1.0 / std::sqrt(dot(a, a));
    return {a.x * inv, a.y * inv, a.z * inv};
}
V3 scl(V3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }

struct Model { double R[9], t[3]; };
constexpr int kMaxCand = 8;  // P3P candidates: real roots + non-crossing minima of |p| (<= 4 + 3)

V3 apply(const Model& M, V3 p) {
    return {M.R[0] * p.x + M.R[1] * p.y + M.R[2] * p.z + M.t[0], M.R[3] * p.x + M.R[4] * p.y + M.R[5] * p.z + M.t[1],
            M.R[6] * p.x + M.R[7] * p.y + M.R[8] * p.z + M.t[2]};
}

// squared reprojection error of world point p against pixel (u, v); false when behind the camera
bool reproj_sq(const Model& M, V3 p, double u, double v, const double* cam, double* err) {
    const V3 pc = apply(M, p);
    if (!(pc.z > 0.0)) return false;
    const double iz = 1.0 / pc.z;
    const double du = cam[0] * (pc.x * iz) + cam[2] - u;
    const double dv = cam[1] * (pc.y * iz) + cam[3] - v;
    *err = du * du + dv * dv;
    return true;
}

// Grunert: world points P[0..2], unit bearings f[0..2] -> up to kMaxCand (R, t) with s_i f_i = R P_i + t
int p3p(const V3* P, const V3* f, Model* out) {
    const V3 d12 = sub(P[1], P[2]), d02 = sub(P[0], P[2]), d01 = sub(P[0], P[1]);
    const double a2 = dot(d12, d12), b2 = dot(d02, d02), c2 = dot(d01, d01);
    if (!(a2 > 0.0 && b2 > 0.0 && c2 > 0.0)) return 0;
    const double ca = dot(f[1], f[2]), cb = dot(f[0], f[2]), cg = dot(f[0], f[1]);
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
    for (int k = 0; k < 5; ++k) scale = std::max(scale, std::fabs(A[k]));
    if (!(scale > 0.0)) return 0;
    const int deg = std::fabs(A[4]) <= 1e-12 * scale ? 3 : 4;
    // candidates: the real roots, then every local minimum of |p| that stays off zero (a double
    // root that measurement noise split into a complex pair: the classic P3P near-degeneracy)
    double roots[8], crit[4];
    int nc = 0;
    int nr = real_roots(A, deg, roots, crit, &nc);
    for (int k = 0; k < nc; ++k) {
        const double pc = peval(A, deg, crit[k]);
        double d2 = 0.0;  // p''(x)
        for (int j = deg; j >= 2; --j) d2 = d2 * crit[k] + (double)(j * (j - 1)) * A[j];
        if (pc != 0.0 && ((pc > 0.0) == (d2 > 0.0)) && d2 != 0.0) roots[nr++] = crit[k];
    }
    // world triad
    const V3 we1 = unit(sub(P[1], P[0]));
    const V3 we3 = unit(crs(sub(P[1], P[0]), sub(P[2], P[0])));
    const V3 we2 = crs(we3, we1);
    int ns = 0;
    for (int k = 0; k < nr; ++k) {
        const double v = roots[k];
        if (!(v > 0.0)) continue;
        const double den = 2.0 * (cg - v * ca);
        if (den == 0.0) continue;
        const double u = ((amc - 1.0) * v * v - 2.0 * amc * cb * v + 1.0 + amc) / den;
        if (!(u > 0.0)) continue;
        const double s0sq = b2 / (1.0 + v * v - 2.0 * v * cb);
        if (!(s0sq > 0.0)) continue;
        const double s0 = std::sqrt(s0sq);
        const V3 C0 = scl(f[0], s0), C1 = scl(f[1], u * s0), C2 = scl(f[2], v * s0);
        const V3 ce1 = unit(sub(C1, C0));
        const V3 ce3 = unit(crs(sub(C1, C0), sub(C2, C0)));
        const V3 ce2 = crs(ce3, ce1);
        Model& M = out[ns];
        const double cw[3][3] = {{ce1.x, ce2.x, ce3.x}, {ce1.y, ce2.y, ce3.y}, {ce1.z, ce2.z, ce3.z}};
        const double ww[3][3] = {{we1.x, we2.x, we3.x}, {we1.y, we2.y, we3.y}, {we1.z, we2.z, we3.z}};
        for (int r = 0; r < 3; ++r)
            for (int cc = 0; cc < 3; ++cc)
                M.R[3 * r + cc] = cw[r][0] * ww[cc][0] + cw[r][1] * ww[cc][1] + cw[r][2] * ww[cc][2];
        const V3 rp = {M.R[0] * P[0].x + M.R[1] * P[0].y + M.R[2] * P[0].z,
                       M.R[3] * P[0].x + M.R[4] * P[0].y + M.R[5] * P[0].z,
                       M.R[6] * P[0].x + M.R[7] * P[0].y + M.R[8] * P[0].z};
        M.t[0] = C0.x - rp.x;
        M.t[1] = C0.y - rp.y;
        M.t[2] = C0.z - rp.z;
        ++ns;
    }
    return ns;
}

V3 world_pt(const float* obj, int i) { return {(double)obj[3 * i], (double)obj[3 * i + 1], (double)obj[3 * i + 2]}; }

V3 bearing(const float* img, int i, const double* cam) {
    const double x = ((double)img[2 * i] - cam[2]) / cam[0];
    const double y = ((double)img[2 * i + 1] - cam[3]) / cam[1];
    const double inv = 1.0 / std::sqrt(x * x + y * y + 1.0);
    return {x * inv, y * inv, inv};
}

// sample 4 distinct indices of [0, n) for hypothesis h; false if the stream runs dry (n < 4)
bool sample4(uint64_t seed, int h, int n, int* idx) {
    int got = 0;
    for (int a = 0; a < 64 && got < 4; ++a) {
        const uint64_t x = mix64(seed + (uint64_t)h * 64u + (uint64_t)a);
        const int i = (int)(((x >> 32) * (uint64_t)n) >> 32);
        bool dup = false;
        for (int k = 0; k < got; ++k) dup |= idx[k] == i;
        if (!dup) idx[got++] = i;
    }
    return got == 4;
}

bool hypothesis(const float* obj, const float* img, int n, const double* cam, uint64_t seed, int h, Model* best) {
    int idx[4];
    if (!sample4(seed, h, n, idx)) return false;
    V3 P[3], f[3];
    for (int k = 0; k < 3; ++k) {
        P[k] = world_pt(obj, idx[k]);
        f[k] = bearing(img, idx[k], cam);
    }
    Model sols[kMaxCand];
    const int ns = p3p(P, f, sols);
    const V3 P3 = world_pt(obj, idx[3]);
    double best_err = INFINITY;
    int bi = -1;
    for (int s = 0; s < ns; ++s) {
        double e;
        if (!reproj_sq(sols[s], P3, (double)img[2 * idx[3]], (double)img[2 * idx[3] + 1], cam, &e)) continue;
        if (e < best_err) {
            best_err = e;
            bi = s;
        }
    }
    if (bi < 0) return false;
    *best = sols[bi];
    return true;
}

int count_inliers(const Model& M, const float* obj, const float* img, int n, const double* cam, double thr2,
                  uint8_t* mask) {
    int cnt = 0;
    for (int i = 0; i < n; ++i) {
        double e;
        const bool in = reproj_sq(M, world_pt(obj, i), (double)img[2 * i], (double)img[2 * i + 1], cam, &e) && e <= thr2;
        if (mask) mask[i] = in ? 1 : 0;
        cnt += in ? 1 : 0;
    }
    return cnt;
}

// RANSACUpdateNumIters (OpenCV calib3d ptsetreg.cpp) for modelPoints = 4
int update_num_iters(double p, double ep, int max_iters) {
    p = std::max(p, 0.0);
    p = std::min(p, 1.0);
    ep = std::max(ep, 0.0);
    ep = std::min(ep, 1.0);
    double num = std::max(1.0 - p, DBL_MIN);
    const double x = 1.0 - ep;
    double denom = 1.0 - (x * x) * (x * x);
    if (denom < DBL_MIN) return 0;
    num = std::log(num);
    denom = std::log(denom);
    return denom >= 0.0 || -num >= (double)max_iters * -denom ? max_iters : (int)std::rint(num / denom);
}

// rotation matrix -> unit quaternion (x y z w), Shepperd's branch on the largest diagonal term
void quat_of(const double* R, double* q) {
    const double tr = R[0] + R[4] + R[8];
    double x, y, z, w;
    if (tr > 0.0) {
        const double s = std::sqrt(tr + 1.0) * 2.0;
        w = 0.25 * s; x = (R[7] - R[5]) / s; y = (R[2] - R[6]) / s; z = (R[3] - R[1]) / s;
    } else if (R[0] > R[4] && R[0] > R[8]) {
        const double s = std::sqrt(1.0 + R[0] - R[4] - R[8]) * 2.0;
        w = (R[7] - R[5]) / s; x = 0.25 * s; y = (R[1] + R[3]) / s; z = (R[2] + R[6]) / s;
    } else if (R[4] > R[8]) {
        const double s = std::sqrt(1.0 + R[4] - R[0] - R[8]) * 2.0;
        w = (R[2] - R[6]) / s; x = (R[1] + R[3]) / s; y = 0.25 * s; z = (R[5] + R[7]) / s;
    } else {
        const double s = std::sqrt(1.0 + R[8] - R[0] - R[4]) * 2.0;
        w = (R[3] - R[1]) / s; x = (R[2] + R[6]) / s; y = (R[5] + R[7]) / s; z = 0.25 * s;
    }
    const double inv = 1.0 / std::sqrt(x * x + y * y + z * z + w * w);
    q[0] = x * inv; q[1] = y * inv; q[2] = z * inv; q[3] = w * inv;
}

struct Acc { double H[36], g[6], cost; int cnt; };

void accumulate(const SE3& T, const float* obj, const float* img, int n, const uint8_t* mask, const Cam& cam, Acc& a) {
    std::memset(&a, 0, sizeof(a));
    for (int i = 0; i < n; ++i) {
        if (!mask[i]) continue;
        const Vec3 pw{(double)obj[3 * i], (double)obj[3 * i + 1], (double)obj[3 * i + 2]};
        double uv[2];
        Vec3 pc;
        if (!project(cam, T, pw, uv, pc)) continue;
        const double e[2] = {(double)img[2 * i] - uv[0], (double)img[2 * i + 1] - uv[1]};
        double J[12];
        pose_jac(cam, pc, J);
        for (int r = 0; r < 6; ++r) {
            for (int c = 0; c < 6; ++c) a.H[6 * r + c] += J[r] * J[c] + J[6 + r] * J[6 + c];
            a.g[r] += J[r] * e[0] + J[6 + r] * e[1];
        }
        a.cost += e[0] * e[0] + e[1] * e[1];
        ++a.cnt;
    }
}

void solve_one(const float* obj, const float* img, int n, const double* cam4, const orc_pnp_options& o,
               uint8_t* mask, orc_pnp_result& r) {
    std::memset(&r, 0, sizeof(r));
    r.best_hypothesis = -1;
    r.pose[3] = 1.0;
    if (mask) std::memset(mask, 0, (size_t)n);
    const int H = std::min(std::max(o.max_iterations, 0), ORC_PNP_MAX_HYP);
    if (n < 4 || H == 0) return;
    std::vector<Model> models(H);
    std::vector<int> valid(H), count(H);
    const double thr2 = o.reproj_error * o.reproj_error;
    for (int h = 0; h < H; ++h) {
        valid[h] = hypothesis(obj, img, n, cam4, o.seed, h, &models[h]);
        count[h] = valid[h] ? count_inliers(models[h], obj, img, n, cam4, thr2, nullptr) : 0;
    }
    int niters = H, best = -1, max_good = 0, h = 0;
    for (; h < niters; ++h) {
        if (!valid[h]) continue;
        if (count[h] > std::max(max_good, 3)) {
            best = h;
            max_good = count[h];
            niters = update_num_iters(o.confidence, (double)(n - count[h]) / (double)n, niters);
        }
    }
    r.hypotheses_run = h;
    if (best < 0) return;
    std::vector<uint8_t> m(n);
    r.ok = 1;
    r.best_hypothesis = best;
    r.n_inliers = count_inliers(models[best], obj, img, n, cam4, thr2, m.data());
    if (mask) std::memcpy(mask, m.data(), (size_t)n);

    SE3 T;
    double q[4];
    quat_of(models[best].R, q);
    T.q = {q[0], q[1], q[2], q[3]};
    T.t = {models[best].t[0], models[best].t[1], models[best].t[2]};
    const Cam cam{cam4[0], cam4[1], cam4[2], cam4[3]};
    Acc a;
    accumulate(T, obj, img, n, m.data(), cam, a);
    r.cost0 = a.cost;
    double lambda = 1e-3;
    for (int it = 0; it < o.refine_iterations; ++it) {
        double A[36], dx[6];
        std::memcpy(A, a.H, sizeof(A));
        for (int k = 0; k < 6; ++k) A[7 * k] += lambda * a.H[7 * k];
        ldlt_solve<6>(A, a.g, dx);
        r.refine_iterations = it + 1;
        if (!all_finite(dx, 6)) break;
        const SE3 T1 = left_update(dx, T);
        Acc a1;
        accumulate(T1, obj, img, n, m.data(), cam, a1);
        if (a1.cost < a.cost) {
            const double prev = a.cost;
            T = T1;
            a = a1;
            lambda = std::max(lambda * 0.1, 1e-12);
            if (prev - a.cost <= 1e-10 * prev) break;
        } else {
            lambda *= 10.0;
            if (lambda > 1e8) break;
        }
    }
    r.cost = a.cost;
    double qq[4] = {T.q.x, T.q.y, T.q.z, T.q.w};
    if (qq[3] < 0.0)
        for (double& v : qq) v = -v;
    r.pose[0] = qq[0]; r.pose[1] = qq[1]; r.pose[2] = qq[2]; r.pose[3] = qq[3];
    r.pose[4] = T.t.x; r.pose[5] = T.t.y; r.pose[6] = T.t.z;
    const double s = std::sqrt(qq[0] * qq[0] + qq[1] * qq[1] + qq[2] * qq[2]);
    const double k = s > 0.0 ? 2.0 * std::atan2(s, qq[3]) / s : 2.0;
    for (int j = 0; j < 3; ++j) {
        r.rvec[j] = k * qq[j];
        r.tvec[j] = r.pose[4 + j];
    }
}

}  // namespace

extern "C" {

int orc_pnp_hypothesis(const float* obj, const float* img, int n, const double* intr4, uint64_t seed, int h,
                       double* R9, double* t3) {
    Model M;
    if (!hypothesis(obj, img, n, intr4, seed, h, &M)) return 0;
    std::memcpy(R9, M.R, sizeof(M.R));
    std::memcpy(t3, M.t, sizeof(M.t));
    return 1;
}

int orc_p3p(const double* P9, const double* f9, double* R72, double* t24) {
    V3 P[3], f[3];
    for (int k = 0; k < 3; ++k) {
        P[k] = {P9[3 * k], P9[3 * k + 1], P9[3 * k + 2]};
        f[k] = {f9[3 * k], f9[3 * k + 1], f9[3 * k + 2]};
    }
    Model M[kMaxCand];
    const int ns = p3p(P, f, M);
    for (int s = 0; s < ns; ++s) {
        std::memcpy(R72 + 9 * s, M[s].R, sizeof(M[s].R));
        std::memcpy(t24 + 3 * s, M[s].t, sizeof(M[s].t));
    }
    return ns;
}

int orc_poly_roots(const double* c, int d, double* out) { return real_roots(c, d, out); }

int orc_pnp_update_iters(double p, double ep, int max_iters) { return update_num_iters(p, ep, max_iters); }

int orc_pnp_ransac_batch(int n_problems, const int32_t* offsets, const float* obj, const float* img,
                         const double* intr4, const orc_pnp_options* opt, uint8_t* mask, orc_pnp_result* out) {
    for (int p = 0; p < n_problems; ++p) {
        const int b = offsets[p], n = offsets[p + 1] - offsets[p];
        solve_one(obj + 3 * (size_t)b, img + 2 * (size_t)b, n, intr4 + 4 * p, opt[p], mask ? mask + b : nullptr, out[p]);
    }
    return 0;
}

}  // extern "C"
