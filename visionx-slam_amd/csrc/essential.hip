// essential.hip — essential-matrix RANSAC + pose recovery for Tracking::EstimatePoseByEssential
// (core/frontend/tracking.cpp:503-547):
//     E = cv::findEssentialMat(pts_last, pts_curr, K, cv::RANSAC, 0.999, 1.0, mask);
//     inliers = cv::recoverPose(E, pts_last, pts_curr, K, R, t, mask);
//
//   k_em_hyp     grid (H, problems)  lane 0: 5-sample + five-point solver (null space, 10 x 20
//                                    cubic constraints, Gauss-Jordan, action matrix, Hessenberg +
//                                    Francis QR, eigenvectors) -> up to 10 E; the workgroup scores
//                                    every E by Sampson error over the problem's matches
//   k_em_pick    grid (problems)     wave 0 replays RANSACPointSetRegistrator::run over the
//                                    (hypothesis, model) counts; E = U S V^T -> R1, R2, t
//   k_em_cheir   grid (matches/256, problems)  RANSAC mask; the four (R, +-t) scored by DLT
//                                    triangulation of the inliers (one match per thread)
//   k_em_final   grid (matches/256, problems)  OpenCV's candidate choice, output mask, result
//
// Every step uses + - * / sqrt only, in the order of the CPU restatement (oracle/essential_oracle.cpp,
// the specification; -ffp-contract=off), so models, counts, the kept model, R, t and both masks are
// bit-identical to it.  The (R, -t) candidates reuse the (R, t) triangulation with w negated — the
// Jacobi rotations are odd in that column, so this is exactly what triangulating them gives.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>

#include "vx_internal.hpp"

namespace vx {
namespace {

constexpr int kThreads = 64;  // one wave per hypothesis: the five-point solve is wave-parallel
constexpr int kMaxHyp = 4096;
constexpr int kMaxModels = 10;

struct EmRec {
    double E[kMaxModels][9];
    int count[kMaxModels];
    int nm, pad;
};

struct EmArgs {
    const int* offsets;                // P + 1
    const double* intr;                // 4 per problem
    const vx_essential_options* opt;   // per problem
    const float* p1;                   // 2 per match (pts_last)
    const float* p2;                   // 2 per match (pts_curr)
    EmRec* rec;                        // [P][hmax]
    int hmax;
    vx_essential_result* out;          // per problem
    uint8_t* mask;                     // per match
};

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

template <class T>
__device__ __forceinline__ void swp(T& a, T& b) {
    const T t = a;
    a = b;
    b = t;
}

// ---------------------------------------------------------------- polynomials in x, y, z
// degree 1 [x y z 1]; degree 2 [x2 xy xz y2 yz z2 x y z 1];
// degree 3 [x3 x2y x2z xy2 xyz xz2 y3 y2z yz2 z3 | x2 xy xz y2 yz z2 x y z 1]
// (product tables; the loops using them are fully unrolled, so the indices are constants and the
// operands stay in registers)
constexpr int kM11[4][4] = {{0, 1, 2, 6}, {1, 3, 4, 7}, {2, 4, 5, 8}, {6, 7, 8, 9}};
constexpr int kM21[10][4] = {{0, 1, 2, 10},   {1, 3, 4, 11},   {2, 4, 5, 12},   {3, 6, 7, 13},
                             {4, 7, 8, 14},   {5, 8, 9, 15},   {10, 11, 12, 16}, {11, 13, 14, 17},
                             {12, 14, 15, 18}, {16, 17, 18, 19}};

__device__ __forceinline__ void mul11(const double* a, const double* b, double* c) {
#pragma unroll
    for (int k = 0; k < 10; ++k) c[k] = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) c[kM11[i][j]] += a[i] * b[j];
}
__device__ __forceinline__ void mul21_acc(const double* p, const double* a, double* c) {
#pragma unroll
    for (int i = 0; i < 10; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) c[kM21[i][j]] += p[i] * a[j];
}

// ---------------------------------------------------------------- five-point solver, one wave
// The working set of one solve lives in LDS and the wave runs the algorithm together: scalar
// control flow (pivot searches, the QR iteration's shifts and deflation tests) is evaluated
// identically by all 64 lanes from the same LDS values; every loop over independent matrix elements
// (row swaps / scaling / elimination, the Hessenberg and QR row and column updates) is split across
// lanes; the up-to-10 eigenvector solves run one per lane.  Each element still sees exactly the
// operations, in the order, of the sequential restatement.
struct FpWork {
    double s1[10], s2[10];  // the sample, normalised (pts_last, pts_curr)
    double Q[45];
    double basis[4][9];
    double EEt[9][10];
    double tr[10];
    double M[10][20];
    double At[100];
    double H[100];
    double wr[10], wi[10];
    double NB[10][100];
    double Es[kMaxModels][9];
    int valid[kMaxModels];
    int used[9], pc[5];
};

#define WSYNC __syncthreads()

__device__ __forceinline__ void load_E(const FpWork& w, int k, double* e) {
    e[0] = w.basis[0][k];
    e[1] = w.basis[1][k];
    e[2] = w.basis[2][k];
    e[3] = w.basis[3][k];
}

// elmhes on w.H (10 x 10)
__device__ void elmhes_wave(double* a, int lane) {
    constexpr int n = 10;
    auto A = [&](int i, int j) -> double& { return a[i * n + j]; };
    for (int m = 1; m < n - 1; ++m) {
        double x = 0.0;
        int i = m;
        for (int j = m; j < n; ++j) {
            if (fabs(A(j, m - 1)) > fabs(x)) {
                x = A(j, m - 1);
                i = j;
            }
        }
        WSYNC;
        if (i != m) {
            if (lane >= m - 1 && lane < n) swp(A(i, lane), A(m, lane));
            WSYNC;
            if (lane < n) swp(A(lane, i), A(lane, m));
            WSYNC;
        }
        if (x != 0.0) {
            for (int i2 = m + 1; i2 < n; ++i2) {
                double y = A(i2, m - 1);
                if (y != 0.0) {
                    y /= x;
                    WSYNC;
                    if (lane == 0) A(i2, m - 1) = y;
                    if (lane >= m && lane < n) A(i2, lane) -= y * A(m, lane);
                    WSYNC;
                    if (lane < n) A(lane, m) += y * A(lane, i2);
                    WSYNC;
                }
            }
        }
    }
    for (int e = lane; e < n * n; e += 64) {
        const int i = e / n, j = e - i * n;
        if (i >= 2 && j < i - 1) A(i, j) = 0.0;
    }
    WSYNC;
}

// Francis double-shift QR on w.H: eigenvalues into wr / wi; false after 30 iterations on one
__device__ bool hqr_wave(double* a, double* wr, double* wi, int lane) {
    constexpr int n = 10;
    auto A = [&](int i, int j) -> double& { return a[i * n + j]; };
    double anorm = 0.0;
    for (int i = 0; i < n; ++i)
        for (int j = max(i - 1, 0); j < n; ++j) anorm += fabs(A(i, j));
    int nn = n - 1;
    double t = 0.0;
    while (nn >= 0) {
        int its = 0, l;
        do {
            for (l = nn; l >= 1; --l) {
                double s = fabs(A(l - 1, l - 1)) + fabs(A(l, l));
                if (s == 0.0) s = anorm;
                if (fabs(A(l, l - 1)) <= DBL_EPSILON * s) {
                    WSYNC;
                    if (lane == 0) A(l, l - 1) = 0.0;
                    WSYNC;
                    break;
                }
            }
            double x = A(nn, nn);
            if (l == nn) {
                if (lane == 0) {
                    wr[nn] = x + t;
                    wi[nn] = 0.0;
                }
                --nn;
            } else {
                double y = A(nn - 1, nn - 1);
                double w = A(nn, nn - 1) * A(nn - 1, nn);
                if (l == nn - 1) {
                    const double p = 0.5 * (y - x);
                    const double q = p * p + w;
                    double z = sqrt(fabs(q));
                    x += t;
                    if (lane == 0) {
                        if (q >= 0.0) {
                            z = p + (p >= 0.0 ? fabs(z) : -fabs(z));
                            wr[nn - 1] = wr[nn] = x + z;
                            if (z != 0.0) wr[nn] = x - w / z;
                            wi[nn - 1] = wi[nn] = 0.0;
                        } else {
                            wr[nn - 1] = wr[nn] = x + p;
                            wi[nn - 1] = -z;
                            wi[nn] = z;
                        }
                    }
                    nn -= 2;
                } else {
                    if (its == 30) return false;
                    if (its == 10 || its == 20) {
                        t += x;
                        WSYNC;
                        if (lane <= nn) A(lane, lane) -= x;
                        WSYNC;
                        const double s = fabs(A(nn, nn - 1)) + fabs(A(nn - 1, nn - 2));
                        y = x = 0.75 * s;
                        w = -0.4375 * s * s;
                    }
                    ++its;
                    int m;
                    double p = 0.0, q = 0.0, r = 0.0, z;
                    for (m = nn - 2; m >= l; --m) {
                        z = A(m, m);
                        r = x - z;
                        double s = y - z;
                        p = (r * s - w) / A(m + 1, m) + A(m, m + 1);
                        q = A(m + 1, m + 1) - z - r - s;
                        r = A(m + 2, m + 1);
                        s = fabs(p) + fabs(q) + fabs(r);
                        p /= s;
                        q /= s;
                        r /= s;
                        if (m == l) break;
                        const double u = fabs(A(m, m - 1)) * (fabs(q) + fabs(r));
                        const double v = fabs(p) * (fabs(A(m - 1, m - 1)) + fabs(z) + fabs(A(m + 1, m + 1)));
                        if (u <= DBL_EPSILON * v) break;
                    }
                    WSYNC;
                    {
                        const int i = m + 2 + lane;
                        if (i <= nn) {
                            A(i, i - 2) = 0.0;
                            if (i != m + 2) A(i, i - 3) = 0.0;
                        }
                    }
                    WSYNC;
                    for (int k = m; k <= nn - 1; ++k) {
                        if (k != m) {
                            p = A(k, k - 1);
                            q = A(k + 1, k - 1);
                            r = 0.0;
                            if (k != nn - 1) r = A(k + 2, k - 1);
                            x = fabs(p) + fabs(q) + fabs(r);
                            if (x != 0.0) {
                                p /= x;
                                q /= x;
                                r /= x;
                            }
                        }
                        const double sq = sqrt(p * p + q * q + r * r);
                        const double s = p >= 0.0 ? sq : -sq;
                        if (s != 0.0) {
                            const double akk1 = k >= 1 ? A(k, k - 1) : 0.0;
                            WSYNC;
                            if (lane == 0) {
                                if (k == m) {
                                    if (l != m) A(k, k - 1) = -akk1;
                                } else {
                                    A(k, k - 1) = -s * x;
                                }
                            }
                            p += s;
                            x = p / s;
                            y = q / s;
                            z = r / s;
                            q /= p;
                            r /= p;
                            {  // row modification, one column per lane
                                const int j = k + lane;
                                if (j <= nn) {
                                    double pj = A(k, j) + q * A(k + 1, j);
                                    if (k != nn - 1) {
                                        pj += r * A(k + 2, j);
                                        A(k + 2, j) -= pj * z;
                                    }
                                    A(k + 1, j) -= pj * y;
                                    A(k, j) -= pj * x;
                                }
                            }
                            WSYNC;
                            {  // column modification, one row per lane
                                const int mmin = nn < k + 3 ? nn : k + 3;
                                const int i = l + lane;
                                if (i <= mmin) {
                                    double pi = x * A(i, k) + y * A(i, k + 1);
                                    if (k != nn - 1) {
                                        pi += z * A(i, k + 2);
                                        A(i, k + 2) -= pi * r;
                                    }
                                    A(i, k + 1) -= pi * q;
                                    A(i, k) -= pi;
                                }
                            }
                            WSYNC;
                        }
                    }
                }
            }
        } while (nn >= 0 && l < nn - 1);
    }
    WSYNC;
    return true;
}

// null vector of a (10 x 10, destroyed) by full-pivot elimination, sequential (one lane)
__device__ bool null_vector10(double* a, double* v) {
    constexpr int n = 10;
    auto A = [&](int i, int j) -> double& { return a[i * n + j]; };
    int perm[n];
    for (int j = 0; j < n; ++j) perm[j] = j;
    for (int k = 0; k < n - 1; ++k) {
        int bi = k, bj = k;
        double bv = -1.0;
        for (int i = k; i < n; ++i)
            for (int j = k; j < n; ++j)
                if (fabs(A(i, j)) > bv) {
                    bv = fabs(A(i, j));
                    bi = i;
                    bj = j;
                }
        if (!(bv > 0.0)) return false;
        if (bi != k)
            for (int j = 0; j < n; ++j) swp(A(bi, j), A(k, j));
        if (bj != k) {
            for (int i = 0; i < n; ++i) swp(A(i, bj), A(i, k));
            swp(perm[bj], perm[k]);
        }
        for (int i = k + 1; i < n; ++i) {
            const double f = A(i, k) / A(k, k);
            for (int j = k + 1; j < n; ++j) A(i, j) -= f * A(k, j);
            A(i, k) = 0.0;
        }
    }
    double y[n];
    y[n - 1] = 1.0;
    for (int k = n - 2; k >= 0; --k) {
        double s = 0.0;
        for (int j = k + 1; j < n; ++j) s += A(k, j) * y[j];
        y[k] = -s / A(k, k);
    }
    for (int j = 0; j < n; ++j) v[perm[j]] = y[j];
    return true;
}

// five-point solve of w.s1 / w.s2 by the whole wave; returns the number of E (w.Es / w.valid
// compacted in eigenvalue order into out[ns][9] by lane 0)
__device__ int five_point_wave(FpWork& w, double* out, int lane) {
    if (lane < 45) {
        const int i = lane / 9, r = (lane % 9) / 3, c = lane % 3;
        const double av = c == 2 ? 1.0 : w.s1[2 * i + c];
        const double bv = r == 2 ? 1.0 : w.s2[2 * i + r];
        w.Q[lane] = bv * av;
    }
    if (lane < 9) w.used[lane] = 0;
    WSYNC;
    // null space: Gauss-Jordan with full pivoting over the unused columns
    for (int k = 0; k < 5; ++k) {
        int bi = -1, bj = -1;
        double bv = 0.0;
        for (int i = k; i < 5; ++i)
            for (int j = 0; j < 9; ++j)
                if (!w.used[j] && fabs(w.Q[9 * i + j]) > bv) {
                    bv = fabs(w.Q[9 * i + j]);
                    bi = i;
                    bj = j;
                }
        if (bi < 0) return 0;
        WSYNC;
        if (bi != k && lane < 9) swp(w.Q[9 * bi + lane], w.Q[9 * k + lane]);
        WSYNC;
        const double p = w.Q[9 * k + bj];
        WSYNC;
        if (lane == 0) {
            w.used[bj] = 1;
            w.pc[k] = bj;
        }
        if (lane < 9) w.Q[9 * k + lane] = lane == bj ? 1.0 : w.Q[9 * k + lane] / p;
        WSYNC;
        const int r = lane / 9, j = lane % 9;
        double nv = 0.0;
        if (lane < 45 && r != k) {
            const double f = w.Q[9 * r + bj];
            nv = j == bj ? 0.0 : w.Q[9 * r + j] - f * w.Q[9 * k + j];
        }
        WSYNC;
        if (lane < 45 && r != k) w.Q[9 * r + j] = nv;
        WSYNC;
    }
    if (lane < 36) {
        const int m = lane / 9, j = lane % 9;
        int f = -1, cnt = 0;
        for (int c = 0; c < 9; ++c)
            if (!w.used[c]) {
                if (cnt == m) f = c;
                ++cnt;
            }
        double v = 0.0;
        if (j == f) {
            v = 1.0;
        } else {
            for (int k = 0; k < 5; ++k)
                if (w.pc[k] == j) v = -w.Q[9 * k + f];
        }
        w.basis[m][j] = v;
    }
    WSYNC;
    // E E^T (one entry per lane), its trace, then the ten cubic constraint rows (one per lane)
    if (lane < 9) {
        const int i = lane / 3, j = lane % 3;
        double acc[10], tmp[10], ea[4], eb[4];
#pragma unroll
        for (int m = 0; m < 10; ++m) acc[m] = 0.0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            load_E(w, 3 * i + k, ea);
            load_E(w, 3 * j + k, eb);
            mul11(ea, eb, tmp);
#pragma unroll
            for (int m = 0; m < 10; ++m) acc[m] += tmp[m];
        }
#pragma unroll
        for (int m = 0; m < 10; ++m) w.EEt[lane][m] = acc[m];
    }
    WSYNC;
    if (lane < 10) w.tr[lane] = w.EEt[0][lane] + w.EEt[4][lane] + w.EEt[8][lane];
    WSYNC;
    if (lane < 9) {
        const int i = lane / 3, j = lane % 3;
        double acc[20], te[20], pe[10], e[4];
#pragma unroll
        for (int m = 0; m < 20; ++m) acc[m] = te[m] = 0.0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
#pragma unroll
            for (int m = 0; m < 10; ++m) pe[m] = w.EEt[3 * i + k][m];
            load_E(w, 3 * k + j, e);
            mul21_acc(pe, e, acc);
        }
#pragma unroll
        for (int m = 0; m < 10; ++m) pe[m] = w.tr[m];
        load_E(w, 3 * i + j, e);
        mul21_acc(pe, e, te);
#pragma unroll
        for (int m = 0; m < 20; ++m) w.M[lane][m] = 2.0 * acc[m] - te[m];
    } else if (lane == 9) {
        double E[9][4];
#pragma unroll
        for (int k = 0; k < 9; ++k) load_E(w, k, E[k]);
        double m0[10], m1[10], m2[10], ta[10], tb[10];
        mul11(E[4], E[8], ta); mul11(E[5], E[7], tb);
#pragma unroll
        for (int m = 0; m < 10; ++m) m0[m] = ta[m] - tb[m];
        mul11(E[3], E[8], ta); mul11(E[5], E[6], tb);
#pragma unroll
        for (int m = 0; m < 10; ++m) m1[m] = ta[m] - tb[m];
        mul11(E[3], E[7], ta); mul11(E[4], E[6], tb);
#pragma unroll
        for (int m = 0; m < 10; ++m) m2[m] = ta[m] - tb[m];
        double d0[20], d1[20], d2[20];
#pragma unroll
        for (int m = 0; m < 20; ++m) d0[m] = d1[m] = d2[m] = 0.0;
        mul21_acc(m0, E[0], d0);
        mul21_acc(m1, E[1], d1);
        mul21_acc(m2, E[2], d2);
#pragma unroll
        for (int m = 0; m < 20; ++m) w.M[9][m] = d0[m] - d1[m] + d2[m];
    }
    WSYNC;
    // Gauss-Jordan on the cubic block (partial pivoting)
    for (int k = 0; k < 10; ++k) {
        int bi = k;
        double bv = fabs(w.M[k][k]);
        for (int i = k + 1; i < 10; ++i)
            if (fabs(w.M[i][k]) > bv) {
                bv = fabs(w.M[i][k]);
                bi = i;
            }
        if (!(bv > 0.0)) return 0;
        WSYNC;
        if (bi != k && lane < 20) swp(w.M[bi][lane], w.M[k][lane]);
        WSYNC;
        const double p = w.M[k][k];
        WSYNC;
        if (lane > k && lane < 20) w.M[k][lane] = w.M[k][lane] / p;
        if (lane == k) w.M[k][k] = 1.0;
        WSYNC;
        const int ncol = 19 - k;  // columns k+1 .. 19
        double nv[3];
        int ne = 0;
        for (int e = lane; e < 10 * ncol; e += 64, ++ne) {
            const int r = e / ncol, j = k + 1 + (e - r * ncol);
            const double f = w.M[r][k];
            nv[ne] = (r != k && f != 0.0) ? w.M[r][j] - f * w.M[k][j] : w.M[r][j];
        }
        double fz = 0.0;
        if (lane < 10) fz = w.M[lane][k];
        WSYNC;
        ne = 0;
        for (int e = lane; e < 10 * ncol; e += 64, ++ne) {
            const int r = e / ncol, j = k + 1 + (e - r * ncol);
            w.M[r][j] = nv[ne];
        }
        if (lane < 10 && lane != k && fz != 0.0) w.M[lane][k] = 0.0;
        WSYNC;
    }
    // action matrix of multiplication by x on [x2 xy xz y2 yz z2 x y z 1]
    for (int e = lane; e < 100; e += 64) {
        const int s = e / 10, j = e - 10 * s;
        double v;
        if (s < 6) {
            v = -w.M[s][10 + j];
        } else {
            const int lin = s == 9 ? 6 : s - 6;  // x*x = x2, x*y = xy, x*z = xz, x*1 = x
            v = j == lin ? 1.0 : 0.0;
        }
        w.At[e] = v;
        w.H[e] = v;
    }
    WSYNC;
    elmhes_wave(w.H, lane);
    if (!hqr_wave(w.H, w.wr, w.wi, lane)) return 0;
    // one eigenvector per lane
    if (lane < 10) {
        int ok = 0;
        if (w.wi[lane] == 0.0) {
            double* B = w.NB[lane];
            for (int q = 0; q < 100; ++q) B[q] = w.At[q];
            for (int d = 0; d < 10; ++d) B[11 * d] -= w.wr[lane];
            double v[10];
            if (null_vector10(B, v) && v[9] != 0.0) {
                const double x = v[6] / v[9], y = v[7] / v[9], z = v[8] / v[9];
                double e[9], nrm = 0.0;
                for (int m = 0; m < 9; ++m) {
                    e[m] = x * w.basis[0][m] + y * w.basis[1][m] + z * w.basis[2][m] + w.basis[3][m];
                    nrm += e[m] * e[m];
                }
                if (nrm > 0.0) {
                    const double inv = 1.0 / sqrt(nrm);
                    for (int m = 0; m < 9; ++m) w.Es[lane][m] = e[m] * inv;
                    ok = 1;
                }
            }
        }
        w.valid[lane] = ok;
    }
    WSYNC;
    int ns = 0;
    for (int k = 0; k < 10; ++k) {
        if (!w.valid[k]) continue;
        if (lane < 9) out[9 * ns + lane] = w.Es[k][lane];
        ++ns;
    }
    WSYNC;
    return ns;
}

__device__ __forceinline__ double sampson(const double* E, double x1, double y1, double x2, double y2) {
    const double Ex1[3] = {E[0] * x1 + E[1] * y1 + E[2], E[3] * x1 + E[4] * y1 + E[5], E[6] * x1 + E[7] * y1 + E[8]};
    const double Etx2[3] = {E[0] * x2 + E[3] * y2 + E[6], E[1] * x2 + E[4] * y2 + E[7], E[2] * x2 + E[5] * y2 + E[8]};
    const double x2tEx1 = x2 * Ex1[0] + y2 * Ex1[1] + Ex1[2];
    const double a = Ex1[0] * Ex1[0] + Ex1[1] * Ex1[1];
    const double b = Etx2[0] * Etx2[0] + Etx2[1] * Etx2[1];
    return x2tEx1 * x2tEx1 / (a + b);
}

__device__ int update_num_iters5(double p, double ep, int max_iters) {
    p = fmax(p, 0.0);
    p = fmin(p, 1.0);
    ep = fmax(ep, 0.0);
    ep = fmin(ep, 1.0);
    double num = fmax(1.0 - p, DBL_MIN);
    const double x = 1.0 - ep;
    double denom = 1.0 - ((x * x) * (x * x)) * x;
    if (denom < DBL_MIN) return 0;
    num = log(num);
    denom = log(denom);
    return denom >= 0.0 || -num >= (double)max_iters * -denom ? max_iters : (int)rint(num / denom);
}

// normalised coordinates of match i (findEssentialMat / recoverPose with a camera matrix)
__device__ __forceinline__ void norm_pts(const float* p1, const float* p2, int i, const double* K, double* q) {
    q[0] = ((double)p1[2 * i] - K[2]) / K[0];
    q[1] = ((double)p1[2 * i + 1] - K[3]) / K[1];
    q[2] = ((double)p2[2 * i] - K[2]) / K[0];
    q[3] = ((double)p2[2 * i + 1] - K[3]) / K[1];
}

__device__ __forceinline__ void block_count(int flag, int* lds_cnt) {
    const uint64_t b = __ballot(flag);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(lds_cnt, __popcll(b));
}

__global__ void __launch_bounds__(kThreads) k_em_hyp(EmArgs a, int h0, const int* gate) {
    const int p = blockIdx.y, h = h0 + blockIdx.x, lane = threadIdx.x;
    const vx_essential_options o = a.opt[p];
    const int H = min(max(o.max_iterations, 0), kMaxHyp);
    if (h >= H || (gate && h >= gate[p])) return;
    const int b = a.offsets[p], n = a.offsets[p + 1] - b;
    const float* p1 = a.p1 + 2 * (size_t)b;
    const float* p2 = a.p2 + 2 * (size_t)b;
    const double K[4] = {a.intr[4 * p], a.intr[4 * p + 1], a.intr[4 * p + 2], a.intr[4 * p + 3]};
    __shared__ FpWork w;
    __shared__ double sE[kMaxModels * 9];
    __shared__ int sgot, scnt[kMaxModels];
    if (lane < kMaxModels) scnt[lane] = 0;
    if (lane == 0) {
        int idx[5];
        int got = 0;
        if (n >= 5) {
            for (int at = 0; at < 64 && got < 5; ++at) {
                const uint64_t x = mix64(o.seed + (uint64_t)h * 64u + (uint64_t)at);
                const int i = (int)(((x >> 32) * (uint64_t)n) >> 32);
                bool dup = false;
                for (int k = 0; k < got; ++k) dup |= idx[k] == i;
                if (!dup) idx[got++] = i;
            }
        }
        if (got == 5) {
            double q[4];
            for (int k = 0; k < 5; ++k) {
                norm_pts(p1, p2, idx[k], K, q);
                w.s1[2 * k] = q[0];
                w.s1[2 * k + 1] = q[1];
                w.s2[2 * k] = q[2];
                w.s2[2 * k + 1] = q[3];
            }
        }
        sgot = got;
    }
    WSYNC;
    const int nm = sgot == 5 ? five_point_wave(w, sE, lane) : 0;
    const double thr = o.threshold / ((K[0] + K[1]) * 0.5);
    const double thr2 = thr * thr;
    for (int i0 = 0; i0 < n && nm > 0; i0 += kThreads) {
        const int i = i0 + lane;
        double q[4] = {0.0, 0.0, 0.0, 0.0};
        if (i < n) norm_pts(p1, p2, i, K, q);
        for (int m = 0; m < nm; ++m)
            block_count(i < n && sampson(sE + 9 * m, q[0], q[1], q[2], q[3]) <= thr2, &scnt[m]);
    }
    WSYNC;
    EmRec* r = a.rec + (size_t)p * a.hmax + h;
    for (int e = lane; e < nm * 9; e += kThreads) r->E[e / 9][e % 9] = sE[e];
    if (lane < kMaxModels) r->count[lane] = lane < nm ? scnt[lane] : -1;
    if (lane == 0) r->nm = nm;
}

// ---------------------------------------------------------------- recoverPose
__device__ void jacobi_svd3(const double* A, double* U, double* S, double* V) {
    double B[9];
    for (int k = 0; k < 9; ++k) B[k] = A[k];
    for (int k = 0; k < 9; ++k) V[k] = (k % 4 == 0) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 30; ++sweep) {
        bool rotated = false;
        for (int p = 0; p < 2; ++p)
            for (int q = p + 1; q < 3; ++q) {
                double alpha = 0.0, beta = 0.0, gamma = 0.0;
                for (int r = 0; r < 3; ++r) {
                    alpha += B[3 * r + p] * B[3 * r + p];
                    beta += B[3 * r + q] * B[3 * r + q];
                    gamma += B[3 * r + p] * B[3 * r + q];
                }
                if (!(fabs(gamma) > 1e-15 * sqrt(alpha * beta))) continue;
                rotated = true;
                const double zeta = (beta - alpha) / (2.0 * gamma);
                const double t = (zeta >= 0.0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
                for (int r = 0; r < 3; ++r) {
                    const double bp = B[3 * r + p], bq = B[3 * r + q];
                    B[3 * r + p] = c * bp - s * bq;
                    B[3 * r + q] = s * bp + c * bq;
                    const double vp = V[3 * r + p], vq = V[3 * r + q];
                    V[3 * r + p] = c * vp - s * vq;
                    V[3 * r + q] = s * vp + c * vq;
                }
            }
        if (!rotated) break;
    }
    double sv[3];
    for (int c = 0; c < 3; ++c) sv[c] = sqrt(B[c] * B[c] + B[3 + c] * B[3 + c] + B[6 + c] * B[6 + c]);
    int ord[3] = {0, 1, 2};
    for (int i = 0; i < 3; ++i)
        for (int j = i + 1; j < 3; ++j)
            if (sv[ord[j]] > sv[ord[i]]) swp(ord[i], ord[j]);
    double Vs[9];
    for (int c = 0; c < 3; ++c) {
        S[c] = sv[ord[c]];
        for (int r = 0; r < 3; ++r) {
            Vs[3 * r + c] = V[3 * r + ord[c]];
            U[3 * r + c] = S[c] > 0.0 ? B[3 * r + ord[c]] / S[c] : 0.0;
        }
    }
    for (int k = 0; k < 9; ++k) V[k] = Vs[k];
    U[2] = U[3] * U[7] - U[6] * U[4];
    U[5] = U[6] * U[1] - U[0] * U[7];
    U[8] = U[0] * U[4] - U[3] * U[1];
}

__device__ __forceinline__ double det3(const double* M) {
    return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) + M[2] * (M[3] * M[7] - M[4] * M[6]);
}

__device__ void triangulate(const double* R, const double* t, double x1, double y1, double x2, double y2, double* X) {
    double A[16] = {-1.0, 0.0, x1, 0.0, 0.0, -1.0, y1, 0.0,
                    x2 * R[6] - R[0], x2 * R[7] - R[1], x2 * R[8] - R[2], x2 * t[2] - t[0],
                    y2 * R[6] - R[3], y2 * R[7] - R[4], y2 * R[8] - R[5], y2 * t[2] - t[1]};
    double V[16];
    for (int k = 0; k < 16; ++k) V[k] = (k % 5 == 0) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 12; ++sweep) {
        bool rotated = false;
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int q = p + 1; q < 4; ++q) {
                double alpha = 0.0, beta = 0.0, gamma = 0.0;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    alpha += A[4 * r + p] * A[4 * r + p];
                    beta += A[4 * r + q] * A[4 * r + q];
                    gamma += A[4 * r + p] * A[4 * r + q];
                }
                if (!(fabs(gamma) > 1e-12 * sqrt(alpha * beta))) continue;
                rotated = true;
                const double zeta = (beta - alpha) / (2.0 * gamma);
                const double tt = (zeta >= 0.0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / sqrt(1.0 + tt * tt), s = c * tt;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const double ap = A[4 * r + p], aq = A[4 * r + q];
                    A[4 * r + p] = c * ap - s * aq;
                    A[4 * r + q] = s * ap + c * aq;
                    const double vp = V[4 * r + p], vq = V[4 * r + q];
                    V[4 * r + p] = c * vp - s * vq;
                    V[4 * r + q] = s * vp + c * vq;
                }
            }
        if (!rotated) break;
    }
    int best = 0;
    double bn = INFINITY;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const double nrm = A[c] * A[c] + A[4 + c] * A[4 + c] + A[8 + c] * A[8 + c] + A[12 + c] * A[12 + c];
        if (nrm < bn) {
            bn = nrm;
            best = c;
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {  // X[r] = V[4 r + best], selected without dynamic register indexing
        double xr = V[4 * r];
#pragma unroll
        for (int c = 1; c < 4; ++c)
            if (best == c) xr = V[4 * r + c];
        X[r] = xr;
    }
}

__device__ __forceinline__ bool cheirality(const double* R, const double* t, const double* X, double dist) {
    if (!(X[2] * X[3] > 0.0)) return false;
    const double px = X[0] / X[3], py = X[1] / X[3], pz = X[2] / X[3];
    if (!(pz < dist)) return false;
    const double z2 = R[6] * px + R[7] * py + R[8] * pz + t[2];
    return z2 > 0.0 && z2 < dist;
}

// RANSACPointSetRegistrator::run replayed by wave 0 over the (hypothesis, model) records in
// order, 64 at a time (in-wave prefix max + ballot finds the entries that beat every earlier
// count and 4; the budget test applies when a new hypothesis starts, as in the sequential loop).
__device__ int4 replay(const EmRec* rec, int H, int n, double confidence, int hlimit = kMaxHyp,
                       int* budget = nullptr) {
    const int lane = threadIdx.x & 63;
    int niters = n >= 5 ? H : 0, best = -1, good = 0, last_h = -1;
    bool stop = false;
    for (int base = 0; !stop && base < min(niters, hlimit) * kMaxModels; base += 64) {
        const int f = base + lane;
        const int h = f / kMaxModels, m = f - h * kMaxModels;
        const int c = h < niters && h < hlimit ? rec[h].count[m] : -1;
        int incl = c;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(incl, off);
            if (lane >= off) incl = max(incl, y);
        }
        int excl = __shfl_up(incl, 1);
        if (lane == 0) excl = -1;
        uint64_t bits = __ballot(c > max(max(excl, good), 4));
        while (bits) {
            const int k = __ffsll((unsigned long long)bits) - 1;
            const int fk = base + k, hk = fk / kMaxModels;
            if (hk != last_h && hk >= niters) {
                stop = true;
                break;
            }
            const int ck = __shfl(c, k);
            best = fk;
            last_h = hk;
            good = ck;
            niters = update_num_iters5(confidence, (double)(n - ck) / (double)n, niters);
            bits &= bits - 1;
        }
    }
    const int hb = best >= 0 ? best / kMaxModels : -1;
    if (budget) *budget = stop ? 0 : niters;
    return make_int4(hb, best >= 0 ? best - hb * kMaxModels : -1, best >= 0 ? max(niters, hb + 1) : niters, good);
}

// k_em_gate: after the first kFirstChunk hypotheses, the budget the sequential loop has left
// (RANSACUpdateNumIters only shrinks it): later hypotheses at or beyond it are never evaluated, so
// the second k_em_hyp launch skips them (0 when the loop already ended inside the first chunk)
constexpr int kFirstChunk = 128;
__global__ void __launch_bounds__(64) k_em_gate(EmArgs a, int* gate) {
    const int p = blockIdx.x;
    const vx_essential_options o = a.opt[p];
    const int H = min(max(o.max_iterations, 0), kMaxHyp);
    const int n = a.offsets[p + 1] - a.offsets[p];
    int budget = 0;
    replay(a.rec + (size_t)p * a.hmax, H, n, o.confidence, kFirstChunk, &budget);
    if (threadIdx.x == 0) gate[p] = budget <= kFirstChunk ? 0 : budget;
}

// per-problem state between the three recoverPose kernels
struct EmState {
    int h, m, run, good;
    int cnt[4];
    double E[9], R[2][9], t[3];
};

// k_em_pick: one wave per problem — the loop replay, the kept E, its decomposition
__global__ void __launch_bounds__(64) k_em_pick(EmArgs a, EmState* st) {
    const int p = blockIdx.x;
    const vx_essential_options o = a.opt[p];
    const int H = min(max(o.max_iterations, 0), kMaxHyp);
    const int n = a.offsets[p + 1] - a.offsets[p];
    const EmRec* rec = a.rec + (size_t)p * a.hmax;
    EmState* s = st + p;
    const int4 r = replay(rec, H, n, o.confidence);
    if (threadIdx.x < 4) s->cnt[threadIdx.x] = 0;
    if (threadIdx.x != 0) return;
    s->h = r.x;
    s->m = r.y;
    s->run = r.z;
    s->good = r.w;
    if (r.x < 0) return;
    double E[9], U[9], S[3], V[9];
    for (int k = 0; k < 9; ++k) E[k] = s->E[k] = rec[r.x].E[r.y][k];
    jacobi_svd3(E, U, S, V);
    if (det3(V) < 0.0)
        for (int k = 0; k < 9; ++k) V[k] = -V[k];
    const double W[9] = {0, 1, 0, -1, 0, 0, 0, 0, 1};
    double UW[9], UWt[9];
    for (int rr = 0; rr < 3; ++rr)
        for (int c = 0; c < 3; ++c) {
            UW[3 * rr + c] = U[3 * rr] * W[c] + U[3 * rr + 1] * W[3 + c] + U[3 * rr + 2] * W[6 + c];
            UWt[3 * rr + c] = U[3 * rr] * W[3 * c] + U[3 * rr + 1] * W[3 * c + 1] + U[3 * rr + 2] * W[3 * c + 2];
        }
    for (int rr = 0; rr < 3; ++rr)
        for (int c = 0; c < 3; ++c) {
            s->R[0][3 * rr + c] = UW[3 * rr] * V[3 * c] + UW[3 * rr + 1] * V[3 * c + 1] + UW[3 * rr + 2] * V[3 * c + 2];
            s->R[1][3 * rr + c] = UWt[3 * rr] * V[3 * c] + UWt[3 * rr + 1] * V[3 * c + 1] + UWt[3 * rr + 2] * V[3 * c + 2];
        }
    s->t[0] = U[2];
    s->t[1] = U[5];
    s->t[2] = U[8];
}

// k_em_cheir: one thread per match — RANSAC inlier test under the kept E and, for inliers, DLT
// triangulation under (R1, t) and (R2, t) (the -t candidates reuse them with w negated); flags
// (bit 0 inlier, bit 1 + k candidate k in front) into the mask buffer, per-candidate counts
__global__ void __launch_bounds__(kThreads * 4) k_em_cheir(EmArgs a, const EmState* st) {
    const int p = blockIdx.y;
    const EmState* s = st + p;
    if (s->h < 0) return;
    const int b = a.offsets[p], n = a.offsets[p + 1] - b;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (blockIdx.x * blockDim.x >= n) return;
    const vx_essential_options o = a.opt[p];
    const double K[4] = {a.intr[4 * p], a.intr[4 * p + 1], a.intr[4 * p + 2], a.intr[4 * p + 3]};
    const double thr = o.threshold / ((K[0] + K[1]) * 0.5);
    const double thr2 = thr * thr;
    __shared__ int scnt[4];
    if (threadIdx.x < 4) scnt[threadIdx.x] = 0;
    __syncthreads();
    bool f[4] = {false, false, false, false};
    if (i < n) {
        double q[4], E[9];
        norm_pts(a.p1 + 2 * (size_t)b, a.p2 + 2 * (size_t)b, i, K, q);
        for (int k = 0; k < 9; ++k) E[k] = s->E[k];
        const bool in = sampson(E, q[0], q[1], q[2], q[3]) <= thr2;
        int flags = in ? 1 : 0;
        if (in) {
            double R[9], tp[3], tn[3], X[4];
            for (int k = 0; k < 3; ++k) {
                tp[k] = s->t[k];
                tn[k] = -s->t[k];
            }
            for (int c = 0; c < 2; ++c) {
                for (int k = 0; k < 9; ++k) R[k] = s->R[c][k];
                triangulate(R, tp, q[0], q[1], q[2], q[3], X);
                f[c] = cheirality(R, tp, X, o.distance_thresh);
                X[3] = -X[3];
                f[2 + c] = cheirality(R, tn, X, o.distance_thresh);
            }
            for (int k = 0; k < 4; ++k) flags |= f[k] ? 2 << k : 0;
        }
        a.mask[b + i] = (uint8_t)flags;
    }
    for (int k = 0; k < 4; ++k) block_count(f[k], &scnt[k]);
    __syncthreads();
    if (threadIdx.x < 4 && scnt[threadIdx.x]) atomicAdd(const_cast<int*>(&s->cnt[threadIdx.x]), scnt[threadIdx.x]);
}

__device__ __forceinline__ int pick_candidate(const int* g) {
    if (g[0] >= g[1] && g[0] >= g[2] && g[0] >= g[3]) return 0;
    if (g[1] >= g[0] && g[1] >= g[2] && g[1] >= g[3]) return 1;
    if (g[2] >= g[0] && g[2] >= g[1] && g[2] >= g[3]) return 2;
    return 3;
}

// k_em_final: recoverPose's candidate choice (OpenCV's tie order), the output mask, the result
__global__ void __launch_bounds__(kThreads * 4) k_em_final(EmArgs a, const EmState* st) {
    const int p = blockIdx.y;
    const EmState* s = st + p;
    const int b = a.offsets[p], n = a.offsets[p + 1] - b;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    int g[4];
    for (int k = 0; k < 4; ++k) g[k] = s->cnt[k];
    const int sel = pick_candidate(g);
    if (i < n) a.mask[b + i] = s->h >= 0 && (a.mask[b + i] & (2 << sel)) ? 1 : 0;
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    vx_essential_result z{};
    z.best_hypothesis = s->h;
    z.best_model = s->m;
    z.hypotheses_run = s->run;
    if (s->h < 0) {
        z.best_model = -1;
        z.R[0] = z.R[4] = z.R[8] = 1.0;
    } else {
        z.ok = 1;
        z.n_inliers = g[sel];
        z.n_ransac_inliers = s->good;
        z.pose_candidate = sel;
        for (int k = 0; k < 9; ++k) {
            z.E[k] = s->E[k];
            z.R[k] = s->R[sel & 1][k];
        }
        for (int k = 0; k < 3; ++k) z.t[k] = sel >= 2 ? -s->t[k] : s->t[k];
    }
    a.out[p] = z;
}

size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

}  // namespace
}  // namespace vx

using namespace vx;

static_assert(sizeof(vx_essential_options) == 40, "vx_essential_options layout (python EM_OPTIONS_DTYPE)");
static_assert(sizeof(vx_essential_result) == 200, "vx_essential_result layout (python EM_RESULT_DTYPE)");

extern "C" {

void vx_essential_default_options(vx_essential_options* o) {
    if (!o) return;
    o->max_iterations = 1000;  // cv::findEssentialMat maxIters default
    o->reserved = 0;
    o->threshold = 1.0;        // tracking.cpp:521
    o->confidence = 0.999;     // tracking.cpp:521
    o->distance_thresh = 50.0; // cv::recoverPose default
    o->seed = 0x5EEDull;
}

int vx_essential_ransac_batch(vx_ctx* c, int P, const int32_t* offsets, const float* p1, const float* p2,
                              const double* intr4, const vx_essential_options* opt, uint8_t* mask,
                              vx_essential_result* out) {
    if (!c || P < 0 || (P > 0 && (!offsets || !intr4 || !opt || !out)))
        return c ? set_error(c, VX_ERR_INVALID, "vx_essential_ransac_batch: bad arguments") : VX_ERR_INVALID;
    if (P == 0) return VX_OK;
    if (P > 65535) return set_error(c, VX_ERR_INVALID, "at most 65535 problems per batch");
    if (offsets[0] != 0) return set_error(c, VX_ERR_INVALID, "offsets[0] must be 0");
    int hmax = 1;
    for (int p = 0; p < P; ++p) {
        if (offsets[p + 1] < offsets[p]) return set_error(c, VX_ERR_INVALID, "offsets must be non-decreasing");
        if (opt[p].max_iterations > kMaxHyp)
            return set_error(c, VX_ERR_INVALID, "max_iterations %d > %d", opt[p].max_iterations, kMaxHyp);
        if (!(opt[p].threshold >= 0.0)) return set_error(c, VX_ERR_INVALID, "bad threshold (problem %d)", p);
        const double* k = intr4 + 4 * p;
        if (!(k[0] != 0.0 && k[1] != 0.0 && k[0] + k[1] != 0.0))
            return set_error(c, VX_ERR_INVALID, "bad focal length (problem %d)", p);
        hmax = std::max(hmax, opt[p].max_iterations);
    }
    const int64_t N = offsets[P];
    if (N > 0 && (!p1 || !p2)) return set_error(c, VX_ERR_INVALID, "vx_essential_ransac_batch: null points");
    if (N > INT32_MAX / 2) return set_error(c, VX_ERR_INVALID, "too many matches");
    VX_HIP(c, hipSetDevice(c->device));
    const size_t o_off = 0, o_intr = align16(o_off + (P + 1) * sizeof(int32_t)),
                 o_opt = align16(o_intr + (size_t)P * 4 * sizeof(double)),
                 o_p1 = align16(o_opt + (size_t)P * sizeof(vx_essential_options)),
                 o_p2 = align16(o_p1 + (size_t)N * 2 * sizeof(float)),
                 in_bytes = align16(o_p2 + (size_t)N * 2 * sizeof(float));
    VX_HIP(c, c->rs_host.ensure(in_bytes));
    uint8_t* hs = static_cast<uint8_t*>(c->rs_host.p);
    std::memcpy(hs + o_off, offsets, (P + 1) * sizeof(int32_t));
    std::memcpy(hs + o_intr, intr4, (size_t)P * 4 * sizeof(double));
    std::memcpy(hs + o_opt, opt, (size_t)P * sizeof(vx_essential_options));
    if (N) {
        std::memcpy(hs + o_p1, p1, (size_t)N * 2 * sizeof(float));
        std::memcpy(hs + o_p2, p2, (size_t)N * 2 * sizeof(float));
    }
    VX_HIP(c, c->rs_in.ensure(in_bytes));
    VX_HIP(c, hipMemcpyAsync(c->rs_in.p, hs, in_bytes, hipMemcpyHostToDevice, c->stream));
    const size_t rec_bytes = align16((size_t)P * hmax * sizeof(EmRec));
    VX_HIP(c, c->rs_hyp.ensure(rec_bytes + (size_t)P * (sizeof(EmState) + sizeof(int))));
    int nmax = 1;
    for (int p = 0; p < P; ++p) nmax = std::max(nmax, offsets[p + 1] - offsets[p]);
    const size_t out_bytes = align16((size_t)P * sizeof(vx_essential_result)) + (size_t)std::max<int64_t>(N, 1);
    VX_HIP(c, c->rs_out.ensure(out_bytes));
    uint8_t* din = c->rs_in.as<uint8_t>();
    EmArgs a{};
    a.offsets = reinterpret_cast<const int*>(din + o_off);
    a.intr = reinterpret_cast<const double*>(din + o_intr);
    a.opt = reinterpret_cast<const vx_essential_options*>(din + o_opt);
    a.p1 = reinterpret_cast<const float*>(din + o_p1);
    a.p2 = reinterpret_cast<const float*>(din + o_p2);
    a.rec = c->rs_hyp.as<EmRec>();
    a.hmax = hmax;
    a.out = c->rs_out.as<vx_essential_result>();
    a.mask = c->rs_out.as<uint8_t>() + align16((size_t)P * sizeof(vx_essential_result));
    int* gate = reinterpret_cast<int*>(c->rs_hyp.as<uint8_t>() + rec_bytes + (size_t)P * sizeof(EmState));
    // everything at once while the whole hypothesis grid is resident at the same time (8 one-wave
    // workgroups per CU at this kernel's register count); beyond that, gate by the remaining budget
    if (!c->n_cus) c->n_cus = std::max(vx_device_cus(c->device), 1);
    const int first = (int64_t)P * hmax <= 8 * (int64_t)c->n_cus ? hmax : std::min(hmax, kFirstChunk);
    VX_HIP(c, launch(c, kStEmHyp, k_em_hyp, dim3(first, P), dim3(kThreads), 0, c->stream, a, 0, (const int*)nullptr));
    if (hmax > first) {
        VX_HIP(c, launch(c, kStEmSelect, k_em_gate, dim3(P), dim3(64), 0, c->stream, a, gate));
        VX_HIP(c, launch(c, kStEmHyp, k_em_hyp, dim3(hmax - first, P), dim3(kThreads), 0, c->stream, a, first,
                         (const int*)gate));
    }
    EmState* st = reinterpret_cast<EmState*>(c->rs_hyp.as<uint8_t>() + rec_bytes);
    const dim3 pgrid((nmax + 4 * kThreads - 1) / (4 * kThreads), P);
    VX_HIP(c, launch(c, kStEmSelect, k_em_pick, dim3(P), dim3(64), 0, c->stream, a, st));
    VX_HIP(c, launch(c, kStEmSelect, k_em_cheir, pgrid, dim3(4 * kThreads), 0, c->stream, a, (const EmState*)st));
    VX_HIP(c, launch(c, kStEmSelect, k_em_final, pgrid, dim3(4 * kThreads), 0, c->stream, a, (const EmState*)st));
    VX_HIP(c, c->rs_host_out.ensure(out_bytes));
    VX_HIP(c, hipMemcpyAsync(c->rs_host_out.p, c->rs_out.p, out_bytes, hipMemcpyDeviceToHost, c->stream));
    VX_HIP(c, hipStreamSynchronize(c->stream));
    const uint8_t* ho = static_cast<const uint8_t*>(c->rs_host_out.p);
    std::memcpy(out, ho, (size_t)P * sizeof(vx_essential_result));
    if (mask && N) std::memcpy(mask, ho + align16((size_t)P * sizeof(vx_essential_result)), (size_t)N);
    return VX_OK;
}

int vx_essential_ransac(vx_ctx* c, const float* p1, const float* p2, int n, const double* intr4,
                        const vx_essential_options* opt, uint8_t* mask, vx_essential_result* out) {
    if (!c || n < 0 || !intr4 || !opt || !out)
        return c ? set_error(c, VX_ERR_INVALID, "vx_essential_ransac: bad arguments") : VX_ERR_INVALID;
    const int32_t offsets[2] = {0, n};
    return vx_essential_ransac_batch(c, 1, offsets, p1, p2, intr4, opt, mask, out);
}

}  // extern "C"
