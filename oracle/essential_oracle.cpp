// essential_oracle.cpp — CPU restatement of the essential-matrix RANSAC + pose recovery the GPU runs
// for Tracking::EstimatePoseByEssential (core/frontend/tracking.cpp:503-547):
//     E = cv::findEssentialMat(pts_last, pts_curr, K, cv::RANSAC, 0.999, 1.0, mask);
//     inliers = cv::recoverPose(E, pts_last, pts_curr, K, R, t, mask);
// TEST INFRASTRUCTURE ONLY.  The arithmetic lives in OpenCV (calib3d five-point.cpp, ptsetreg.cpp,
// triangulate.cpp; vcpkg opencv4, not installed here), so this file is the SPECIFICATION the build
// chose for the same contract, written independently of csrc/essential.hip:
//   * pixels normalised by K; threshold divided by (fx + fy) / 2 (as findEssentialMat does);
//   * hypothesis h samples 5 distinct correspondences from a splitmix64 counter stream;
//   * five-point solver: null space of the 5 x 9 epipolar system (Gauss-Jordan, full pivoting),
//     E = xX + yY + zZ + W, the ten cubic constraints det(E) = 0 and 2 E E^T E - tr(E E^T) E = 0 as a
//     10 x 20 matrix over the monomials [cubics | x^2 xy xz y^2 yz z^2 x y z 1], Gauss-Jordan on its
//     cubic block, the 10 x 10 action matrix of multiplication by x, its real eigenvalues (Hessenberg
//     reduction + Francis double-shift QR) and eigenvectors (null vectors of A - lambda I);
//   * Sampson error, inlier if <= thr^2; the sequential RANSACPointSetRegistrator::run loop
//     (modelPoints 5, every model of a sample scored, budget shrunk by RANSACUpdateNumIters);
//   * recoverPose: E = U diag V^T (one-sided Jacobi), R1 = U W V^T, R2 = U W^T V^T, t = U e3, the
//     four (R, +-t) scored by DLT triangulation (positive depth < 50 in both views, within the
//     RANSAC mask), OpenCV's tie order.
// Only + - * / and sqrt are used, in a fixed order, so the GPU reproduces every decision bit for
// bit.  Pinned by tests/test_essential_cpu.py (constraints, ground truth, numpy re-derivations).
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "oracle.h"

namespace {

uint64_t mix64(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

// ---------------------------------------------------------------- polynomials in x, y, z
// degree 1: [x y z 1]; degree 2: [x2 xy xz y2 yz z2 x y z 1];
// degree 3: [x3 x2y x2z xy2 xyz xz2 y3 y2z yz2 z3 | x2 xy xz y2 yz z2 x y z 1]
const int kE1[4][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 0}};
const int kE2[10][3] = {{2, 0, 0}, {1, 1, 0}, {1, 0, 1}, {0, 2, 0}, {0, 1, 1}, {0, 0, 2},
                        {1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 0}};
const int kE3[20][3] = {{3, 0, 0}, {2, 1, 0}, {2, 0, 1}, {1, 2, 0}, {1, 1, 1}, {1, 0, 2}, {0, 3, 0},
                        {0, 2, 1}, {0, 1, 2}, {0, 0, 3}, {2, 0, 0}, {1, 1, 0}, {1, 0, 1}, {0, 2, 0},
                        {0, 1, 1}, {0, 0, 2}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 0}};

int find_mon(const int (*tab)[3], int n, int a, int b, int c) {
    for (int k = 0; k < n; ++k)
        if (tab[k][0] == a && tab[k][1] == b && tab[k][2] == c) return k;
    return -1;
}

struct MulTabs {
    int m11[4][4], m21[10][4];
    MulTabs() {
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j)
                m11[i][j] = find_mon(kE2, 10, kE1[i][0] + kE1[j][0], kE1[i][1] + kE1[j][1], kE1[i][2] + kE1[j][2]);
        for (int i = 0; i < 10; ++i)
            for (int j = 0; j < 4; ++j)
                m21[i][j] = find_mon(kE3, 20, kE2[i][0] + kE1[j][0], kE2[i][1] + kE1[j][1], kE2[i][2] + kE1[j][2]);
    }
};
const MulTabs kTabs;

// c (deg 2) = a * b (deg 1), accumulated in (i, j) order
void mul11(const double* a, const double* b, double* c) {
    for (int k = 0; k < 10; ++k) c[k] = 0.0;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) c[kTabs.m11[i][j]] += a[i] * b[j];
}
// c (deg 3) += p (deg 2) * a (deg 1)
void mul21_acc(const double* p, const double* a, double* c) {
    for (int i = 0; i < 10; ++i)
        for (int j = 0; j < 4; ++j) c[kTabs.m21[i][j]] += p[i] * a[j];
}

// ---------------------------------------------------------------- dense helpers
// Francis double-shift QR on an upper Hessenberg matrix (n x n, row-major, destroyed): eigenvalues
// (wr, wi).  false if an eigenvalue needs more than 30 iterations.
bool hqr(double* a, int n, double* wr, double* wi) {
    auto A = [&](int i, int j) -> double& { return a[i * n + j]; };
    double anorm = 0.0;
    for (int i = 0; i < n; ++i)
        for (int j = std::max(i - 1, 0); j < n; ++j) anorm += std::fabs(A(i, j));
    int nn = n - 1;
    double t = 0.0;
    while (nn >= 0) {
        int its = 0, l;
        do {
            for (l = nn; l >= 1; --l) {
                double s = std::fabs(A(l - 1, l - 1)) + std::fabs(A(l, l));
                if (s == 0.0) s = anorm;
                if (std::fabs(A(l, l - 1)) <= DBL_EPSILON * s) {
                    A(l, l - 1) = 0.0;
                    break;
                }
            }
            double x = A(nn, nn);
            if (l == nn) {
                wr[nn] = x + t;
                wi[nn] = 0.0;
                --nn;
            } else {
                double y = A(nn - 1, nn - 1);
                double w = A(nn, nn - 1) * A(nn - 1, nn);
                if (l == nn - 1) {
                    const double p = 0.5 * (y - x);
                    const double q = p * p + w;
                    double z = std::sqrt(std::fabs(q));
                    x += t;
                    if (q >= 0.0) {
                        z = p + (p >= 0.0 ? std::fabs(z) : -std::fabs(z));
                        wr[nn - 1] = wr[nn] = x + z;
                        if (z != 0.0) wr[nn] = x - w / z;
                        wi[nn - 1] = wi[nn] = 0.0;
                    } else {
                        wr[nn - 1] = wr[nn] = x + p;
                        wi[nn - 1] = -z;
                        wi[nn] = z;
                    }
                    nn -= 2;
                } else {
                    if (its == 30) return false;
                    if (its == 10 || its == 20) {
                        t += x;
                        for (int i = 0; i <= nn; ++i) A(i, i) -= x;
                        const double s = std::fabs(A(nn, nn - 1)) + std::fabs(A(nn - 1, nn - 2));
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
                        s = std::fabs(p) + std::fabs(q) + std::fabs(r);
                        p /= s;
                        q /= s;
                        r /= s;
                        if (m == l) break;
                        const double u = std::fabs(A(m, m - 1)) * (std::fabs(q) + std::fabs(r));
                        const double v = std::fabs(p) * (std::fabs(A(m - 1, m - 1)) + std::fabs(z) + std::fabs(A(m + 1, m + 1)));
                        if (u <= DBL_EPSILON * v) break;
                    }
                    for (int i = m + 2; i <= nn; ++i) {
                        A(i, i - 2) = 0.0;
                        if (i != m + 2) A(i, i - 3) = 0.0;
                    }
                    for (int k = m; k <= nn - 1; ++k) {
                        if (k != m) {
                            p = A(k, k - 1);
                            q = A(k + 1, k - 1);
                            r = 0.0;
                            if (k != nn - 1) r = A(k + 2, k - 1);
                            x = std::fabs(p) + std::fabs(q) + std::fabs(r);
                            if (x != 0.0) {
                                p /= x;
                                q /= x;
                                r /= x;
                            }
                        }
                        const double sq = std::sqrt(p * p + q * q + r * r);
                        const double s = p >= 0.0 ? sq : -sq;
                        if (s != 0.0) {
                            if (k == m) {
                                if (l != m) A(k, k - 1) = -A(k, k - 1);
                            } else {
                                A(k, k - 1) = -s * x;
                            }
                            p += s;
                            x = p / s;
                            y = q / s;
                            z = r / s;
                            q /= p;
                            r /= p;
                            for (int j = k; j <= nn; ++j) {
                                p = A(k, j) + q * A(k + 1, j);
                                if (k != nn - 1) {
                                    p += r * A(k + 2, j);
                                    A(k + 2, j) -= p * z;
                                }
                                A(k + 1, j) -= p * y;
                                A(k, j) -= p * x;
                            }
                            const int mmin = nn < k + 3 ? nn : k + 3;
                            for (int i = l; i <= mmin; ++i) {
                                p = x * A(i, k) + y * A(i, k + 1);
                                if (k != nn - 1) {
                                    p += z * A(i, k + 2);
                                    A(i, k + 2) -= p * r;
                                }
                                A(i, k + 1) -= p * q;
                                A(i, k) -= p;
                            }
                        }
                    }
                }
            }
        } while (nn >= 0 && l < nn - 1);
    }
    return true;
}

// reduction to upper Hessenberg form by stabilised elementary similarity transforms (elmhes)
void elmhes(double* a, int n) {
    auto A = [&](int i, int j) -> double& { return a[i * n + j]; };
    for (int m = 1; m < n - 1; ++m) {
        double x = 0.0;
        int i = m;
        for (int j = m; j < n; ++j) {
            if (std::fabs(A(j, m - 1)) > std::fabs(x)) {
                x = A(j, m - 1);
                i = j;
            }
        }
        if (i != m) {
            for (int j = m - 1; j < n; ++j) std::swap(A(i, j), A(m, j));
            for (int j = 0; j < n; ++j) std::swap(A(j, i), A(j, m));
        }
        if (x != 0.0) {
            for (i = m + 1; i < n; ++i) {
                double y = A(i, m - 1);
                if (y != 0.0) {
                    y /= x;
                    A(i, m - 1) = y;
                    for (int j = m; j < n; ++j) A(i, j) -= y * A(m, j);
                    for (int j = 0; j < n; ++j) A(j, m) += y * A(j, i);
                }
            }
        }
    }
    for (int i = 2; i < n; ++i)
        for (int j = 0; j < i - 1; ++j) A(i, j) = 0.0;
}

// null vector of the n x n matrix a (destroyed) by Gaussian elimination with full pivoting: the
// last pivot is dropped, its unknown set to 1, the rest back-substituted.  false if an earlier pivot
// is zero (null space of dimension > 1).
bool null_vector(double* a, int n, double* v) {
    auto A = [&](int i, int j) -> double& { return a[i * n + j]; };
    int perm[16];
    for (int j = 0; j < n; ++j) perm[j] = j;
    for (int k = 0; k < n - 1; ++k) {
        int bi = k, bj = k;
        double bv = -1.0;
        for (int i = k; i < n; ++i)
            for (int j = k; j < n; ++j)
                if (std::fabs(A(i, j)) > bv) {
                    bv = std::fabs(A(i, j));
                    bi = i;
                    bj = j;
                }
        if (!(bv > 0.0)) return false;
        if (bi != k)
            for (int j = 0; j < n; ++j) std::swap(A(bi, j), A(k, j));
        if (bj != k) {
            for (int i = 0; i < n; ++i) std::swap(A(i, bj), A(i, k));
            std::swap(perm[bj], perm[k]);
        }
        for (int i = k + 1; i < n; ++i) {
            const double f = A(i, k) / A(k, k);
            for (int j = k + 1; j < n; ++j) A(i, j) -= f * A(k, j);
            A(i, k) = 0.0;
        }
    }
    double y[16];
    y[n - 1] = 1.0;
    for (int k = n - 2; k >= 0; --k) {
        double s = 0.0;
        for (int j = k + 1; j < n; ++j) s += A(k, j) * y[j];
        y[k] = -s / A(k, k);
    }
    for (int j = 0; j < n; ++j) v[perm[j]] = y[j];
    return true;
}

// ---------------------------------------------------------------- five-point solver
// x1 / x2: 5 normalised points (pts_last, pts_curr) -> up to 10 essential matrices (row-major),
// x2^T E x1 = 0
int five_point(const double* x1, const double* x2, double* Es) {
    double Q[5 * 9];
    for (int i = 0; i < 5; ++i) {
        const double a[3] = {x1[2 * i], x1[2 * i + 1], 1.0}, b[3] = {x2[2 * i], x2[2 * i + 1], 1.0};
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) Q[9 * i + 3 * r + c] = b[r] * a[c];
    }
    // null space by Gauss-Jordan with full pivoting
    bool used[9] = {};
    int pc[5];
    for (int k = 0; k < 5; ++k) {
        int bi = -1, bj = -1;
        double bv = 0.0;
        for (int i = k; i < 5; ++i)
            for (int j = 0; j < 9; ++j)
                if (!used[j] && std::fabs(Q[9 * i + j]) > bv) {
                    bv = std::fabs(Q[9 * i + j]);
                    bi = i;
                    bj = j;
                }
        if (bi < 0) return 0;
        if (bi != k)
            for (int j = 0; j < 9; ++j) std::swap(Q[9 * bi + j], Q[9 * k + j]);
        used[bj] = true;
        pc[k] = bj;
        const double p = Q[9 * k + bj];
        for (int j = 0; j < 9; ++j) Q[9 * k + j] = j == bj ? 1.0 : Q[9 * k + j] / p;
        for (int r = 0; r < 5; ++r) {
            if (r == k) continue;
            const double f = Q[9 * r + bj];
            for (int j = 0; j < 9; ++j) Q[9 * r + j] = j == bj ? 0.0 : Q[9 * r + j] - f * Q[9 * k + j];
        }
    }
    double basis[4][9];
    int nf = 0;
    for (int f = 0; f < 9; ++f) {
        if (used[f]) continue;
        for (int j = 0; j < 9; ++j) basis[nf][j] = 0.0;
        basis[nf][f] = 1.0;
        for (int k = 0; k < 5; ++k) basis[nf][pc[k]] = -Q[9 * k + f];
        ++nf;
    }
    // E entries as degree-1 polynomials [x y z 1]
    double E[9][4];
    for (int k = 0; k < 9; ++k) {
        E[k][0] = basis[0][k];
        E[k][1] = basis[1][k];
        E[k][2] = basis[2][k];
        E[k][3] = basis[3][k];
    }
    // E E^T (degree 2) and its trace
    double EEt[9][10], tmp[10];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            for (int m = 0; m < 10; ++m) EEt[3 * i + j][m] = 0.0;
            for (int k = 0; k < 3; ++k) {
                mul11(E[3 * i + k], E[3 * j + k], tmp);
                for (int m = 0; m < 10; ++m) EEt[3 * i + j][m] += tmp[m];
            }
        }
    double tr[10];
    for (int m = 0; m < 10; ++m) tr[m] = EEt[0][m] + EEt[4][m] + EEt[8][m];
    double M[10][20];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double acc[20] = {}, te[20] = {};
            for (int k = 0; k < 3; ++k) mul21_acc(EEt[3 * i + k], E[3 * k + j], acc);
            mul21_acc(tr, E[3 * i + j], te);
            for (int m = 0; m < 20; ++m) M[3 * i + j][m] = 2.0 * acc[m] - te[m];
        }
    {  // det(E) by the first row
        double m0[10], m1[10], m2[10], a[10], b[10];
        mul11(E[4], E[8], a); mul11(E[5], E[7], b);
        for (int m = 0; m < 10; ++m) m0[m] = a[m] - b[m];
        mul11(E[3], E[8], a); mul11(E[5], E[6], b);
        for (int m = 0; m < 10; ++m) m1[m] = a[m] - b[m];
        mul11(E[3], E[7], a); mul11(E[4], E[6], b);
        for (int m = 0; m < 10; ++m) m2[m] = a[m] - b[m];
        double d0[20] = {}, d1[20] = {}, d2[20] = {};
        mul21_acc(m0, E[0], d0);
        mul21_acc(m1, E[1], d1);
        mul21_acc(m2, E[2], d2);
        for (int m = 0; m < 20; ++m) M[9][m] = d0[m] - d1[m] + d2[m];
    }
    // Gauss-Jordan on the cubic block (partial pivoting)
    for (int k = 0; k < 10; ++k) {
        int bi = k;
        double bv = std::fabs(M[k][k]);
        for (int i = k + 1; i < 10; ++i)
            if (std::fabs(M[i][k]) > bv) {
                bv = std::fabs(M[i][k]);
                bi = i;
            }
        if (!(bv > 0.0)) return 0;
        if (bi != k)
            for (int j = 0; j < 20; ++j) std::swap(M[bi][j], M[k][j]);
        const double p = M[k][k];
        for (int j = k + 1; j < 20; ++j) M[k][j] = M[k][j] / p;
        M[k][k] = 1.0;
        for (int r = 0; r < 10; ++r) {
            if (r == k) continue;
            const double f = M[r][k];
            if (f == 0.0) continue;
            for (int j = k + 1; j < 20; ++j) M[r][j] -= f * M[k][j];
            M[r][k] = 0.0;
        }
    }
    // action matrix of multiplication by x on the basis [x2 xy xz y2 yz z2 x y z 1]
    double At[100];
    for (int s = 0; s < 6; ++s)
        for (int j = 0; j < 10; ++j) At[10 * s + j] = -M[s][10 + j];
    const int lin[4] = {0, 1, 2, 6};  // x*x = x2, x*y = xy, x*z = xz, x*1 = x
    for (int s = 6; s < 10; ++s)
        for (int j = 0; j < 10; ++j) At[10 * s + j] = j == lin[s - 6] ? 1.0 : 0.0;
    double H[100], wr[10], wi[10];
    std::memcpy(H, At, sizeof(H));
    elmhes(H, 10);
    if (!hqr(H, 10, wr, wi)) return 0;
    int ns = 0;
    for (int k = 0; k < 10; ++k) {
        if (wi[k] != 0.0) continue;
        double B[100], v[10];
        std::memcpy(B, At, sizeof(B));
        for (int d = 0; d < 10; ++d) B[11 * d] -= wr[k];
        if (!null_vector(B, 10, v)) continue;
        if (v[9] == 0.0) continue;
        const double x = v[6] / v[9], y = v[7] / v[9], z = v[8] / v[9];
        double* e = Es + 9 * ns;
        double nrm = 0.0;
        for (int m = 0; m < 9; ++m) {
            e[m] = x * basis[0][m] + y * basis[1][m] + z * basis[2][m] + basis[3][m];
            nrm += e[m] * e[m];
        }
        if (!(nrm > 0.0)) continue;
        const double inv = 1.0 / std::sqrt(nrm);
        for (int m = 0; m < 9; ++m) e[m] = e[m] * inv;
        ++ns;
    }
    return ns;
}

// Sampson distance (EMEstimatorCallback::computeError)
double sampson(const double* E, double x1, double y1, double x2, double y2) {
    const double Ex1[3] = {E[0] * x1 + E[1] * y1 + E[2], E[3] * x1 + E[4] * y1 + E[5], E[6] * x1 + E[7] * y1 + E[8]};
    const double Etx2[3] = {E[0] * x2 + E[3] * y2 + E[6], E[1] * x2 + E[4] * y2 + E[7], E[2] * x2 + E[5] * y2 + E[8]};
    const double x2tEx1 = x2 * Ex1[0] + y2 * Ex1[1] + Ex1[2];
    const double a = Ex1[0] * Ex1[0] + Ex1[1] * Ex1[1];
    const double b = Etx2[0] * Etx2[0] + Etx2[1] * Etx2[1];
    return x2tEx1 * x2tEx1 / (a + b);
}

int update_num_iters5(double p, double ep, int max_iters) {
    p = std::max(p, 0.0);
    p = std::min(p, 1.0);
    ep = std::max(ep, 0.0);
    ep = std::min(ep, 1.0);
    double num = std::max(1.0 - p, DBL_MIN);
    const double x = 1.0 - ep;
    double denom = 1.0 - ((x * x) * (x * x)) * x;
    if (denom < DBL_MIN) return 0;
    num = std::log(num);
    denom = std::log(denom);
    return denom >= 0.0 || -num >= (double)max_iters * -denom ? max_iters : (int)std::rint(num / denom);
}

bool sample5(uint64_t seed, int h, int n, int* idx) {
    int got = 0;
    for (int a = 0; a < 64 && got < 5; ++a) {
        const uint64_t x = mix64(seed + (uint64_t)h * 64u + (uint64_t)a);
        const int i = (int)(((x >> 32) * (uint64_t)n) >> 32);
        bool dup = false;
        for (int k = 0; k < got; ++k) dup |= idx[k] == i;
        if (!dup) idx[got++] = i;
    }
    return got == 5;
}

// ---------------------------------------------------------------- recoverPose
// one-sided Jacobi SVD of a 3 x 3 matrix: A V = U S (columns of A V orthogonal)
void jacobi_svd3(const double* A, double* U, double* S, double* V) {
    double B[9];
    std::memcpy(B, A, sizeof(B));
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
                if (!(std::fabs(gamma) > 1e-15 * std::sqrt(alpha * beta))) continue;
                rotated = true;
                const double zeta = (beta - alpha) / (2.0 * gamma);
                const double t = (zeta >= 0.0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / std::sqrt(1.0 + t * t), s = c * t;
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
    for (int c = 0; c < 3; ++c) sv[c] = std::sqrt(B[c] * B[c] + B[3 + c] * B[3 + c] + B[6 + c] * B[6 + c]);
    int ord[3] = {0, 1, 2};  // descending singular values, stable
    for (int i = 0; i < 3; ++i)
        for (int j = i + 1; j < 3; ++j)
            if (sv[ord[j]] > sv[ord[i]]) std::swap(ord[i], ord[j]);
    double Vs[9];
    for (int c = 0; c < 3; ++c) {
        S[c] = sv[ord[c]];
        for (int r = 0; r < 3; ++r) {
            Vs[3 * r + c] = V[3 * r + ord[c]];
            U[3 * r + c] = S[c] > 0.0 ? B[3 * r + ord[c]] / S[c] : 0.0;
        }
    }
    std::memcpy(V, Vs, sizeof(Vs));
    // rank 2: the third left vector completes a right-handed frame
    U[2] = U[3] * U[7] - U[6] * U[4];
    U[5] = U[6] * U[1] - U[0] * U[7];
    U[8] = U[0] * U[4] - U[3] * U[1];
}

double det3(const double* M) {
    return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) + M[2] * (M[3] * M[7] - M[4] * M[6]);
}

// DLT triangulation of normalised (x1, y1) in [I | 0] and (x2, y2) in [R | t]: the right null
// vector of the 4 x 4 system (one-sided Jacobi on its columns, smallest column norm)
void triangulate(const double* R, const double* t, double x1, double y1, double x2, double y2, double* X) {
    double A[16] = {-1.0, 0.0, x1, 0.0, 0.0, -1.0, y1, 0.0,
                    x2 * R[6] - R[0], x2 * R[7] - R[1], x2 * R[8] - R[2], x2 * t[2] - t[0],
                    y2 * R[6] - R[3], y2 * R[7] - R[4], y2 * R[8] - R[5], y2 * t[2] - t[1]};
    double V[16];
    for (int k = 0; k < 16; ++k) V[k] = (k % 5 == 0) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 12; ++sweep) {
        bool rotated = false;
        for (int p = 0; p < 3; ++p)
            for (int q = p + 1; q < 4; ++q) {
                double alpha = 0.0, beta = 0.0, gamma = 0.0;
                for (int r = 0; r < 4; ++r) {
                    alpha += A[4 * r + p] * A[4 * r + p];
                    beta += A[4 * r + q] * A[4 * r + q];
                    gamma += A[4 * r + p] * A[4 * r + q];
                }
                if (!(std::fabs(gamma) > 1e-12 * std::sqrt(alpha * beta))) continue;  // near-null column: 1e-12 suffices
                rotated = true;
                const double zeta = (beta - alpha) / (2.0 * gamma);
                const double tt = (zeta >= 0.0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / std::sqrt(1.0 + tt * tt), s = c * tt;
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
    for (int c = 0; c < 4; ++c) {
        const double nrm = A[c] * A[c] + A[4 + c] * A[4 + c] + A[8 + c] * A[8 + c] + A[12 + c] * A[12 + c];
        if (nrm < bn) {
            bn = nrm;
            best = c;
        }
    }
    for (int r = 0; r < 4; ++r) X[r] = V[4 * r + best];
}

// cheirality of one correspondence under (R, t): OpenCV recoverPose's tests on the triangulated
// point (z w > 0, depth < dist in the first view, 0 < depth < dist in the second)
bool in_front(const double* R, const double* t, double x1, double y1, double x2, double y2, double dist) {
    double X[4];
    triangulate(R, t, x1, y1, x2, y2, X);
    if (!(X[2] * X[3] > 0.0)) return false;
    const double px = X[0] / X[3], py = X[1] / X[3], pz = X[2] / X[3];
    if (!(pz < dist)) return false;
    const double z2 = R[6] * px + R[7] * py + R[8] * pz + t[2];
    return z2 > 0.0 && z2 < dist;
}

void solve_one(const float* p1, const float* p2, int n, const double* K, const orc_essential_options& o,
               uint8_t* mask, orc_essential_result& res) {
    std::memset(&res, 0, sizeof(res));
    res.best_hypothesis = -1;
    res.best_model = -1;
    res.R[0] = res.R[4] = res.R[8] = 1.0;
    if (mask) std::memset(mask, 0, (size_t)n);
    const int H = std::min(std::max(o.max_iterations, 0), ORC_EM_MAX_HYP);
    if (n < 5 || H == 0) return;
    std::vector<double> x1(2 * (size_t)n), x2(2 * (size_t)n);
    for (int i = 0; i < n; ++i) {
        x1[2 * i] = ((double)p1[2 * i] - K[2]) / K[0];
        x1[2 * i + 1] = ((double)p1[2 * i + 1] - K[3]) / K[1];
        x2[2 * i] = ((double)p2[2 * i] - K[2]) / K[0];
        x2[2 * i + 1] = ((double)p2[2 * i + 1] - K[3]) / K[1];
    }
    const double thr = o.threshold / ((K[0] + K[1]) * 0.5);
    const double thr2 = thr * thr;
    auto count = [&](const double* E, uint8_t* m) {
        int c = 0;
        for (int i = 0; i < n; ++i) {
            const bool in = sampson(E, x1[2 * i], x1[2 * i + 1], x2[2 * i], x2[2 * i + 1]) <= thr2;
            if (m) m[i] = in ? 1 : 0;
            c += in ? 1 : 0;
        }
        return c;
    };
    int niters = H, best_h = -1, best_m = -1, good = 0, h = 0;
    double bestE[9];
    for (; h < niters; ++h) {
        int idx[5];
        if (!sample5(o.seed, h, n, idx)) continue;
        double s1[10], s2[10], Es[90];
        for (int k = 0; k < 5; ++k) {
            s1[2 * k] = x1[2 * idx[k]];
            s1[2 * k + 1] = x1[2 * idx[k] + 1];
            s2[2 * k] = x2[2 * idx[k]];
            s2[2 * k + 1] = x2[2 * idx[k] + 1];
        }
        const int nm = five_point(s1, s2, Es);
        for (int m = 0; m < nm; ++m) {
            const int c = count(Es + 9 * m, nullptr);
            if (c > std::max(good, 4)) {
                best_h = h;
                best_m = m;
                good = c;
                std::memcpy(bestE, Es + 9 * m, sizeof(bestE));
                niters = update_num_iters5(o.confidence, (double)(n - c) / (double)n, niters);
            }
        }
    }
    res.hypotheses_run = h;
    if (best_h < 0) return;
    std::vector<uint8_t> rm(n);
    count(bestE, rm.data());
    res.ok = 1;
    res.best_hypothesis = best_h;
    res.best_model = best_m;
    res.n_ransac_inliers = good;
    std::memcpy(res.E, bestE, sizeof(bestE));
    // recoverPose
    double U[9], S[3], V[9];
    jacobi_svd3(bestE, U, S, V);
    if (det3(V) < 0.0)
        for (double& v : V) v = -v;
    const double W[9] = {0, 1, 0, -1, 0, 0, 0, 0, 1};
    double R1[9], R2[9], UW[9], UWt[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            UW[3 * r + c] = U[3 * r] * W[c] + U[3 * r + 1] * W[3 + c] + U[3 * r + 2] * W[6 + c];
            UWt[3 * r + c] = U[3 * r] * W[3 * c] + U[3 * r + 1] * W[3 * c + 1] + U[3 * r + 2] * W[3 * c + 2];
        }
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {  // X V^T
            R1[3 * r + c] = UW[3 * r] * V[3 * c] + UW[3 * r + 1] * V[3 * c + 1] + UW[3 * r + 2] * V[3 * c + 2];
            R2[3 * r + c] = UWt[3 * r] * V[3 * c] + UWt[3 * r + 1] * V[3 * c + 1] + UWt[3 * r + 2] * V[3 * c + 2];
        }
    const double tp[3] = {U[2], U[5], U[8]}, tn[3] = {-U[2], -U[5], -U[8]};
    const double* Rc[4] = {R1, R2, R1, R2};
    const double* tc[4] = {tp, tp, tn, tn};
    int goodc[4];
    for (int k = 0; k < 4; ++k) {
        goodc[k] = 0;
        for (int i = 0; i < n; ++i)
            if (rm[i] && in_front(Rc[k], tc[k], x1[2 * i], x1[2 * i + 1], x2[2 * i], x2[2 * i + 1], o.distance_thresh))
                ++goodc[k];
    }
    int sel;
    if (goodc[0] >= goodc[1] && goodc[0] >= goodc[2] && goodc[0] >= goodc[3]) sel = 0;
    else if (goodc[1] >= goodc[0] && goodc[1] >= goodc[2] && goodc[1] >= goodc[3]) sel = 1;
    else if (goodc[2] >= goodc[0] && goodc[2] >= goodc[1] && goodc[2] >= goodc[3]) sel = 2;
    else sel = 3;
    res.pose_candidate = sel;
    std::memcpy(res.R, Rc[sel], sizeof(res.R));
    std::memcpy(res.t, tc[sel], sizeof(res.t));
    int npos = 0;
    for (int i = 0; i < n; ++i) {
        const bool keep = rm[i] && in_front(Rc[sel], tc[sel], x1[2 * i], x1[2 * i + 1], x2[2 * i], x2[2 * i + 1],
                                            o.distance_thresh);
        if (mask) mask[i] = keep ? 1 : 0;
        npos += keep ? 1 : 0;
    }
    res.n_inliers = npos;
}

}  // namespace

extern "C" {

int orc_five_point(const double* x1, const double* x2, double* Es) { return five_point(x1, x2, Es); }

int orc_essential_ransac_batch(int n_problems, const int32_t* offsets, const float* pts1, const float* pts2,
                               const double* intr4, const orc_essential_options* opt, uint8_t* mask,
                               orc_essential_result* out) {
    for (int p = 0; p < n_problems; ++p) {
        const int b = offsets[p], n = offsets[p + 1] - offsets[p];
        solve_one(pts1 + 2 * (size_t)b, pts2 + 2 * (size_t)b, n, intr4 + 4 * p, opt[p], mask ? mask + b : nullptr,
                  out[p]);
    }
    return 0;
}

}  // extern "C"
