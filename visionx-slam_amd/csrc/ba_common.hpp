// ba_common.hpp — FP64 / SE(3) / wavefront helpers shared by the LocalBA (ba.hip) and the
// Schur-complement BA (sba.hip) translation units, and the host-side window selection both
// plans start from (SelectKeyFrames + landmark filter, local_ba.cpp:42-108).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <type_traits>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "vx_slam.h"

namespace vx {
namespace ba {

struct D3 { double x, y, z; };

// 1 / b: v_rcp_f64 (~2.5e8 ulp, i.e. ~28 bits) and one Newton step: within 11 ulp (2.4e-15
// relative; scripts/probes/rcp_accuracy.hip on gfx950) instead of the ~12-instruction IEEE division
// sequence, which sits on every dependency chain below — a second step (0 ulp) costs two more
// dependent FMAs.  BA parity is a tolerance (1e-4, gate margins >= 1e-8), not a bit pattern;
// b = 0 / denormal operands do not reach these call sites (gated by the caller).
__device__ __forceinline__ double frcp(double b) {
    const double r = __builtin_amdgcn_rcp(b);
    return fma(fma(-b, r, 1.0), r, r);
}

// 1 / sqrt(x): v_rsq_f64 and one Newton step (within 20 ulp; x > 0 at the call sites).
__device__ __forceinline__ double frsq(double x) {
    const double r = __builtin_amdgcn_rsq(x);
    return r * fma(-(0.5 * x) * r, r, 1.5);
}

// 64-bit cross-lane exchanges for the reduction butterfly, on the VALU instead of the LDS crossbar
// (ds_bpermute): gfx950's v_permlane32/16_swap exchange a register pair across lane halves /
// 16-lane groups; DPP row_ror:8 and quad_perm give xor 8, 2, 1; ds_swizzle's xor mode gives xor 4.
__device__ __forceinline__ void swap_lanes32(double& a, double& b) {
    const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(a), __double2loint(b), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(a), __double2hiint(b), false, false);
    a = __hiloint2double(hi[0], lo[0]);
    b = __hiloint2double(hi[1], lo[1]);
}
__device__ __forceinline__ void swap_lanes16(double& a, double& b) {
    const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(a), __double2loint(b), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(a), __double2hiint(b), false, false);
    a = __hiloint2double(hi[0], lo[0]);
    b = __hiloint2double(hi[1], lo[1]);
}
template <int CTRL>
__device__ __forceinline__ double dpp64(double x) {
    return __hiloint2double(__builtin_amdgcn_update_dpp(0, __double2hiint(x), CTRL, 0xF, 0xF, false),
                            __builtin_amdgcn_update_dpp(0, __double2loint(x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ double xor4_64(double x) {
    constexpr int kXor4 = 0x1F | (4 << 10);  // ds_swizzle bitmask mode: and 0x1F, or 0, xor 4
    return __hiloint2double(__builtin_amdgcn_ds_swizzle(__double2hiint(x), kXor4),
                            __builtin_amdgcn_ds_swizzle(__double2loint(x), kXor4));
}

// Halving butterfly over a wave: r holds 32 terms per lane; afterwards lanes 2t and 2t + 1 hold
// term t summed over the 64 lanes.  Each stage keeps half of the remaining terms (which half is
// chosen by the lane bit of that stage) and adds the partner's copy of it: 16 + 8 + 4 + 2 + 1 + 1
// exchanges instead of 32 x 6.  Fixed order, so the result is deterministic.
__device__ __forceinline__ double wave_sum32(double* r) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < 16; ++i) {  // xor 32: lanes < 32 keep terms 0..15
        swap_lanes32(r[i], r[i + 16]);
        r[i] = r[i] + r[i + 16];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {   // xor 16
        swap_lanes16(r[i], r[i + 8]);
        r[i] = r[i] + r[i + 8];
    }
    {
        const bool up = lane & 8;
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // xor 8: row rotate by 8 within 16-lane rows
            const double send = up ? r[i] : r[i + 4], keep = up ? r[i + 4] : r[i];
            r[i] = keep + dpp64<0x128>(send);
        }
    }
    {
        const bool up = lane & 4;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const double send = up ? r[i] : r[i + 2], keep = up ? r[i + 2] : r[i];
            r[i] = keep + xor4_64(send);
        }
    }
    {
        const bool up = lane & 2;
        const double send = up ? r[0] : r[1], keep = up ? r[1] : r[0];
        r[0] = keep + dpp64<0x4E>(send);  // quad_perm [2,3,0,1]: xor 2
    }
    return r[0] + dpp64<0xB1>(r[0]);      // quad_perm [1,0,3,2]: xor 1
}

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

// Pairwise (tree) sum of v[0..n): log2(n) dependent adds instead of n - 1.
template <int n>
__device__ __forceinline__ double tsum(const double* v) {
    if constexpr (n == 0) return 0.0;
    else if constexpr (n == 1) return v[0];
    else return tsum<n / 2>(v) + tsum<n - n / 2>(v + n / 2);
}

__device__ __forceinline__ D3 cross3(D3 a, D3 b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

// Eigen _transformVector + translation (Sophus SE3 * point)
__device__ __forceinline__ D3 se3_apply(const double* T, D3 p) {
    const D3 qv{T[0], T[1], T[2]};
    D3 uv = cross3(qv, p);
    uv = {uv.x + uv.x, uv.y + uv.y, uv.z + uv.z};
    const D3 c = cross3(qv, uv);
    const double w = T[3];
    return {p.x + w * uv.x + c.x + T[4], p.y + w * uv.y + c.y + T[5], p.z + w * uv.z + c.z + T[6]};
}

// Eigen Quaternion::toRotationMatrix
__device__ __forceinline__ void rot_from_quat(const double* q, double* R) {
    const double tx = 2.0 * q[0], ty = 2.0 * q[1], tz = 2.0 * q[2];
    const double twx = tx * q[3], twy = ty * q[3], twz = tz * q[3];
    const double txx = tx * q[0], txy = ty * q[0], txz = tz * q[0];
    const double tyy = ty * q[1], tyz = tz * q[1], tzz = tz * q[2];
    R[0] = 1.0 - (tyy + tzz); R[1] = txy - twz;         R[2] = txz + twy;
    R[3] = txy + twz;         R[4] = 1.0 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;         R[7] = tyz + twx;         R[8] = 1.0 - (txx + tyy);
}

// Solution of H x = b for the SPD systems of both stages (H = sum w J^T J + 1e-6 I,
// local_ba.cpp:167-168 and :232-233) by an UNPIVOTED LDL^T with tree-summed dot products.  Eigen's
// LDLT pivots on the diagonal; on an SPD matrix the factors are the same up to rounding, and the
// unpivoted form with pairwise sums roughly halves the FP64 dependency chain the solve sits on
// (each dependent FP64 op costs ~35 cycles on gfx950).  Zero pivots are treated as Eigen does
// (column left unscaled, solution component 0).  A: row-major N x N, lower triangle read.
template <int N>
__device__ __forceinline__ void ldlt_spd_solve(const double* A, const double* b, double* x) {
    double L[N][N], d[N], inv[N];
    static_for<0, N>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        double v[N > 1 ? N : 1], t[N > 1 ? N : 1];
#pragma unroll
        for (int j = 0; j < k; ++j) v[j] = L[k][j] * d[j];
#pragma unroll
        for (int j = 0; j < k; ++j) t[j] = L[k][j] * v[j];
        d[k] = A[k * N + k] - tsum<k>(t);
        const bool nz = fabs(d[k]) > 0.0;
        const double ik = nz ? frcp(d[k]) : 1.0;
        inv[k] = fabs(d[k]) > 2.2250738585072014e-308 ? frcp(d[k]) : 0.0;
#pragma unroll
        for (int i = k + 1; i < N; ++i) {
            double u[N > 1 ? N : 1];
#pragma unroll
            for (int j = 0; j < k; ++j) u[j] = L[i][j] * v[j];
            L[i][k] = (A[i * N + k] - tsum<k>(u)) * ik;
        }
    });
    double y[N];
    static_for<0, N>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        double u[N > 1 ? N : 1];
#pragma unroll
        for (int j = 0; j < i; ++j) u[j] = L[i][j] * y[j];
        y[i] = b[i] - tsum<i>(u);
    });
#pragma unroll
    for (int i = 0; i < N; ++i) y[i] *= inv[i];
    static_for<0, N>([&](auto rc) {
        constexpr int i = N - 1 - decltype(rc)::value;
        double u[N > 1 ? N : 1];
#pragma unroll
        for (int j = i + 1; j < N; ++j) u[j - i - 1] = L[j][i] * x[j];
        x[i] = y[i] - tsum<N - 1 - i>(u);
    });
}

// Symmetric 3x3 inverse by cofactors: m = {m00 m01 m02 m11 m12 m22}, out the same layout.
// Dependent depth ~11 FP64 ops (2 cofactor, 3 determinant, 5 reciprocal, 1 scale).
__device__ __forceinline__ void sym3_inv(const double* m, double* out) {
    const double c00 = m[3] * m[5] - m[4] * m[4];
    const double c01 = m[2] * m[4] - m[1] * m[5];
    const double c02 = m[1] * m[4] - m[2] * m[3];
    const double c11 = m[0] * m[5] - m[2] * m[2];
    const double c12 = m[1] * m[2] - m[0] * m[4];
    const double c22 = m[0] * m[3] - m[1] * m[1];
    const double id = frcp(m[0] * c00 + (m[1] * c01 + m[2] * c02));
    out[0] = c00 * id;
    out[1] = c01 * id;
    out[2] = c02 * id;
    out[3] = c11 * id;
    out[4] = c12 * id;
    out[5] = c22 * id;
}

// x = H^-1 b for the damped SPD 6x6 pose system given as its upper triangle (hidx layout), by 3x3
// blocks: H = [A B; B^T C], W = A^-1 B, S = C - B^T W, x2 = S^-1 (b2 - B^T A^-1 b1), x1 = A^-1 b1 -
// W x2.  Same solution as an LDLT up to rounding, with a dependent chain of ~35 FP64 ops instead
// of ~100 (the one-thread-per-keyframe pose solve of k_landmark_solve sits on the LocalBA
// critical path).  A singular block gives a non-finite x, which the caller rejects.
__device__ __forceinline__ void spd6_block_solve(const double* U, const double* b, double* x) {
    const double A[6] = {U[0], U[1], U[2], U[6], U[7], U[11]};  // (00 01 02 11 12 22)
    const double B[3][3] = {{U[3], U[4], U[5]}, {U[8], U[9], U[10]}, {U[12], U[13], U[14]}};
    double Ai[6];
    sym3_inv(A, Ai);
    const double Ai3[3][3] = {{Ai[0], Ai[1], Ai[2]}, {Ai[1], Ai[3], Ai[4]}, {Ai[2], Ai[4], Ai[5]}};
    double W[3][3], y1[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
        for (int j = 0; j < 3; ++j) W[i][j] = Ai3[i][0] * B[0][j] + (Ai3[i][1] * B[1][j] + Ai3[i][2] * B[2][j]);
        y1[i] = Ai3[i][0] * b[0] + (Ai3[i][1] * b[1] + Ai3[i][2] * b[2]);
    }
    const int cu[6][2] = {{0, 0}, {0, 1}, {0, 2}, {1, 1}, {1, 2}, {2, 2}};
    const double Cu[6] = {U[15], U[16], U[17], U[18], U[19], U[20]};
    double S[6], Si[6];
#pragma unroll
    for (int e = 0; e < 6; ++e) {
        const int i = cu[e][0], j = cu[e][1];
        S[e] = Cu[e] - (B[0][i] * W[0][j] + (B[1][i] * W[1][j] + B[2][i] * W[2][j]));
    }
    sym3_inv(S, Si);
    double r2[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) r2[i] = b[3 + i] - (B[0][i] * y1[0] + (B[1][i] * y1[1] + B[2][i] * y1[2]));
    const double Si3[3][3] = {{Si[0], Si[1], Si[2]}, {Si[1], Si[3], Si[4]}, {Si[2], Si[4], Si[5]}};
#pragma unroll
    for (int i = 0; i < 3; ++i) x[3 + i] = Si3[i][0] * r2[0] + (Si3[i][1] * r2[1] + Si3[i][2] * r2[2]);
#pragma unroll
    for (int i = 0; i < 3; ++i) x[i] = y1[i] - (W[i][0] * x[3] + (W[i][1] * x[4] + W[i][2] * x[5]));
}

// upper-triangle index of the 6x6 pose Hessian
__device__ __forceinline__ int hidx(int i, int j) {  // i <= j
    return i * 6 - (i * (i - 1)) / 2 + (j - i);
}

// Sophus SE3::exp(dx) * T, written into T (8 doubles)
__device__ void se3_left_update(const double* dx, double* T) {
    const double eps = 1e-10;  // Sophus::Constants<double>::epsilon()
    const double wx = dx[3], wy = dx[4], wz = dx[5];
    const double theta_sq = wx * wx + wy * wy + wz * wz;
    double imag, real, c1 = 0.0, c2 = 0.0;
    const double t = theta_sq;
    const bool tiny = t < eps * eps;  // Sophus: theta < epsilon -> first-order V = R
    if (tiny) {
        const double t4 = t * t;
        imag = 0.5 - (1.0 / 48.0) * t + (1.0 / 3840.0) * t4;
        real = 1.0 - (1.0 / 8.0) * t + (1.0 / 384.0) * t4;
    } else {
        // theta < 0.1 (every Gauss-Newton step of a converging window): Taylor series in
        // theta^2 (truncation < 1e-22 relative) of sin(theta/2)/theta, cos(theta/2),
        // (1 - cos theta)/theta^2 and (theta - sin theta)/theta^3 — no sqrt / sincos / division
        imag = 0.5 + t * (-1.0 / 48 + t * (1.0 / 3840 + t * (-1.0 / 645120 + t * (1.0 / 185794560 + t * (-1.0 / 81749606400.0)))));
        real = 1.0 + t * (-1.0 / 8 + t * (1.0 / 384 + t * (-1.0 / 46080 + t * (1.0 / 10321920 + t * (-1.0 / 3715891200.0)))));
        c1 = 0.5 + t * (-1.0 / 24 + t * (1.0 / 720 + t * (-1.0 / 40320 + t * (1.0 / 3628800 + t * (-1.0 / 479001600.0)))));
        c2 = 1.0 / 6 + t * (-1.0 / 120 + t * (1.0 / 5040 + t * (-1.0 / 362880 + t * (1.0 / 39916800 + t * (-1.0 / 6227020800.0)))));
    }
    // theta >= 0.1: the exact forms.  The wave-uniform vote keeps this a real branch — as a plain
    // per-lane branch the compiler if-converted it, and every pose solve paid the double-precision
    // sincos (~150 FP64 instructions) whether or not a lane needed it.
    const bool big = !tiny && !(t < 1e-2);
    if (__ballot(big) != 0ull) {
        if (big) {
            const double theta = sqrt(t);
            double sh, ch;
            sincos(0.5 * theta, &sh, &ch);
            const double it = frcp(theta);
            imag = sh * it;
            real = ch;
            // 1 - cos theta = 2 sin^2(theta/2), sin theta = 2 sin(theta/2) cos(theta/2)
            const double rsq = it * it;
            c1 = (2.0 * sh * sh) * rsq;
            c2 = (theta - 2.0 * sh * ch) * (rsq * it);
        }
    }
    const double eq[4] = {imag * wx, imag * wy, imag * wz, real};
    const double O[9] = {0, -wz, wy, wz, 0, -wx, -wy, wx, 0};
    double V[9];
    if (tiny) {
        rot_from_quat(eq, V);
    } else {
        double O2[9];
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c)
                O2[3 * r + c] = O[3 * r] * O[c] + O[3 * r + 1] * O[3 + c] + O[3 * r + 2] * O[6 + c];
#pragma unroll
        for (int i = 0; i < 9; ++i) V[i] = ((i % 4 == 0) ? 1.0 : 0.0) + c1 * O[i] + c2 * O2[i];
    }
    const double et[3] = {V[0] * dx[0] + V[1] * dx[1] + V[2] * dx[2], V[3] * dx[0] + V[4] * dx[1] + V[5] * dx[2],
                          V[6] * dx[0] + V[7] * dx[1] + V[8] * dx[2]};
    // q <- normalize(eq * q)   (Sophus SO3 product + normalize)
    const double ax = eq[0], ay = eq[1], az = eq[2], aw = eq[3];
    const double bx = T[0], by = T[1], bz = T[2], bw = T[3];
    const double q[4] = {aw * bx + ax * bw + ay * bz - az * by, aw * by + ay * bw + az * bx - ax * bz,
                         aw * bz + az * bw + ax * by - ay * bx, aw * bw - ax * bx - ay * by - az * bz};
    const double rn = frsq((q[0] * q[0] + q[1] * q[1]) + (q[2] * q[2] + q[3] * q[3]));
    // t <- et + rotate(eq, t)
    const double rt[8] = {eq[0], eq[1], eq[2], eq[3], 0, 0, 0, 0};
    const D3 r = se3_apply(rt, {T[4], T[5], T[6]});
    T[0] = q[0] * rn; T[1] = q[1] * rn; T[2] = q[2] * rn; T[3] = q[3] * rn;
    T[4] = et[0] + r.x; T[5] = et[1] + r.y; T[6] = et[2] + r.z;
}

inline uint64_t splitmix64(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

// landmark id -> map index: open addressing over a power-of-two table (splitmix64 probe start,
// linear probing); ids are unique in a map.  Several times faster than std::unordered_map for the
// 10^5-landmark maps of C4 / C5, where the host plan builds spend most of their time here.
struct FlatIdMap {
    std::vector<uint64_t> key;
    std::vector<int> val;
    uint64_t mask = 0;
    void build(const uint64_t* ids, int n) {
        size_t cap = 16;
        while (cap < 2 * (size_t)std::max(n, 1)) cap <<= 1;
        key.assign(cap, 0);
        val.assign(cap, -1);
        mask = cap - 1;
        for (int i = 0; i < n; ++i) {
            uint64_t h = splitmix64(ids[i]) & mask;
            while (val[h] >= 0 && key[h] != ids[i]) h = (h + 1) & mask;
            key[h] = ids[i];
            val[h] = i;
        }
    }
    int get(uint64_t id) const {  // map index or -1
        if (val.empty()) return -1;
        uint64_t h = splitmix64(id) & mask;
        while (val[h] >= 0) {
            if (key[h] == id) return val[h];
            h = (h + 1) & mask;
        }
        return -1;
    }
};

// SelectKeyFrames (local_ba.cpp:42-62) and the optimised landmark set (:77-108) of a map snapshot:
// `win` = map keyframe indices of the window in ascending id order (the reference's std::map
// order), `opt_all` = map indices of the landmarks that pass !IsBad and the total observation
// count filter, ascending.  status 1 = the reference's early returns (:67-75, :106-108).
struct Window {
    int status = 1;
    std::vector<int> win;
    std::unordered_map<uint64_t, int> win_row;  // keyframe id -> window row
    FlatIdMap lm_by_id;                         // landmark id -> map index
    std::vector<int> opt_all;
};

inline void select_window(const vx_map_view* m, uint64_t ref_kf_id, int has_ref, int window_size,
                          int min_point_observations, Window& w) {
    w = Window{};
    if (!m || m->n_kf <= 0) return;
    std::vector<int> order(m->n_kf);
    for (int i = 0; i < m->n_kf; ++i) order[i] = i;
    std::sort(order.begin(), order.end(), [&](int x, int y) { return m->kf_id[x] < m->kf_id[y]; });
    const int window = std::max(1, window_size);
    const uint64_t max_id = has_ref ? ref_kf_id : m->kf_id[order.back()];
    for (int i = m->n_kf - 1; i >= 0 && (int)w.win.size() < window; --i) {
        if (m->kf_id[order[i]] > max_id) continue;
        w.win.push_back(order[i]);
    }
    std::reverse(w.win.begin(), w.win.end());
    if (w.win.size() < 2) return;
    for (int r = 0; r < (int)w.win.size(); ++r) w.win_row[m->kf_id[w.win[r]]] = r;
    w.lm_by_id.build(m->lm_id, m->n_lm);
    // landmarks referenced by a window feature (the reference's unordered_set of ids), then the
    // filter, in map-index order
    std::vector<uint8_t> ref((size_t)std::max(m->n_lm, 1), 0);
    for (int k : w.win)
        for (int64_t f = m->kf_feat_ptr[k]; f < m->kf_feat_ptr[k + 1]; ++f)
            if (m->feat_flags[f] & 1) {
                const int l = w.lm_by_id.get(m->feat_lm_id[f]);
                if (l >= 0) ref[l] = 1;
            }
    for (int l = 0; l < m->n_lm; ++l) {
        if (!ref[l] || m->lm_bad[l]) continue;
        if (m->lm_obs_ptr[l + 1] - m->lm_obs_ptr[l] < (int64_t)min_point_observations) continue;
        w.opt_all.push_back(l);
    }
    if (!w.opt_all.empty()) w.status = 0;
}

}  // namespace ba
}  // namespace vx
