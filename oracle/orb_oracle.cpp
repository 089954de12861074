// orb_oracle.cpp — CPU restatement of the ORB path.  TEST INFRASTRUCTURE ONLY (see oracle.h).
//
// Restates cv::ORB::detectAndCompute as called by ORBExtractor::Extract
// (/root/reference/core/feature/orb_extractor.cpp:13, created at :6 with (n, 1.2f, 8) and
// OpenCV defaults edgeThreshold 31, firstLevel 0, WTA_K 2, HARRIS_SCORE, patchSize 31,
// fastThreshold 20).  OpenCV itself is absent from this container: the spec followed here is
// SURVEY.md Appendix A (A.1 gray/pyramid, A.2 quotas, A.3 FAST+NMS+retainBest, A.4 Harris and
// IC angle, A.5 blur, A.6 rBRIEF).  Parity against real OpenCV is UNPINNED (no reference
// tests / golden vectors exist).  Build: -O2 -ffp-contract=off (no FMA).
#include "oracle.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

namespace {

// cvRound: round half to even (SSE2 cvtsd2si / lrint under the default rounding mode).
inline int cv_round(double v) { return (int)std::nearbyint(v); }
inline int cv_roundf(float v) { return (int)std::nearbyintf(v); }
inline int cv_floor(double v) { int i = (int)v; return i - (i > v); }
inline int cv_ceil(double v) { int i = (int)v; return i + (i < v); }

struct KeyPoint {  // field order of cv::KeyPoint
    float x, y, size, angle, response;
    int octave;
    int class_id;  // cv::KeyPoint::class_id (-1 from FAST); here: the level's raster index, carried
                   // along by nth_element / partition so the per-stage dumps can name the order
};

struct Img {
    int w = 0, h = 0;
    std::vector<uint8_t> px;
    const uint8_t* row(int y) const { return px.data() + (size_t)y * w; }
    uint8_t at(int y, int x) const { return px[(size_t)y * w + x]; }
};

// A.1 — cvtColor(BGR2GRAY), 8U fixed point: (B*1868 + G*9617 + R*4899 + (1<<13)) >> 14
void to_gray(const uint8_t* img, int w, int h, int ch, int64_t stride, Img& g) {
    g.w = w; g.h = h; g.px.resize((size_t)w * h);
    for (int y = 0; y < h; ++y) {
        const uint8_t* s = img + (size_t)y * stride;
        uint8_t* d = g.px.data() + (size_t)y * w;
        if (ch == 1) { std::memcpy(d, s, w); continue; }
        for (int x = 0; x < w; ++x, s += ch)
            d[x] = (uint8_t)((s[0] * 1868 + s[1] * 9617 + s[2] * 4899 + (1 << 13)) >> 14);
    }
}

// A.1 — linear interpolation coefficients of resize_bitExact (interpolationLinear::getCoeffs):
// scale = 1/(dst/src) in double; f = scale*(d+0.5)-0.5; i = floor(f); alpha = cvRound((f-i)*256).
void linear_coeffs(int src, int dst, std::vector<int>& ofs, std::vector<int>& c0, std::vector<int>& c1) {
    ofs.resize(dst); c0.resize(dst); c1.resize(dst);
    const double inv = (double)dst / (double)src;
    const double scale = 1.0 / inv;
    for (int d = 0; d < dst; ++d) {
        const double f = scale * ((double)d + 0.5) - 0.5;
        const int i = cv_floor(f);
        if (i >= 0 && src > 1) {
            if (i < src - 1) {
                const int a = cv_round((f - (double)i) * 256.0);
                ofs[d] = i; c1[d] = a; c0[d] = 256 - a;
            } else {  // right clamp: pixel src-1 alone
                ofs[d] = src - 1; c0[d] = 256; c1[d] = 0;
            }
        } else {      // left clamp: pixel 0 alone
            ofs[d] = 0; c0[d] = 256; c1[d] = 0;
        }
    }
}

// A.1 — resize(prev, size, INTER_LINEAR_EXACT): u16 8.8 horizontal, u32 16.16 vertical.
void resize_linear_exact(const Img& s, Img& d, int dw, int dh) {
    d.w = dw; d.h = dh; d.px.assign((size_t)dw * dh, 0);
    std::vector<int> xo, xc0, xc1, yo, yc0, yc1;
    linear_coeffs(s.w, dw, xo, xc0, xc1);
    linear_coeffs(s.h, dh, yo, yc0, yc1);
    std::vector<uint32_t> h0(dw), h1(dw);
    auto hline = [&](int sy, std::vector<uint32_t>& out) {
        const uint8_t* r = s.row(sy);
        for (int x = 0; x < dw; ++x) {
            const int o = xo[x];
            const int o1 = std::min(o + 1, s.w - 1);
            out[x] = (uint32_t)(r[o] * xc0[x] + r[o1] * xc1[x]);
        }
    };
    for (int y = 0; y < dh; ++y) {
        const int o = yo[y];
        hline(o, h0);
        hline(std::min(o + 1, s.h - 1), h1);
        uint8_t* dr = d.px.data() + (size_t)y * dw;
        for (int x = 0; x < dw; ++x) {
            const uint32_t v = h0[x] * (uint32_t)yc0[y] + h1[x] * (uint32_t)yc1[y];
            const uint32_t o8 = (v + 32768u) >> 16;
            dr[x] = (uint8_t)std::min<uint32_t>(o8, 255u);
        }
    }
}

struct Geometry {
    std::vector<float> scale;
    std::vector<int> w, h;
};

// ORB_Impl::detectAndCompute layer sizes: s_l = (float)pow((double)scaleFactor, l),
// size = (cvRound(W * (1/s_l)), cvRound(H * (1/s_l))).  scaleFactor is a double holding 1.2f.
Geometry level_geometry(int W, int H, float scale_factor, int n_levels) {
    Geometry g;
    g.scale.resize(n_levels); g.w.resize(n_levels); g.h.resize(n_levels);
    const double sf = (double)scale_factor;
    for (int l = 0; l < n_levels; ++l) {
        const float s = (float)std::pow(sf, (double)l);
        const float inv = 1.0f / s;
        g.scale[l] = s;
        g.w[l] = cv_roundf((float)W * inv);
        g.h[l] = cv_roundf((float)H * inv);
    }
    return g;
}

// A.2 — per-level feature quotas (computeKeyPoints).
std::vector<int> quotas(int n, float scale_factor, int nlevels) {
    std::vector<int> q(nlevels);
    const float factor = (float)(1.0 / (double)scale_factor);
    float nd = (float)n * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int l = 0; l < nlevels - 1; ++l) {
        q[l] = cv_roundf(nd);
        sum += q[l];
        nd *= factor;
    }
    q[nlevels - 1] = std::max(n - sum, 0);
    return q;
}

// A.3 — FAST ring (makeOffsets, patternSize 16), k = 16..24 repeat k = 0..8.
const int kRing[16][2] = {{0, 3},  {1, 3},  {2, 2},  {3, 1},   {3, 0},   {3, -1}, {2, -2}, {1, -3},
                          {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

// cornerScore<16>
int corner_score(const Img& im, int x, int y, int threshold) {
    const int v = im.at(y, x);
    int d[25];
    for (int k = 0; k < 25; ++k) {
        const int* o = kRing[k & 15];
        d[k] = v - im.at(y + o[1], x + o[0]);
    }
    int a0 = threshold;
    for (int k = 0; k < 16; k += 2) {
        int a = std::min(d[k + 1], d[k + 2]);
        a = std::min(a, d[k + 3]);
        if (a <= a0) continue;
        for (int j = 4; j <= 8; ++j) a = std::min(a, d[k + j]);
        a0 = std::max(a0, std::min(a, d[k]));
        a0 = std::max(a0, std::min(a, d[k + 9]));
    }
    int b0 = -a0;
    for (int k = 0; k < 16; k += 2) {
        int b = std::max(d[k + 1], d[k + 2]);
        b = std::max(b, d[k + 3]);
        b = std::max(b, d[k + 4]);
        b = std::max(b, d[k + 5]);
        if (b >= b0) continue;
        b = std::max(b, d[k + 6]);
        b = std::max(b, d[k + 7]);
        b = std::max(b, d[k + 8]);
        b0 = std::min(b0, std::max(b, d[k]));
        b0 = std::min(b0, std::max(b, d[k + 9]));
    }
    return -b0 - 1;
}

// FAST_t<16>: >=9 contiguous ring pixels all darker than v-t or all brighter than v+t.
bool is_corner(const Img& im, int x, int y, int t) {
    const int v = im.at(y, x);
    // FAST_t's exact pre-test: any 9-arc contains one pixel of every opposite pair (k, k+8).
    auto cls = [&](int k) {
        const int p = im.at(y + kRing[k][1], x + kRing[k][0]);
        return (p < v - t ? 1 : 0) | (p > v + t ? 2 : 0);
    };
    int d = cls(0) | cls(8);
    if (!d) return false;
    d &= cls(4) | cls(12);
    if (!d) return false;
    for (int sign = 0; sign < 2; ++sign) {
        int count = 0;
        for (int k = 0; k < 25; ++k) {
            const int* o = kRing[k & 15];
            const int p = im.at(y + o[1], x + o[0]);
            const bool hit = sign == 0 ? (p < v - t) : (p > v + t);
            if (hit) {
                if (++count > 8) return true;
            } else {
                count = 0;
            }
        }
    }
    return false;
}

// FAST with nonmax suppression: corners on rows [3, H-3), cols [3, W-3); strict 3x3 NMS where
// non-corners score 0; raster output KeyPoint(x, y, 7, -1, score).
std::vector<KeyPoint> fast_nms(const Img& im, int threshold) {
    std::vector<KeyPoint> out;
    const int W = im.w, H = im.h;
    if (W < 7 || H < 7) return out;
    std::vector<uint8_t> score((size_t)W * H, 0);
    for (int y = 3; y < H - 3; ++y)
        for (int x = 3; x < W - 3; ++x)
            if (is_corner(im, x, y, threshold))
                score[(size_t)y * W + x] = (uint8_t)corner_score(im, x, y, threshold);
    for (int y = 3; y < H - 3; ++y)
        for (int x = 3; x < W - 3; ++x) {
            const int s = score[(size_t)y * W + x];
            if (!s) continue;
            bool keep = true;
            for (int dy = -1; dy <= 1 && keep; ++dy)
                for (int dx = -1; dx <= 1; ++dx) {
                    if (!dx && !dy) continue;
                    if (!(s > score[(size_t)(y + dy) * W + x + dx])) { keep = false; break; }
                }
            if (keep) out.push_back(KeyPoint{(float)x, (float)y, 7.f, -1.f, (float)s, 0, -1});
        }
    return out;
}

// KeyPointsFilter::runByImageBorder(kps, size, 31): stable remove_if outside [b, W-b) x [b, H-b)
void run_by_image_border(std::vector<KeyPoint>& kps, int W, int H, int b) {
    if (H <= 2 * b || W <= 2 * b) { kps.clear(); return; }
    kps.erase(std::remove_if(kps.begin(), kps.end(),
                             [&](const KeyPoint& k) {
                                 return !(k.x >= (float)b && k.x < (float)(W - b) &&
                                          k.y >= (float)b && k.y < (float)(H - b));
                             }),
              kps.end());
}

// KeyPointsFilter::retainBest.  STL mode reproduces OpenCV's nth_element + partition permutation;
// RASTER mode keeps the identical set ({response >= k-th largest}) in input order.
void retain_best(std::vector<KeyPoint>& kps, int n, int order) {
    if (n < 0 || kps.size() <= (size_t)n) return;
    if (n == 0) { kps.clear(); return; }
    if (order == ORC_ORDER_STL) {
        std::nth_element(kps.begin(), kps.begin() + n - 1, kps.end(),
                         [](const KeyPoint& a, const KeyPoint& b) { return a.response > b.response; });
        const float thr = kps[n - 1].response;
        auto new_end = std::partition(kps.begin() + n, kps.end(),
                                      [thr](const KeyPoint& k) { return k.response >= thr; });
        kps.resize(new_end - kps.begin());
    } else {
        std::vector<float> r(kps.size());
        for (size_t i = 0; i < kps.size(); ++i) r[i] = kps[i].response;
        std::nth_element(r.begin(), r.begin() + n - 1, r.end(), std::greater<float>());
        const float thr = r[n - 1];
        std::vector<KeyPoint> kept;
        kept.reserve(n);
        for (const auto& k : kps)
            if (k.response >= thr) kept.push_back(k);
        kps.swap(kept);
    }
}

// A.4 — HarrisResponses(blockSize 7, k 0.04f) at the integer level coordinate.
float harris(const Img& im, int x0, int y0) {
    const int r = 3;
    int a = 0, b = 0, c = 0;
    for (int i = 0; i < 7; ++i)
        for (int j = 0; j < 7; ++j) {
            const int y = y0 - r + i, x = x0 - r + j;
            auto P = [&](int dy, int dx) { return (int)im.at(y + dy, x + dx); };
            const int Ix = (P(0, 1) - P(0, -1)) * 2 + (P(-1, 1) - P(-1, -1)) + (P(1, 1) - P(1, -1));
            const int Iy = (P(1, 0) - P(-1, 0)) * 2 + (P(1, -1) - P(-1, -1)) + (P(1, 1) - P(-1, 1));
            a += Ix * Ix;
            b += Iy * Iy;
            c += Ix * Iy;
        }
    const float scale = 1.f / ((1 << 2) * 7 * 255.f);
    const float s4 = scale * scale * scale * scale;
    const float k = 0.04f;
    return ((float)a * (float)b - (float)c * (float)c - k * ((float)a + (float)b) * ((float)a + (float)b)) * s4;
}

// umax table of computeKeyPoints (halfPatchSize 15).
std::vector<int> make_umax(int half) {
    std::vector<int> umax(half + 2);
    const int vmax = cv_floor(half * std::sqrt(2.f) / 2 + 1);
    const int vmin = cv_ceil(half * std::sqrt(2.f) / 2);
    for (int v = 0; v <= vmax; ++v) umax[v] = cv_round(std::sqrt((double)half * half - v * v));
    for (int v = half, v0 = 0; v >= vmin; --v) {
        while (umax[v0] == umax[v0 + 1]) ++v0;
        umax[v] = v0;
        ++v0;
    }
    return umax;
}

// fastAtan2 (core/src/mathfuncs_core): polynomial atan in degrees, [0, 360).
float fast_atan2(float y, float x) {
    static const float p1 = 0.9997878412794807f * (float)(180 / M_PI);
    static const float p3 = -0.3258083974640975f * (float)(180 / M_PI);
    static const float p5 = 0.1555786518463281f * (float)(180 / M_PI);
    static const float p7 = -0.04432655554792128f * (float)(180 / M_PI);
    const float ax = std::fabs(x), ay = std::fabs(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// A.4 — ICAngles (half_k 15).
float ic_angle(const Img& im, int cx, int cy, const std::vector<int>& umax) {
    const int half = 15;
    int m01 = 0, m10 = 0;
    for (int u = -half; u <= half; ++u) m10 += u * im.at(cy, cx + u);
    for (int v = 1; v <= half; ++v) {
        int vsum = 0;
        const int d = umax[v];
        for (int u = -d; u <= d; ++u) {
            const int vp = im.at(cy + v, cx + u), vm = im.at(cy - v, cx + u);
            vsum += vp - vm;
            m10 += u * (vp + vm);
        }
        m01 += v * vsum;
    }
    return fast_atan2((float)m01, (float)m10);
}

// A.5 — float Gaussian taps: (float) of getGaussianKernelBitExact(7, sigma 2).
void gauss_taps(float k[7]) {
    double v[3], sum = 0;
    for (int i = 0, x = -6; i < 3; ++i, x += 2) {
        v[i] = std::exp((double)(x * x) * (-0.125 / 4.0));
        sum += v[i];
    }
    sum = sum * 2 + 1;
    const double mul = 1.0 / sum;
    for (int i = 0; i < 3; ++i) k[i] = k[6 - i] = (float)(v[i] * mul);
    k[3] = (float)(1.0 * mul);
}

inline int reflect101(int p, int n) {
    if (n == 1) return 0;
    while (p < 0 || p >= n) {
        if (p < 0) p = -p;
        if (p >= n) p = 2 * n - 2 - p;
    }
    return p;
}

// GaussianBlur 7x7 sigma 2 on a non-isolated ROI: float separable filter, row pass 8U->32F
// (sequential sum k0*p0 + ... + k6*p6), column pass symmetric form k3*r0 + k2*(r-1+r+1) +
// k1*(r-2+r+2) + k0*(r-3+r+3) then saturate_cast<uchar> (round half even).
uint8_t blur_at(const Img& im, int x, int y, const float k[7]) {
    float rows[7];
    for (int dy = -3; dy <= 3; ++dy) {
        const int yy = reflect101(y + dy, im.h);
        float s = k[0] * (float)im.at(yy, reflect101(x - 3, im.w));
        for (int j = 1; j < 7; ++j) s += k[j] * (float)im.at(yy, reflect101(x - 3 + j, im.w));
        rows[dy + 3] = s;
    }
    float s = k[3] * rows[3] + 0.0f;
    s += k[4] * (rows[4] + rows[2]);
    s += k[5] * (rows[5] + rows[1]);
    s += k[6] * (rows[6] + rows[0]);
    int r = cv_roundf(s);
    return (uint8_t)std::min(255, std::max(0, r));
}

// Whole-level blur with exactly blur_at's arithmetic (same taps, same summation order), written
// as two separable passes so the CPU baseline is not dominated by recomputation.
void blur_image(const Img& im, Img& out, const float k[7]) {
    const int W = im.w, H = im.h;
    out.w = W; out.h = H; out.px.resize((size_t)W * H);
    std::vector<int> xi((size_t)W + 6);
    for (int x = -3; x < W + 3; ++x) xi[x + 3] = reflect101(x, W);
    std::vector<float> rows((size_t)W * H);
    for (int y = 0; y < H; ++y) {
        const uint8_t* r = im.row(y);
        float* o = rows.data() + (size_t)y * W;
        for (int x = 0; x < W; ++x) {
            const int* ix = xi.data() + x;
            float s = k[0] * (float)r[ix[0]];
            for (int j = 1; j < 7; ++j) s += k[j] * (float)r[ix[j]];
            o[x] = s;
        }
    }
    for (int y = 0; y < H; ++y) {
        const float* rr[7];
        for (int d = -3; d <= 3; ++d) rr[d + 3] = rows.data() + (size_t)reflect101(y + d, H) * W;
        uint8_t* o = out.px.data() + (size_t)y * W;
        for (int x = 0; x < W; ++x) {
            float s = k[3] * rr[3][x] + 0.0f;
            s += k[4] * (rr[4][x] + rr[2][x]);
            s += k[5] * (rr[5][x] + rr[1][x]);
            s += k[6] * (rr[6][x] + rr[0][x]);
            const int v = cv_roundf(s);
            o[x] = (uint8_t)std::min(255, std::max(0, v));
        }
    }
}

struct OrbParams {
    int n_features = 1000;
    float scale_factor = 1.2f;
    int n_levels = 8;
    int fast_threshold = 20;
    int edge_threshold = 31;
};

void build_pyramid(const uint8_t* img, int w, int h, int ch, int64_t stride, const Geometry& g,
                   std::vector<Img>& pyr) {
    const int L = (int)g.w.size();
    pyr.resize(L);
    to_gray(img, w, h, ch, stride, pyr[0]);
    for (int l = 1; l < L; ++l) resize_linear_exact(pyr[l - 1], pyr[l], g.w[l], g.h[l]);
}

// Per-level stage data of one extraction (SURVEY.md §8(c)(i) per-stage dumps).
struct LevelStages {
    std::vector<KeyPoint> fast;   // FAST + NMS, raster order, before runByImageBorder
    std::vector<KeyPoint> cand;   // after runByImageBorder (raster order)
    std::vector<float> harris;    // Harris response of every cand entry
    std::vector<int> keep1;       // retainBest(2q) output order, as indices into cand
    std::vector<int> fin;         // retainBest(q) output order, as indices into cand
};

// ORB_Impl::detectAndCompute's keypoint part (computeKeyPoints): FAST -> runByImageBorder ->
// retainBest(2 q_l) per level -> Harris -> retainBest(q_l) per level -> IC angle -> scaling.
// Fills st (when non-null) with every level's intermediate lists.
std::vector<KeyPoint> compute_keypoints(const std::vector<Img>& pyr, const Geometry& g, const OrbParams& P,
                                        int order, std::vector<LevelStages>* st) {
    const int n_levels = (int)pyr.size();
    const auto q = quotas(P.n_features, P.scale_factor, n_levels);
    if (st) st->assign(n_levels, LevelStages{});
    std::vector<KeyPoint> all;
    std::vector<int> counters(n_levels);
    for (int l = 0; l < n_levels; ++l) {
        auto kps = fast_nms(pyr[l], P.fast_threshold);
        if (st) (*st)[l].fast = kps;
        run_by_image_border(kps, pyr[l].w, pyr[l].h, P.edge_threshold);
        for (size_t i = 0; i < kps.size(); ++i) kps[i].class_id = (int)i;
        if (st) {
            (*st)[l].cand = kps;
            for (auto& k : kps) (*st)[l].harris.push_back(harris(pyr[l], cv_roundf(k.x), cv_roundf(k.y)));
        }
        retain_best(kps, 2 * q[l], order);
        counters[l] = (int)kps.size();
        for (auto& k : kps) { k.octave = l; k.size = 31 * g.scale[l]; }
        if (st) for (auto& k : kps) (*st)[l].keep1.push_back(k.class_id);
        all.insert(all.end(), kps.begin(), kps.end());
    }
    if (all.empty()) return all;
    for (auto& k : all) k.response = harris(pyr[k.octave], cv_roundf(k.x), cv_roundf(k.y));
    std::vector<KeyPoint> sel;
    size_t off = 0;
    for (int l = 0; l < n_levels; ++l) {
        std::vector<KeyPoint> kps(all.begin() + off, all.begin() + off + counters[l]);
        off += counters[l];
        retain_best(kps, q[l], order);
        if (st) for (auto& k : kps) (*st)[l].fin.push_back(k.class_id);
        sel.insert(sel.end(), kps.begin(), kps.end());
    }
    const auto umax = make_umax(15);
    for (auto& k : sel) k.angle = ic_angle(pyr[k.octave], cv_roundf(k.x), cv_roundf(k.y), umax);
    for (auto& k : sel) { const float s = g.scale[k.octave]; k.x *= s; k.y *= s; }
    return sel;
}

}  // namespace

extern "C" {

int orc_orb_quotas(int n_features, float scale_factor, int n_levels, int32_t* out) {
    auto q = quotas(n_features, scale_factor, n_levels);
    for (int l = 0; l < n_levels; ++l) out[l] = q[l];
    return 0;
}

int orc_orb_level_sizes(int w, int h, float scale_factor, int n_levels, int32_t* lw, int32_t* lh,
                        float* scales) {
    auto g = level_geometry(w, h, scale_factor, n_levels);
    for (int l = 0; l < n_levels; ++l) { lw[l] = g.w[l]; lh[l] = g.h[l]; scales[l] = g.scale[l]; }
    return 0;
}

int orc_orb_pyramid(const uint8_t* img, int w, int h, int channels, int64_t stride,
                    float scale_factor, int n_levels, uint8_t* out, int64_t cap) {
    auto g = level_geometry(w, h, scale_factor, n_levels);
    std::vector<Img> pyr;
    build_pyramid(img, w, h, channels, stride, g, pyr);
    int64_t off = 0;
    for (auto& p : pyr) {
        if (off + (int64_t)p.px.size() > cap) return -1;
        std::memcpy(out + off, p.px.data(), p.px.size());
        off += (int64_t)p.px.size();
    }
    return 0;
}

int orc_fast_nms(const uint8_t* img, int w, int h, int threshold, int32_t* xys, int cap, int* n_out) {
    Img im; im.w = w; im.h = h; im.px.assign(img, img + (size_t)w * h);
    auto k = fast_nms(im, threshold);
    *n_out = (int)k.size();
    if ((int)k.size() > cap) return -1;
    for (size_t i = 0; i < k.size(); ++i) {
        xys[3 * i] = (int)k[i].x; xys[3 * i + 1] = (int)k[i].y; xys[3 * i + 2] = (int)k[i].response;
    }
    return 0;
}

int orc_fast_scores(const uint8_t* img, int w, int h, int threshold, uint8_t* out) {
    Img im; im.w = w; im.h = h; im.px.assign(img, img + (size_t)w * h);
    std::memset(out, 0, (size_t)w * h);
    for (int y = 3; y < h - 3; ++y)
        for (int x = 3; x < w - 3; ++x)
            if (is_corner(im, x, y, threshold)) out[(size_t)y * w + x] = (uint8_t)corner_score(im, x, y, threshold);
    return 0;
}

float orc_harris(const uint8_t* img, int w, int h, int x, int y) {
    Img im; im.w = w; im.h = h; im.px.assign(img, img + (size_t)w * h);
    return harris(im, x, y);
}

float orc_ic_angle(const uint8_t* img, int w, int h, int x, int y) {
    Img im; im.w = w; im.h = h; im.px.assign(img, img + (size_t)w * h);
    return ic_angle(im, x, y, make_umax(15));
}

float orc_fast_atan2(float y, float x) { return fast_atan2(y, x); }

int orc_blur_level(const uint8_t* img, int w, int h, uint8_t* out) {
    Img im; im.w = w; im.h = h; im.px.assign(img, img + (size_t)w * h);
    float k[7];
    gauss_taps(k);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) out[(size_t)y * w + x] = blur_at(im, x, y, k);
    return 0;
}

int orc_orb_extract(const uint8_t* img, int w, int h, int channels, int64_t stride, int n_features,
                    float scale_factor, int n_levels, int fast_threshold, const int32_t* pattern,
                    int order, orc_keypoint* out_kp, uint8_t* out_desc, int cap, int* n_out) {
    *n_out = 0;
    if (!img || w <= 0 || h <= 0 || n_levels <= 0) return 0;
    OrbParams P;
    P.n_features = n_features; P.scale_factor = scale_factor; P.n_levels = n_levels;
    P.fast_threshold = fast_threshold;
    const Geometry g = level_geometry(w, h, scale_factor, n_levels);
    std::vector<Img> pyr;
    build_pyramid(img, w, h, channels, stride, g, pyr);
    const std::vector<KeyPoint> sel = compute_keypoints(pyr, g, P, order, nullptr);
    const int n = (int)sel.size();
    *n_out = n;
    if (n == 0) return 0;
    if (n > cap) return -1;

    // computeOrbDescriptors on the blurred levels (WTA_K 2, bit_pattern_31_).
    float gk[7];
    gauss_taps(gk);
    std::vector<Img> blurred(n_levels);
    for (int l = 0; l < n_levels; ++l) blur_image(pyr[l], blurred[l], gk);
    for (int i = 0; i < n; ++i) {
        const KeyPoint& k = sel[i];
        const Img& im = blurred[k.octave];
        const float scale = 1.f / g.scale[k.octave];
        float angle = k.angle;
        angle *= (float)(M_PI / 180.f);
        const float a = (float)std::cos((double)angle), b = (float)std::sin((double)angle);
        const int cy = cv_roundf(k.y * scale), cx = cv_roundf(k.x * scale);
        uint8_t* d = out_desc + (size_t)i * 32;
        auto value = [&](int idx) {
            const float px = (float)pattern[2 * idx], py = (float)pattern[2 * idx + 1];
            const float x = px * a - py * b;
            const float y = px * b + py * a;
            return (int)im.at(cy + cv_roundf(y), cx + cv_roundf(x));
        };
        for (int byte = 0; byte < 32; ++byte) {
            int val = 0;
            for (int bit = 0; bit < 8; ++bit) {
                const int base = 16 * byte + 2 * bit;
                val |= (value(base) < value(base + 1)) << bit;
            }
            d[byte] = (uint8_t)val;
        }
        out_kp[i].x = k.x; out_kp[i].y = k.y; out_kp[i].response = k.response;
        out_kp[i].angle = k.angle; out_kp[i].octave = k.octave;
    }
    return 0;
}

int orc_orb_stages(const uint8_t* img, int w, int h, int channels, int64_t stride, int n_features,
                   float scale_factor, int n_levels, int fast_threshold, int order, int32_t* counts,
                   int32_t* fast_xys, float* cand, int32_t* keep1, int32_t* fin, int64_t cap) {
    for (int i = 0; i < 4 * n_levels; ++i) counts[i] = 0;
    if (!img || w <= 0 || h <= 0 || n_levels <= 0) return 0;
    OrbParams P;
    P.n_features = n_features; P.scale_factor = scale_factor; P.n_levels = n_levels;
    P.fast_threshold = fast_threshold;
    const Geometry g = level_geometry(w, h, scale_factor, n_levels);
    std::vector<Img> pyr;
    build_pyramid(img, w, h, channels, stride, g, pyr);
    std::vector<LevelStages> st;
    compute_keypoints(pyr, g, P, order, &st);
    int64_t of = 0, oc = 0, o1 = 0, o2 = 0;
    for (int l = 0; l < n_levels; ++l) {
        const LevelStages& s = st[l];
        counts[4 * l] = (int)s.fast.size();
        counts[4 * l + 1] = (int)s.cand.size();
        counts[4 * l + 2] = (int)s.keep1.size();
        counts[4 * l + 3] = (int)s.fin.size();
        if (of + (int64_t)s.fast.size() > cap || oc + (int64_t)s.cand.size() > cap ||
            o1 + (int64_t)s.keep1.size() > cap || o2 + (int64_t)s.fin.size() > cap)
            return -1;
        for (const auto& k : s.fast) {
            fast_xys[3 * of] = (int)k.x; fast_xys[3 * of + 1] = (int)k.y; fast_xys[3 * of + 2] = (int)k.response;
            ++of;
        }
        for (size_t i = 0; i < s.cand.size(); ++i) {
            cand[4 * oc] = s.cand[i].x; cand[4 * oc + 1] = s.cand[i].y;
            cand[4 * oc + 2] = s.cand[i].response; cand[4 * oc + 3] = s.harris[i];
            ++oc;
        }
        for (int v : s.keep1) keep1[o1++] = v;
        for (int v : s.fin) fin[o2++] = v;
    }
    return 0;
}

int orc_retain_best_keys(const uint32_t* keys, int n, int npts, int32_t* out_idx, int* n_out) {
    struct E { uint32_t key; int32_t idx; };
    std::vector<E> a(n > 0 ? n : 0);
    for (int i = 0; i < n; ++i) a[i] = E{keys[i], i};
    int kept = n;
    if (npts >= 0 && n > npts) {
        if (npts == 0) {
            kept = 0;
        } else {
            auto gt = [](const E& x, const E& y) { return x.key > y.key; };
            std::nth_element(a.begin(), a.begin() + npts - 1, a.end(), gt);
            const uint32_t thr = a[npts - 1].key;
            kept = (int)(std::partition(a.begin() + npts, a.end(), [thr](const E& x) { return x.key >= thr; }) -
                         a.begin());
        }
    }
    for (int i = 0; i < kept; ++i) out_idx[i] = a[i].idx;
    *n_out = kept;
    return 0;
}

int orc_antiqsort(int n, int nth, uint32_t* out_keys) {
    if (n <= 0 || nth < 0 || nth >= n) return -1;
    std::vector<int> val(n, n - 1);  // every item starts as "gas" (= n - 1)
    const int gas = n - 1;
    int nsolid = 0, candidate = 0;
    std::vector<int> ptr(n);
    for (int i = 0; i < n; ++i) ptr[i] = i;
    auto greater = [&](int x, int y) {  // McIlroy's adversary, as the comparator of a descending select
        if (val[x] == gas && val[y] == gas) {
            if (x == candidate) val[x] = nsolid++;
            else val[y] = nsolid++;
        }
        if (val[x] == gas) candidate = x;
        else if (val[y] == gas) candidate = y;
        return val[x] > val[y];
    };
    std::nth_element(ptr.begin(), ptr.begin() + nth, ptr.end(), greater);
    for (int i = 0; i < n; ++i) out_keys[i] = (uint32_t)val[i];
    return 0;
}

}  // extern "C"
