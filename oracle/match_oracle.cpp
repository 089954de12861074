// match_oracle.cpp — CPU restatement of ORBMatcher::Match.  TEST INFRASTRUCTURE ONLY.
//
// Reference: core/feature/orb_matcher.cpp:11-43 — cv::BFMatcher(NORM_HAMMING) (:22),
// knnMatch(desc_last = query, desc_curr = train, knn, 2) (:25), keep knn[0] when
// knn.size() == 2 && m1.distance < nn_ratio * m2.distance (:27-36), nn_ratio = 0.8f
// (orb_matcher.h:13).  The k-NN arithmetic is OpenCV's batchDistance top-K insertion
// (SURVEY.md Appendix A.7): insert j when d < dist[K-1], shifting while dist[k] > d, so ties keep
// the lower train index first.  Unpinned vs OpenCV (no reference fixtures).
#include "oracle.h"

#include <climits>
#include <cstring>

namespace {
inline int hamming32(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    for (int i = 0; i < 32; i += 8) {
        uint64_t x, y;
        std::memcpy(&x, a + i, 8);
        std::memcpy(&y, b + i, 8);
        d += __builtin_popcountll(x ^ y);
    }
    return d;
}
}  // namespace

extern "C" {

int orc_knn2(const uint8_t* q, int nq, const uint8_t* t, int nt, int32_t* idx2, int32_t* dist2) {
    for (int i = 0; i < nq; ++i) {
        int dist[2] = {INT_MAX, INT_MAX}, nidx[2] = {-1, -1};
        const uint8_t* qi = q + (size_t)i * 32;
        for (int j = 0; j < nt; ++j) {
            const int d = hamming32(qi, t + (size_t)j * 32);
            if (d < dist[1]) {
                int k = 0;
                for (k = 0; k >= 0 && dist[k] > d; --k) {
                    nidx[k + 1] = nidx[k];
                    dist[k + 1] = dist[k];
                }
                nidx[k + 1] = j;
                dist[k + 1] = d;
            }
        }
        idx2[2 * i] = nidx[0]; idx2[2 * i + 1] = nidx[1];
        dist2[2 * i] = nidx[0] < 0 ? -1 : dist[0];
        dist2[2 * i + 1] = nidx[1] < 0 ? -1 : dist[1];
    }
    return 0;
}

int orc_match_knn2_ratio(const uint8_t* q, int nq, const uint8_t* t, int nt, float ratio,
                         orc_match* out, int cap, int* n_out) {
    *n_out = 0;
    if (nq <= 0 || nt <= 0) return 0;  // desc1.empty() || desc2.empty() (orb_matcher.cpp:18-20)
    int32_t idx2[2], dist2[2];
    int n = 0;
    for (int i = 0; i < nq; ++i) {
        orc_knn2(q + (size_t)i * 32, 1, t, nt, idx2, dist2);
        if (idx2[1] < 0) continue;  // knn.size() < 2
        const float d1 = (float)dist2[0], d2 = (float)dist2[1];
        if (d1 < ratio * d2) {
            if (n >= cap) return -1;
            out[n].query_idx = i;
            out[n].train_idx = idx2[0];
            out[n].distance = d1;
            ++n;
        }
    }
    *n_out = n;
    return 0;
}

}  // extern "C"
