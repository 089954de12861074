// ba_lean.hip — LocalBA::Optimize from the device-resident map in one call, with no host
// synchronisation between the window selection and the end (vx_ba_optimize_dmap).
//
// The reference rebuilds its problem on every keyframe (local_ba.cpp:66-108: SelectKeyFrames, the
// landmark set from the window's features, then per landmark its observations — mutex-guarded
// GetLandmark / GetFrame, map.cpp:31-47, and unordered_map walks, landmark.h:42-49) and then
// iterates (:110-248).  The plan build of ba_window.hip does the same on the device but reads three
// counts back to size its outputs, packs the landmark-stage workgroups on the host and rebuilds the
// map's landmark-major observation CSR with a radix sort whenever observations were added (every
// keyframe).  Here every size is a capacity the host already knows (window features, map rows,
// observation rows), every count stays in a small device header (dyn[], ba_plan.hpp), and the
// landmark-stage lists are built from the window side, so no sort is needed:
//
//   k_lb_clear    per map landmark row: referenced / pose-referenced flags and the live observation
//                 count cleared; the header zeroed
//   k_lb_feat     per window feature (binary search of its keyframe row): its resident row, the
//                 landmark row from the device id table (Map::GetLandmark), the pose-stage validity
//                 (local_ba.cpp:126-138), the referenced marks (:83-92); rows < nk gather the window
//                 keyframes' poses / intrinsics
//   k_lb_obs      per observation row (Landmark::observations_): the landmark's live observation
//                 count (ObservationCount, :99-101) and, when the pair's keyframe is in the window and
//                 the feature it names is a non-outlier observation of this very landmark (:186-204),
//                 a back-link on that window feature
//   k_lb_flags    per landmark row: optimised = referenced && !bad && count >= min (:93-104), fixed =
//                 seen by the pose stage but not optimised -> one 64-bit key (1 | fixed << 32)
//   (scan)        slots: optimised rows first (map-row order), then fixed rows (map-row order)
//   k_lb_slots    slot tables, initial positions, the counts into the header
//   (scan)        pose-stage CSR positions
//   k_lb_pose     the pose-stage CSR (feature order inside a keyframe, local_ba.cpp:131), keyframe
//                 pointers; each back-linked feature of an optimised landmark sets its window row's
//                 bit in the landmark's keyframe bit set
//   k_lb_lcount   per slot: landmark-stage observations = popcount of its bit set
//   (scan)        landmark-stage CSR pointers
//   k_lb_lfill    the landmark-stage CSR (a landmark's observations in window order: rank = the bits
//                 below its row) and the k_landmark_solve workgroup table: slot s goes to workgroup
//                 (lobs_ptr[s] + s) / Q with Q = 512 - nk, so a workgroup holds < Q landmarks and
//                 < Q + nk <= 512 observations — no sequential packing
//   iterations    ba.hip k_pose_kf + k_landmark_solve over capacity grids (ba_run_dyn)
//   k_lb_apply    the window poses and optimised positions into the resident rows
// A landmark's observations are summed in window (keyframe id) order instead of insertion order;
// the reference's own order is unordered_map iteration order, so parity is the usual 1e-4 with
// identical iteration and observation counts (tests/test_gpu_dmap.py).
#include <algorithm>
#include <climits>
#include <cstring>
#include <vector>

#include <rocprim/rocprim.hpp>

#include "vx_sort.hpp"
#include "vx_copy.hpp"

#include "vx_internal.hpp"
#include "ba_common.hpp"
#include "ba_plan.hpp"
#include "dmap.hpp"
#include "sba_plan.hpp"

namespace vx {
namespace {

constexpr int kT = 256;
constexpr uint64_t kEmptyKey = ~0ull;
inline unsigned grid(long long n) { return (unsigned)std::max(1ll, (n + kT - 1) / kT); }

__device__ __forceinline__ uint64_t mix(uint64_t x) {  // splitmix64
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

// ---------------------------------------------------------------- landmark id table (resident)
__global__ void k_ht_clear(uint64_t* key, unsigned cap) {
    const unsigned i = blockIdx.x * kT + threadIdx.x;
    if (i < cap) key[i] = kEmptyKey;
}
// rows [r0, r1); a removed row is skipped (a later row may hold its id again)
__global__ void k_ht_add(uint64_t* key, int* val, unsigned mask, const uint64_t* lid, const uint8_t* bad, int64_t r0,
                         int64_t r1) {
    const int64_t r = r0 + (int64_t)blockIdx.x * kT + threadIdx.x;
    if (r >= r1 || bad[r] == kLmRemoved) return;
    const uint64_t k = lid[r];
    unsigned h = (unsigned)mix(k) & mask;
    for (;;) {
        const unsigned long long prev = atomicCAS(reinterpret_cast<unsigned long long*>(&key[h]),
                                                  (unsigned long long)kEmptyKey, (unsigned long long)k);
        if (prev == kEmptyKey || prev == k) {
            val[h] = (int)r;
            return;
        }
        h = (h + 1) & mask;
    }
}
__device__ __forceinline__ int ht_get(const uint64_t* key, const int* val, unsigned mask, uint64_t k) {
    unsigned h = (unsigned)mix(k) & mask;
    for (unsigned probe = 0; probe <= mask; ++probe) {
        const uint64_t x = key[h];
        if (x == k) return val[h];
        if (x == kEmptyKey) return -1;
        h = (h + 1) & mask;
    }
    return -1;
}

// ---------------------------------------------------------------- build kernels
struct LeanArgs {
    // window (host tables, one upload): rows in ascending keyframe id order
    int nk, nf, mw;                 // keyframes, features, 64-bit words of a keyframe bit set
    const int64_t* src;             // nk: first resident feature row of window row r
    const uint64_t* wid;            // nk: keyframe ids (ascending)
    const int* wptr;                // nk + 1: window feature offsets
    const int* win;                 // nk: resident keyframe rows
    const uint8_t* cam;             // nk
    // resident map
    int64_t nl, nobs;
    const double* feat_uv;
    const uint64_t* feat_lm;
    const uint8_t* feat_fl;
    const uint64_t* lm_id;
    const uint8_t* lm_bad;
    const double* lm_pos;
    const int* obs_lm;
    const uint64_t* obs_kf;
    const uint64_t* obs_fi;
    const double* map_pose;
    const double* map_intr;
    const uint64_t* ht_key;
    const int* ht_val;
    unsigned ht_mask;
    int min_point;
    // per window feature
    int* f_l;                       // landmark row or -1
    int* f_code;                    // window row << 2 | pose-stage valid | landmark-stage candidate << 1
    int* f_pv;                      // pose-stage valid (scan input, nf + 1)
    int* f_back;                    // a live observation of its landmark names it (landmark stage)
    double2* wuv;
    // per landmark row
    int* l_ref;
    int* l_pv;
    int* l_cnt;
    unsigned long long* key;        // nl + 1
    const unsigned long long* ex;   // its exclusive scan
    int* l_slot;
    int* inv;                       // slot -> landmark row
    int* cnt;                       // slot -> landmark-stage observations (scan input, nl + 1)
    unsigned long long* mask;       // slot x mw keyframe bit sets
    const int* pscan;
    const int* lobs_ptr;
    // plan outputs
    double* lm_pos0;
    double2* puv;
    int* plm;
    int* pkf;                       // (SBA plans) window row of each pose-stage observation, or null
    int* kf_obs_ptr;
    int* lkf;
    int* llm;
    double2* luv;
    int* lm_blk;
    double* kf_pose0;
    double* kf_intr;
    int* kf_flags;
    int* dyn;
    int q;                          // landmark-stage workgroup key span (512 - nk)
};

__global__ __launch_bounds__(kT) void k_lb_clear(LeanArgs a) {
    const int64_t l = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (l < a.nl) {
        a.l_ref[l] = 0;
        a.l_pv[l] = 0;
        a.l_cnt[l] = 0;
    }
    if (l < kDynInts) a.dyn[l] = 0;
}

__device__ __forceinline__ int window_row(const int* wptr, int nk, int f) {
    int lo = 0, hi = nk - 1;  // last row with wptr[row] <= f
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (wptr[mid] <= f) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

__global__ __launch_bounds__(kT) void k_lb_feat(LeanArgs a) {
    const int f = blockIdx.x * kT + threadIdx.x;
    if (f < a.nk) {  // the window keyframes' initial poses, intrinsics and camera flags
        const int k = a.win[f];
        for (int j = 0; j < 7; ++j) a.kf_pose0[8 * f + j] = a.map_pose[7 * (int64_t)k + j];
        a.kf_pose0[8 * f + 7] = 0.0;
        for (int j = 0; j < 4; ++j) a.kf_intr[4 * f + j] = a.map_intr[4 * (int64_t)k + j];
        a.kf_flags[f] = a.cam[f];
    }
    if (f == a.nf) a.f_pv[f] = 0;  // (the scan's extra element)
    if (f >= a.nf) return;
    const int r = window_row(a.wptr, a.nk, f);
    const int64_t g = a.src[r] + (f - a.wptr[r]);
    const uint8_t fl = a.feat_fl[g];
    a.wuv[f] = make_double2(a.feat_uv[2 * g], a.feat_uv[2 * g + 1]);
    int l = -1;
    if (fl & 1) {
        l = ht_get(a.ht_key, a.ht_val, a.ht_mask, a.feat_lm[g]);
        if (l >= 0 && a.lm_bad[l] == kLmRemoved) l = -1;  // Map::GetLandmark -> nullptr
        if (l >= 0) a.l_ref[l] = 1;                       // local_ba.cpp:83-92
    }
    const bool good = (fl & 1) && !(fl & 2) && a.cam[r];
    const bool pv = good && l >= 0 && !a.lm_bad[l];     // local_ba.cpp:126-138
    if (pv) a.l_pv[l] = 1;
    a.f_l[f] = l;
    a.f_code[f] = (r << 2) | (good && l >= 0 ? 2 : 0) | (pv ? 1 : 0);
    a.f_pv[f] = pv ? 1 : 0;
    a.f_back[f] = 0;
}

__global__ __launch_bounds__(kT) void k_lb_obs(LeanArgs a) {
    const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (i >= a.nobs) return;
    const int l = a.obs_lm[i];
    if (l == kDeadObs || a.lm_bad[l] == kLmRemoved) return;
    atomicAdd(&a.l_cnt[l], 1);  // ObservationCount (live pairs)
    const uint64_t kid = a.obs_kf[i];
    int lo = 0, hi = a.nk - 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (a.wid[mid] < kid) lo = mid + 1;
        else hi = mid;
    }
    if (a.wid[lo] != kid) return;  // local_kf_ids.find (local_ba.cpp:187)
    const uint64_t fi = a.obs_fi[i];
    if (fi >= (uint64_t)(a.wptr[lo + 1] - a.wptr[lo])) return;  // :196
    const int f = a.wptr[lo] + (int)fi;
    // camera, has_landmark, !is_outlier (code bit 1) and feature.landmark_id_ == this landmark
    // (:193-201); the pair is unique per (landmark, keyframe), and a feature names one landmark, so
    // at most one row writes a feature
    if ((a.f_code[f] & 2) && a.f_l[f] == l) a.f_back[f] = 1;
}

__global__ __launch_bounds__(kT) void k_lb_flags(LeanArgs a) {
    const int64_t l = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (l == a.nl) a.key[l] = 0;
    if (l >= a.nl) return;
    const bool opt = a.l_ref[l] && !a.lm_bad[l] && a.l_cnt[l] >= a.min_point;
    if (opt) atomicAdd(&a.dyn[kDynGlobal], 1);
    const bool fixed = !opt && a.l_pv[l];
    a.key[l] = (opt ? 1ull : 0ull) | (fixed ? 1ull << 32 : 0ull);
}

__global__ __launch_bounds__(kT) void k_lb_slots(LeanArgs a) {
    const int64_t l = (int64_t)blockIdx.x * kT + threadIdx.x;
    const unsigned long long tot = a.ex[a.nl];
    const int n_opt = (int)(unsigned)tot, n_fixed = (int)(tot >> 32);
    if (l == 0) {
        a.dyn[kDynNOpt] = n_opt;
        a.dyn[kDynNLm] = n_opt + n_fixed;
        a.dyn[kDynNFixed] = n_fixed;
        a.dyn[kDynStatus] = n_opt == 0 ? 1 : 0;  // no optimisable landmark (local_ba.cpp:106-108)
    }
    if (l >= a.nl) return;
    const unsigned long long k = a.key[l], e = a.ex[l];
    int s = -1;
    if (k & 1ull) s = (int)(unsigned)e;
    else if (k >> 32) s = n_opt + (int)(e >> 32);
    a.l_slot[l] = s;
    if (s < 0) return;
    a.inv[s] = (int)l;
    a.lm_pos0[4 * (int64_t)s] = a.lm_pos[3 * l];
    a.lm_pos0[4 * (int64_t)s + 1] = a.lm_pos[3 * l + 1];
    a.lm_pos0[4 * (int64_t)s + 2] = a.lm_pos[3 * l + 2];
    a.lm_pos0[4 * (int64_t)s + 3] = 0.0;
    if (s < n_opt)
        for (int w = 0; w < a.mw; ++w) a.mask[(int64_t)s * a.mw + w] = 0ull;
}

__global__ __launch_bounds__(kT) void k_lb_pose(LeanArgs a) {
    const int f = blockIdx.x * kT + threadIdx.x;
    if (f <= a.nk) a.kf_obs_ptr[f] = a.pscan[a.wptr[f]];  // (wptr[nk] == nf: the total)
    if (f == 0) a.dyn[kDynPoseObs] = a.pscan[a.nf];
    if (f >= a.nf) return;
    const int code = a.f_code[f];
    const int l = a.f_l[f];
    if (code & 1) {
        const int o = a.pscan[f];
        a.puv[o] = a.wuv[f];
        a.plm[o] = a.l_slot[l];
        if (a.pkf) a.pkf[o] = code >> 2;
    }
    if (a.f_back[f]) {
        const int s = a.l_slot[l];
        if (s >= 0 && s < a.dyn[kDynNOpt]) {
            const int r = code >> 2;
            atomicOr(&a.mask[(int64_t)s * a.mw + (r >> 6)], 1ull << (r & 63));
        }
    }
}

__global__ __launch_bounds__(kT) void k_lb_lcount(LeanArgs a) {
    const int64_t s = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (s > a.nl) return;
    int c = 0;
    if (s < a.dyn[kDynNOpt])
        for (int w = 0; w < a.mw; ++w) c += __popcll(a.mask[s * a.mw + w]);
    a.cnt[s] = c;  // (slots past n_opt and the scan's extra element: 0)
    if (c) atomicMax(&a.dyn[kDynMaxObs], c);
}

__global__ __launch_bounds__(kT) void k_lb_lfill(LeanArgs a) {
    const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
    const int n_opt = a.dyn[kDynNOpt];
    if (i < a.nf && a.f_back[i]) {
        const int s = a.l_slot[a.f_l[i]];
        if (s >= 0 && s < n_opt) {
            const int r = a.f_code[i] >> 2;
            const unsigned long long* m = a.mask + (int64_t)s * a.mw;
            int rank = __popcll(m[r >> 6] & ((1ull << (r & 63)) - 1ull));
            for (int w = 0; w < (r >> 6); ++w) rank += __popcll(m[w]);
            const int at = a.lobs_ptr[s] + rank;
            a.lkf[at] = r;
            a.llm[at] = s;
            a.luv[at] = a.wuv[i];
        }
    }
    if (i < n_opt) {  // landmark-stage workgroups: slot s -> (lobs_ptr[s] + s) / q
        // q = 512 - (most landmark-stage observations of one landmark, <= nk <= 255): consecutive
        // keys differ by <= q, so no workgroup is empty, and a workgroup holds < q landmarks and
        // <= q - 1 + that many <= 511 observations (a.q = 512 - nk sizes the host's capacity grid)
        const int q = kBaLmBlock - a.dyn[kDynMaxObs];
        const int s = (int)i;
        const int b = (a.lobs_ptr[s] + s) / q;
        const int bp = s ? (a.lobs_ptr[s - 1] + s - 1) / q : -1;
        if (b != bp) {
            a.lm_blk[2 * b] = s;
            a.lm_blk[2 * b + 1] = a.lobs_ptr[s];
        }
        if (s == n_opt - 1) {
            a.lm_blk[2 * (b + 1)] = n_opt;
            a.lm_blk[2 * (b + 1) + 1] = a.lobs_ptr[n_opt];
            a.dyn[kDynBlocks] = b + 1;
            a.dyn[kDynLmObs] = a.lobs_ptr[n_opt];
        }
    }
}

// the finished run into the resident rows (the last iteration's ping-pong pose buffer)
// pack (optional): the call's read-back in one block — dyn and the iteration state (hdr_words ints),
// then (res_off >= 0) at res_off both pose parities, the positions and the landmark rows by capacity
// nl — so that one copy brings it back instead of five (each a ~3.5 µs blit launch on the call's path)
__global__ __launch_bounds__(kT) void k_lb_apply(const int* dyn, const int* iters, int nk, const int* win,
                                                 const double* kf_pose, const int* inv, int64_t nl,
                                                 const double* lm_pos, double* map_pose, double* map_pos,
                                                 uint8_t* pack, const int* state, int hdr_words, int64_t res_off) {
    const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (pack) {
        int* ph = reinterpret_cast<int*>(pack);
        if (i < kDynInts) ph[i] = dyn[i];
        else if (i < hdr_words) ph[i] = state[i - kDynInts];
        double* pr = reinterpret_cast<double*>(pack + (res_off >= 0 ? res_off : 0));
        for (int64_t k = i; res_off >= 0 && k < 16 * (int64_t)nk; k += (int64_t)gridDim.x * kT) pr[k] = kf_pose[k];
        if (res_off >= 0 && i < nl) {
            const double4 v = reinterpret_cast<const double4*>(lm_pos)[i];
            reinterpret_cast<double4*>(pr + 16 * (int64_t)nk)[i] = v;
            reinterpret_cast<int*>(pr + 16 * (int64_t)nk + 4 * nl)[i] = inv[i];
        }
    }
    if (dyn[kDynStatus]) return;
    if (i < nk) {
        const double* src = kf_pose + (size_t)(*iters & 1) * nk * 8 + 8 * i;
        for (int j = 0; j < 7; ++j) map_pose[7 * (int64_t)win[i] + j] = src[j];
    }
    if (i < nl && i < dyn[kDynNOpt])
        for (int j = 0; j < 3; ++j) map_pos[3 * (int64_t)inv[i] + j] = lm_pos[4 * i + j];
}

// grow-only with headroom (the map grows every keyframe: no hipFree / hipMalloc per call)
hipError_t grow(DevBuf& d, size_t want) {
    if (want <= d.bytes) return hipSuccess;
    size_t cap = 4096;
    while (cap < want) cap += cap / 2;
    return d.ensure(cap);
}

template <class T>
int scan_ex(vx_ctx* c, DevBuf& tmp, const T* in, T* out, int64_t n) {  // n + 1 outputs
    size_t bytes = 0;
    VX_HIP(c, rocprim::exclusive_scan(nullptr, bytes, in, out, T(0), (size_t)n + 1, rocprim::plus<T>(), c->stream));
    VX_HIP(c, grow(tmp, std::max<size_t>(bytes, 16)));
    VX_HIP(c, rocprim::exclusive_scan(tmp.p, bytes, in, out, T(0), (size_t)n + 1, rocprim::plus<T>(), c->stream));
    return VX_OK;
}

// the resident id table covers rows [0, n_lm): new rows added, rebuilt when it has to grow
int ht_sync(vx_ctx* c, vx_dmap* m) {
    const int64_t nl = m->n_lm;
    unsigned need = 1024;
    while ((int64_t)need < 2 * std::max<int64_t>(nl, 1)) need <<= 1;
    int64_t r0 = m->ht_rows;
    if (need > m->ht_cap) {
        unsigned cap = need;
        if (cap < 4 * (unsigned)std::max<int64_t>(nl, 1) && cap < (1u << 30)) cap <<= 1;  // room for growth
        VX_HIP(c, m->ht_key.ensure((size_t)cap * 8));
        VX_HIP(c, m->ht_val.ensure((size_t)cap * 4));
        m->ht_cap = cap;
        hipLaunchKernelGGL(k_ht_clear, dim3(grid(cap)), dim3(kT), 0, c->stream, m->ht_key.as<uint64_t>(), cap);
        r0 = 0;
    }
    if (nl > r0)
        hipLaunchKernelGGL(k_ht_add, dim3(grid(nl - r0)), dim3(kT), 0, c->stream, m->ht_key.as<uint64_t>(),
                           m->ht_val.as<int>(), m->ht_cap - 1, (const uint64_t*)m->lm_id.as<uint64_t>(),
                           (const uint8_t*)m->lm_bad.as<uint8_t>(), r0, nl);
    VX_LAUNCH_CHECK(c, "landmark id table");
    m->ht_rows = nl;
    return VX_OK;
}

}  // namespace

// What a lean build needs to know about the window before launching anything (host mirrors only)
struct LeanCore {
    std::vector<int> win, wptr;
    std::vector<int64_t> src;
    std::vector<uint64_t> wid;
    std::vector<uint8_t> cam;
    int nk = 0, nf = 0, mw = 1;
    int64_t nl = 0, nobs = 0, nvalid = 0, mx = 0;
    LeanArgs a{};
};

void lean_window(const vx_dmap* m, const std::vector<int>& win, LeanCore& K) {
    const int nk = (int)win.size();
    K.win = win;
    K.nk = nk;
    K.wptr.assign(nk + 1, 0);
    K.src.resize(nk);
    K.wid.resize(nk);
    K.cam.resize(nk);
    K.nvalid = K.mx = 0;
    for (int r = 0; r < nk; ++r) {
        const int k = win[r];
        K.src[r] = m->kf_feat_ptr[k];
        K.wptr[r + 1] = K.wptr[r] + (int)(m->kf_feat_ptr[k + 1] - m->kf_feat_ptr[k]);
        K.wid[r] = m->kf_id[k];
        K.cam[r] = m->kf_has_cam[k];
        K.nvalid += m->kf_valid_cnt[k];
        if (K.cam[r]) K.mx = std::max<int64_t>(K.mx, m->kf_valid_cnt[k]);
    }
    K.nf = K.wptr[nk];
    K.nl = m->n_lm;
    K.nobs = m->n_obs;
}

// The window tables (one pinned upload) and the build kernels up to the pose-stage CSR: slots
// (optimised rows first, then fixed rows, map-row order), initial positions by slot, keyframe tables,
// the pose-stage CSR; lstage: also the landmark-stage CSR and workgroup table (key span q).  Every
// count stays in dyn[]; nothing synchronises.
int lean_build_core(vx_ctx* c, vx_dmap* m, int min_point, int q, bool lstage, int cap_blocks, bool with_pkf,
                    LeanCore& K) {
    auto& L = m->lean;
    const int nk = K.nk, nf = K.nf;
    const std::vector<int>& win = K.win;
    const std::vector<int>& wptr = K.wptr;
    const int64_t nl = K.nl, nobs = K.nobs;
    const int mw = (nk + 63) / 64;
    K.mw = mw;
    VX_HIP(c, hipSetDevice(c->device));
    int rc;
    if ((rc = ht_sync(c, m))) return rc;
    // window tables: one pinned block, one upload
    const size_t o_src = 0, o_wid = o_src + 8 * (size_t)nk, o_wptr = o_wid + 8 * (size_t)nk,
                 o_win = o_wptr + 4 * ((size_t)nk + 2), o_cam = o_win + 4 * ((size_t)nk + 2), o_end = o_cam + (size_t)nk + 8;
    VX_HIP(c, L.win_host.ensure(o_end, true));
    VX_HIP(c, grow(L.win, o_end));
    {
        uint8_t* H = static_cast<uint8_t*>(L.win_host.p);
        std::memcpy(H + o_src, K.src.data(), 8 * (size_t)nk);
        std::memcpy(H + o_wid, K.wid.data(), 8 * (size_t)nk);
        std::memcpy(H + o_wptr, wptr.data(), 4 * ((size_t)nk + 1));
        std::memcpy(H + o_win, win.data(), 4 * (size_t)nk);
        std::memcpy(H + o_cam, K.cam.data(), (size_t)nk);
    }
    VX_HIP(c, hipMemcpyAsync(L.win.p, L.win_host.p, o_end, hipMemcpyHostToDevice, c->stream));
    const size_t fN = (size_t)nf + 1, lN = (size_t)nl + 1, kN = (size_t)nk + 1;
    for (DevBuf* d : {&L.f_l, &L.f_code, &L.f_pv, &L.f_back, &L.pscan, &L.plm, &L.lkf, &L.llm}) VX_HIP(c, grow(*d, fN * 4));
    for (DevBuf* d : {&L.wuv, &L.puv, &L.luv}) VX_HIP(c, grow(*d, fN * 16));
    for (DevBuf* d : {&L.l_ref, &L.l_pv, &L.l_cnt, &L.l_slot, &L.inv, &L.cnt, &L.lobs_ptr}) VX_HIP(c, grow(*d, lN * 4));
    for (DevBuf* d : {&L.key, &L.ex}) VX_HIP(c, grow(*d, lN * 8));
    VX_HIP(c, grow(L.mask, lN * mw * 8));
    VX_HIP(c, grow(L.lm_pos0, lN * 32));
    VX_HIP(c, grow(L.lm_blk, (size_t)(cap_blocks + 2) * 8));
    VX_HIP(c, grow(L.kf_pose0, kN * 64));
    VX_HIP(c, grow(L.kf_intr, kN * 32));
    VX_HIP(c, grow(L.kf_flags, kN * 4));
    VX_HIP(c, grow(L.kf_obs_ptr, kN * 4));
    VX_HIP(c, grow(L.dyn, kDynInts * 4));
    if (with_pkf) VX_HIP(c, grow(L.pkf, fN * 4));

    uint8_t* WD = L.win.as<uint8_t>();
    LeanArgs& a = K.a;
    a = LeanArgs{};
    a.nk = nk;
    a.nf = nf;
    a.mw = mw;
    a.src = reinterpret_cast<const int64_t*>(WD + o_src);
    a.wid = reinterpret_cast<const uint64_t*>(WD + o_wid);
    a.wptr = reinterpret_cast<const int*>(WD + o_wptr);
    a.win = reinterpret_cast<const int*>(WD + o_win);
    a.cam = WD + o_cam;
    a.nl = nl;
    a.nobs = nobs;
    a.feat_uv = m->feat_uv.as<double>();
    a.feat_lm = m->feat_lm.as<uint64_t>();
    a.feat_fl = m->feat_fl.as<uint8_t>();
    a.lm_id = m->lm_id.as<uint64_t>();
    a.lm_bad = m->lm_bad.as<uint8_t>();
    a.lm_pos = m->lm_pos.as<double>();
    a.obs_lm = m->obs_lm.as<int>();
    a.obs_kf = m->obs_kf.as<uint64_t>();
    a.obs_fi = m->obs_fi.as<uint64_t>();
    a.map_pose = m->kf_pose.as<double>();
    a.map_intr = m->kf_intr.as<double>();
    a.ht_key = m->ht_key.as<uint64_t>();
    a.ht_val = m->ht_val.as<int>();
    a.ht_mask = m->ht_cap - 1;
    a.min_point = min_point;
    a.f_l = L.f_l.as<int>();
    a.f_code = L.f_code.as<int>();
    a.f_pv = L.f_pv.as<int>();
    a.f_back = L.f_back.as<int>();
    a.wuv = L.wuv.as<double2>();
    a.l_ref = L.l_ref.as<int>();
    a.l_pv = L.l_pv.as<int>();
    a.l_cnt = L.l_cnt.as<int>();
    a.key = L.key.as<unsigned long long>();
    a.ex = L.ex.as<unsigned long long>();
    a.l_slot = L.l_slot.as<int>();
    a.inv = L.inv.as<int>();
    a.cnt = L.cnt.as<int>();
    a.mask = L.mask.as<unsigned long long>();
    a.pscan = L.pscan.as<int>();
    a.lobs_ptr = L.lobs_ptr.as<int>();
    a.lm_pos0 = L.lm_pos0.as<double>();
    a.puv = L.puv.as<double2>();
    a.plm = L.plm.as<int>();
    a.pkf = with_pkf ? L.pkf.as<int>() : nullptr;
    a.kf_obs_ptr = L.kf_obs_ptr.as<int>();
    a.lkf = L.lkf.as<int>();
    a.llm = L.llm.as<int>();
    a.luv = L.luv.as<double2>();
    a.lm_blk = L.lm_blk.as<int>();
    a.kf_pose0 = L.kf_pose0.as<double>();
    a.kf_intr = L.kf_intr.as<double>();
    a.kf_flags = L.kf_flags.as<int>();
    a.dyn = L.dyn.as<int>();
    a.q = q;
    hipStream_t sm = c->stream;
    const long long n_big = std::max<long long>((long long)nl + 1, kDynInts);
    hipLaunchKernelGGL(k_lb_clear, dim3(grid(n_big)), dim3(kT), 0, sm, a);
    hipLaunchKernelGGL(k_lb_feat, dim3(grid(std::max<long long>(nf + 1, nk))), dim3(kT), 0, sm, a);
    if (nobs) hipLaunchKernelGGL(k_lb_obs, dim3(grid(nobs)), dim3(kT), 0, sm, a);
    hipLaunchKernelGGL(k_lb_flags, dim3(grid((long long)nl + 1)), dim3(kT), 0, sm, a);
    VX_LAUNCH_CHECK(c, "lean build: features / observations / flags");
    if ((rc = scan_ex<unsigned long long>(c, L.tmp, a.key, L.ex.as<unsigned long long>(), nl))) return rc;
    hipLaunchKernelGGL(k_lb_slots, dim3(grid((long long)nl + 1)), dim3(kT), 0, sm, a);
    if ((rc = scan_ex<int>(c, L.tmp, a.f_pv, L.pscan.as<int>(), nf))) return rc;
    hipLaunchKernelGGL(k_lb_pose, dim3(grid(std::max<long long>(nf, nk + 1))), dim3(kT), 0, sm, a);
    VX_LAUNCH_CHECK(c, "lean build: slots / pose CSR");
    if (!lstage) return VX_OK;
    hipLaunchKernelGGL(k_lb_lcount, dim3(grid((long long)nl + 1)), dim3(kT), 0, sm, a);
    VX_LAUNCH_CHECK(c, "lean build: landmark-stage counts");
    if ((rc = scan_ex<int>(c, L.tmp, a.cnt, L.lobs_ptr.as<int>(), nl))) return rc;
    hipLaunchKernelGGL(k_lb_lfill, dim3(grid(std::max<long long>(nf, nl))), dim3(kT), 0, sm, a);
    VX_LAUNCH_CHECK(c, "lean build: landmark-stage CSR");
    return VX_OK;
}


// ---------------------------------------------------------------- Schur plan from the resident map
// vx_sba_plan_create_dmap: the observation, pair and block tables of sba.hip's build_sba_plan,
// made on the device from the lean core build's pose-stage CSR (same window, landmark set, slots and
// observation set as the snapshot build: sba.hip keeps the reference's LocalBA selection):
//   observations   the pose-stage observations stably sorted by (optimised slot, or n_opt for the
//                  fixed landmarks): optimised landmarks landmark-major with their keyframes in window
//                  order, then the fixed landmarks' observations keyframe-major (radix sort)
//   keyframe lists every keyframe's observation indices, ascending (stable sort by keyframe row)
//   pairs          per optimised landmark every (a1, a2) of its observations with free keyframes
//                  i = kf(a1) >= j = kf(a2), counted, scanned and emitted in (slot, a1, a2) order,
//                  then stably sorted by block: the diagonal blocks (every window keyframe) first,
//                  then the non-empty off-diagonal blocks by (i, j) — the snapshot build's order
//   k_sba_lm       whole landmarks per workgroup, slot s -> (lm_ptr[s] + s) / (256 - most observations)
// Two read-backs size what follows (the counts; then the block list for the host's covisibility
// components and symbolic factorisation, sba_plan_finish).
struct SbaArgs {
    int nk, nf;
    int64_t nl;
    int pad_kf;
    const int* dyn_r;
    int* dyn;
    const int* plm;
    const int* pkf;
    const double2* puv;
    const int* kflags;        // window row flags (bit1: fixed)
    int* pkey;
    const int* skey;
    int* perm;
    int* scnt;                // per optimised slot: observations (scan input)
    const int* lm_ptr;
    double2* obs_uv;
    int* obs_lm;
    int* obs_kf;
    int* k2;
    int* v2;
    int* pc;                  // per optimised slot: pairs (scan input)
    const int* pptr;
    int* kcnt;                // per (i, j) key, i > j: 1 if a landmark joins keyframes i and j
    int* oflag;
    const int* orank;
    int* bidx;
    int2* bij;
    int* ekey;
    unsigned long long* eval;
    int* lm_blk;
    int q;
};

// The observations in (optimised slot | n_opt) order, stable — what a radix sort by that key gives —
// without the sort (three onesweep passes over every observation): per slot a count (scanned into
// lm_ptr) and a cursor, each slot's few observations then put back in index order (k_sb_fix); the
// fixed landmarks' observations (key n_opt) at the exclusive scan of their flags, in index order.
__global__ __launch_bounds__(kT) void k_sb_keys(SbaArgs a) {
    const int o = blockIdx.x * kT + threadIdx.x;
    if (o >= a.nf) return;
    const int n_obs = a.dyn[kDynPoseObs], n_opt = a.dyn[kDynNOpt];
    int fixed = 0;
    if (o < n_obs) {
        const int s = a.plm[o];
        if (s < n_opt) atomicAdd(&a.scnt[s], 1);
        else fixed = 1;
    }
    a.pkey[o] = fixed;  // (scan input: the fixed observations' ranks)
}

__global__ __launch_bounds__(kT) void k_sb_scatter(SbaArgs a) {
    const int o = blockIdx.x * kT + threadIdx.x;
    if (o >= a.dyn_r[kDynPoseObs]) return;
    const int n_opt = a.dyn_r[kDynNOpt], s = a.plm[o];
    const int p = s < n_opt ? a.lm_ptr[s] + atomicSub(&a.scnt[s], 1) - 1 : a.lm_ptr[n_opt] + a.skey[o];
    a.perm[p] = o;
}

// each optimised slot's observations (at most kSbaLmThreads) in ascending index order
__global__ __launch_bounds__(kT) void k_sb_fix(SbaArgs a) {
    const int s = blockIdx.x * kT + threadIdx.x;
    if (s >= a.dyn_r[kDynNOpt]) return;
    const int p0 = a.lm_ptr[s], p1 = a.lm_ptr[s + 1];
    for (int i = p0 + 1; i < p1; ++i) {
        const int v = a.perm[i];
        int j = i;
        for (; j > p0 && a.perm[j - 1] > v; --j) a.perm[j] = a.perm[j - 1];
        a.perm[j] = v;
    }
}

__global__ __launch_bounds__(kT) void k_sb_obs(SbaArgs a) {
    const int p = blockIdx.x * kT + threadIdx.x;
    if (p >= a.nf) return;
    const int n_obs = a.dyn[kDynPoseObs];
    if (p == 0) a.dyn[kDynSbaOo] = a.lm_ptr[a.dyn[kDynNOpt]];
    int kf = a.pad_kf;
    if (p < n_obs) {
        const int o = a.perm[p];
        kf = a.pkf[o];
        a.obs_uv[p] = a.puv[o];
        a.obs_lm[p] = a.plm[o];
        a.obs_kf[p] = kf;
    }
    a.k2[p] = kf;
    a.v2[p] = p;
}

// pairs of slot s: (a1, a2) over its observations, both keyframes free, kf(a2) <= kf(a1)
template <bool kEmit>
__device__ __forceinline__ int sb_pairs(const SbaArgs& a, int s) {
    const int o0 = a.lm_ptr[s], o1 = a.lm_ptr[s + 1];
    int c = 0;
    const int base = kEmit ? a.pptr[s] : 0;
    for (int a1 = o0; a1 < o1; ++a1) {
        const int i = a.obs_kf[a1];
        if (a.kflags[i] & 2) continue;
        for (int a2 = o0; a2 < o1; ++a2) {
            const int j = a.obs_kf[a2];
            if ((a.kflags[j] & 2) || j > i) continue;
            const int key = i * a.nk + j;
            if (kEmit) {
                a.ekey[base + c] = a.bidx[key];
                a.eval[base + c] = (unsigned long long)(unsigned)a1 | ((unsigned long long)(unsigned)a2 << 32);
            } else if (j != i && !a.kcnt[key]) {
                // an off-diagonal block exists: a flag, not a count (a count per pair was one global
                // atomic per pair, ~1700 of them on each diagonal key; the pairs per block come from
                // the sorted pair list instead, k_sb_bptr)
                a.kcnt[key] = 1;
            }
            ++c;
        }
    }
    return c;
}

__global__ __launch_bounds__(kT) void k_sb_pcount(SbaArgs a) {
    const int64_t s = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (s > a.nl) return;
    const int n_opt = a.dyn[kDynNOpt];
    int c = 0;
    if (s < n_opt) {
        c = sb_pairs<false>(a, (int)s);
        atomicMax(&a.dyn[kDynSbaMaxObs], a.lm_ptr[s + 1] - a.lm_ptr[s]);
    }
    a.pc[s] = c;
}

__global__ __launch_bounds__(kT) void k_sb_bflag(SbaArgs a) {
    const int key = blockIdx.x * kT + threadIdx.x;
    const int n2 = a.nk * a.nk;
    if (key > n2) return;
    int f = 0;
    if (key < n2) {
        const int i = key / a.nk, j = key - i * a.nk;
        f = (i != j && a.kcnt[key] > 0) ? 1 : 0;
    }
    a.oflag[key] = f;
}

__global__ __launch_bounds__(kT) void k_sb_btab(SbaArgs a) {
    const int key = blockIdx.x * kT + threadIdx.x;
    const int n2 = a.nk * a.nk;
    if (key == 0) {
        a.dyn[kDynSbaBlocks] = a.nk + a.orank[n2];
        a.dyn[kDynSbaPairs] = a.pptr[a.dyn[kDynNOpt]];
    }
    if (key >= n2) return;
    const int i = key / a.nk, j = key - i * a.nk;
    int b = -1;
    if (i == j) b = i;
    else if (a.kcnt[key] > 0) b = a.nk + a.orank[key];
    a.bidx[key] = b;
    if (b < 0) return;
    a.bij[b] = make_int2(i, j);
}

// block b's pairs [blk_ptr[b], blk_ptr[b + 1]) from the pairs sorted by block (empty blocks: the
// diagonal blocks of fixed or unobserved keyframes): position p starts every block in (key[p - 1], key[p]]
__global__ __launch_bounds__(kT) void k_sb_bptr(const int* __restrict__ key, int n_pairs, int n_blocks,
                                                int* __restrict__ blk_ptr) {
    const int p = blockIdx.x * kT + threadIdx.x;
    if (p > n_pairs) return;
    const int k0 = p > 0 ? key[p - 1] : -1, k1 = p < n_pairs ? key[p] : n_blocks;
    for (int b = k0 + 1; b <= k1; ++b) blk_ptr[b] = p;
}

__global__ __launch_bounds__(kT) void k_sb_pemit(SbaArgs a) {
    const int s = blockIdx.x * kT + threadIdx.x;
    if (s < a.dyn_r[kDynNOpt]) sb_pairs<true>(a, s);
}

// k_sba_lm workgroups (q = 256 - most observations of one landmark >= that count + 1)
__global__ __launch_bounds__(kT) void k_sb_lmblk(SbaArgs a) {
    const int s = blockIdx.x * kT + threadIdx.x;
    const int n_opt = a.dyn_r[kDynNOpt];
    if (s >= n_opt) return;
    const int b = (a.lm_ptr[s] + s) / a.q;
    const int bp = s ? (a.lm_ptr[s - 1] + s - 1) / a.q : -1;
    if (b != bp) a.lm_blk[b] = s;
    if (s == n_opt - 1) {
        a.lm_blk[b + 1] = n_opt;
        a.dyn[kDynSbaLmBlocks] = b + 1;
    }
}

unsigned bits_for(int64_t v) {  // radix bits holding [0, v]
    unsigned b = 1;
    while ((1ll << b) <= v) ++b;
    return b;
}

template <class K, class V>
int sort_pairs(vx_ctx* c, DevBuf& tmp, K* ki, K* ko, V* vi, V* vo, size_t n, unsigned bits) {
    size_t bytes = 0;
    VX_HIP(c, rocprim::radix_sort_pairs<OnesweepSort>(nullptr, bytes, ki, ko, vi, vo, n, 0, bits, c->stream));
    VX_HIP(c, grow(tmp, std::max<size_t>(bytes, 16)));
    VX_HIP(c, rocprim::radix_sort_pairs<OnesweepSort>(tmp.p, bytes, ki, ko, vi, vo, n, 0, bits, c->stream));
    return VX_OK;
}

// SelectKeyFrames over the resident keyframes (ba_window.hip)
std::vector<int> dmap_select_window(const vx_dmap* m, uint64_t ref_kf_id, int has_ref, int window_size);

// The lean build + run + apply; returns VX_ERR_STATE (*fallback = true) for a window it does not take
// (more than 255 keyframes, a landmark-stage grid beyond the LDS-pose kernels' range).
int lean_optimize(vx_ctx* c, vx_dmap* m, uint64_t ref, int has_ref, const vx_ba_options& o, vx_ba_stats* st,
                  bool* fallback) {
    *fallback = false;
    auto& L = m->lean;
    L.nk = 0;
    L.status = 1;
    L.ran = false;
    L.win_rows.clear();
    vx_ba_stats s{};
    s.gate_margin = -1.0;
    s.status = 1;
    const int n_kf = (int)m->kf_id.size();
    std::vector<int> win = n_kf > 0 ? dmap_select_window(m, ref, has_ref, o.window_size) : std::vector<int>{};
    const int nk = (int)win.size();
    s.n_window_kf = nk;
    if (nk < 2) {  // local_ba.cpp:73-75
        L.ran = true;
        if (st) *st = s;
        return VX_OK;
    }
    const int q = kBaLmBlock - nk;
    LeanCore K;
    lean_window(m, win, K);
    const int cap_blocks = (int)((2 * K.nvalid + q - 1) / q) + 1;
    if (nk > 255 || cap_blocks > 480 || (int64_t)nk * cap_blocks > 80000 || K.nl >= INT_MAX / 2) {
        *fallback = true;
        return VX_ERR_STATE;
    }
    const int n_split = ba_split(K.mx, 1);
    int rc;
    if ((rc = lean_build_core(c, m, o.min_point_observations, q, true, cap_blocks, false, K))) return rc;
    const LeanArgs& a = K.a;
    const int64_t nl = K.nl;
    hipStream_t sm = c->stream;
    VX_HIP(c, grow(L.kf_pose, ((size_t)nk + 1) * 128));
    VX_HIP(c, grow(L.kf_rot, ((size_t)nk + 1) * 72));
    VX_HIP(c, grow(L.kf_part, ((size_t)nk + 1) * n_split * kBaStrideDoubles * 8));
    VX_HIP(c, grow(L.kf_cost, ((size_t)nk + 1) * 16));
    VX_HIP(c, grow(L.state, ba_state_bytes()));
    VX_HIP(c, grow(L.lm_pos, ((size_t)nl + 1) * 32));

    DynPlan d;
    d.n_kf = nk;
    d.n_split = n_split;
    d.grid_blocks = cap_blocks;
    d.opt = o;
    d.kf_pose0 = a.kf_pose0;
    d.kf_pose = L.kf_pose.as<double>();
    d.kf_intr = a.kf_intr;
    d.kf_rot = L.kf_rot.as<double>();
    d.kf_flags = a.kf_flags;
    d.kf_obs_ptr = a.kf_obs_ptr;
    d.kf_part = L.kf_part.as<double>();
    d.kf_cost = L.kf_cost.as<double>();
    d.lm_pos0 = a.lm_pos0;
    d.lm_pos = L.lm_pos.as<double>();
    d.pobs_uv = a.puv;
    d.pobs_lm = a.plm;
    d.lobs_ptr = a.lobs_ptr;
    d.lobs_kf = a.lkf;
    d.lobs_lm = a.llm;
    d.lm_blk = a.lm_blk;
    d.lobs_uv = a.luv;
    d.state = L.state.p;
    d.dyn = a.dyn;
    if (o.max_iterations > 0) {
        if ((rc = ba_run_dyn(c, d))) return rc;
    }
    // the end: the header (and the iteration state) back — the call's only synchronisation; with
    // vx_dmap_prefetch_results the results too (both pose parities, positions and rows by capacity).
    // After a run, k_lb_apply packs all of it into one device block and ONE copy brings it back.
    const size_t sb = ba_state_bytes();
    const size_t hdr_b = kDynInts * 4 + sb, hdr_pad = (hdr_b + 63) & ~(size_t)63;
    const bool pf = L.prefetch && o.max_iterations > 0;
    const size_t pose_b = 2 * (size_t)nk * 64, pos_b = (size_t)nl * 32, rows_b = (size_t)nl * 4;
    const size_t pack_b = o.max_iterations > 0 ? (pf ? hdr_pad + pose_b + pos_b + rows_b : hdr_b) : 0;
    int* H = nullptr;
    if (o.max_iterations > 0) {
        VX_HIP(c, grow(L.pack, pack_b));
        // (the apply takes the last iteration's pose buffer from BAState::iterations on the device)
        const int* iters = reinterpret_cast<const int*>(static_cast<const uint8_t*>(L.state.p) + ba_state_iter_offset());
        hipLaunchKernelGGL(k_lb_apply, dim3(grid(std::max<long long>(std::max<long long>(nk, nl), (long long)hdr_b / 4))),
                           dim3(kT), 0, sm, (const int*)a.dyn, iters, nk, a.win, (const double*)L.kf_pose.as<double>(),
                           (const int*)a.inv, nl, (const double*)L.lm_pos.as<double>(), m->kf_pose.as<double>(),
                           m->lm_pos.as<double>(), L.pack.as<uint8_t>(), L.state.as<int>(), (int)(hdr_b / 4),
                           pf ? (int64_t)hdr_pad : (int64_t)-1);
        VX_LAUNCH_CHECK(c, "k_lb_apply");
        PinnedBuf& dst = pf ? L.res_host : L.rb_host;
        VX_HIP(c, dst.ensure(pack_b + 64, pf));  // (the results' block host-cached, as before)
        VX_HIP(c, hipMemcpyAsync(dst.p, L.pack.p, pack_b, hipMemcpyDeviceToHost, sm));
        H = static_cast<int*>(dst.p);
    } else {
        VX_HIP(c, L.rb_host.ensure(hdr_b));
        H = static_cast<int*>(L.rb_host.p);
        VX_HIP(c, hipMemcpyAsync(H, a.dyn, kDynInts * 4, hipMemcpyDeviceToHost, sm));
    }
    L.prefetched = pf;
    if (pf) {
        L.pf_nl = nl;
        L.res_off = hdr_pad;
    }
    VX_HIP(c, hipStreamSynchronize(sm));
    s.status = H[kDynStatus];
    s.n_landmarks = H[kDynGlobal];
    // (with no optimisable landmark no kernel of the run touched the state: iterations stay 0)
    if (s.status == 0 && o.max_iterations > 0) ba_state_to_stats(H + kDynInts, &s);
    L.nk = nk;
    L.status = s.status;
    L.n_opt = H[kDynNOpt];
    L.iterations = s.iterations;
    L.win_rows = std::move(win);
    L.ran = true;
    if (st) *st = s;
    return VX_OK;
}


// The Schur plan's tables from the resident map (see above); p->opt set by the caller
int build_sba_plan_dmap(vx_ctx* c, vx_dmap* m, uint64_t ref, int has_ref, vx_sba_plan* p) {
    const PlanClock clk;
    const vx_sba_options& o = p->opt;
    p->status = 1;
    p->from_dmap = true;
    // this build reuses (and may reallocate) the lean core's scratch that vx_ba_dmap_results reads
    // (inv, lm_pos0, kf_pose0, win): a LocalBA result from before it can no longer be reported
    // (vx_ba_dmap_results then fails with VX_ERR_STATE until the next vx_ba_optimize_dmap)
    m->lean.ran = false;
    const int n_kf = (int)m->kf_id.size();
    std::vector<int> win = n_kf > 0 ? dmap_select_window(m, ref, has_ref, o.window_size) : std::vector<int>{};
    const int nk = (int)win.size();
    p->n_window_kf = nk;
    p->n_landmarks_global = 0;
    if (nk < 2) return VX_OK;
    LeanCore K;
    lean_window(m, win, K);
    if (nk > 448 || K.nl >= INT_MAX / 2 || (int64_t)K.nf * 2 >= INT_MAX)
        return set_error(c, VX_ERR_INVALID, "vx_sba_plan_create_dmap: window of %d keyframes (max 448)", nk);
    int rc;
    if ((rc = lean_build_core(c, m, o.min_point_observations, 1, false, 0, true, K))) return rc;
    clk.mark("sba core enqueued");
    auto& L = m->lean;
    auto& B = m->sba;
    const int nf = K.nf;
    const int64_t nl = K.nl;
    hipStream_t sm = c->stream;
    // keyframe flags (bit0 camera, bit1 fixed: the oldest fixed_keyframes and camera-less ones)
    std::vector<int> flags(nk);
    for (int r = 0; r < nk; ++r) flags[r] = (K.cam[r] ? 1 : 0) | ((r < o.fixed_keyframes || !K.cam[r]) ? 2 : 0);
    VX_HIP(c, p->kf_flags.ensure((size_t)nk * 4));
    VX_HIP(c, hipMemcpyAsync(p->kf_flags.p, flags.data(), (size_t)nk * 4, hipMemcpyHostToDevice, sm));
    const size_t fN = (size_t)nf + 1, lN = (size_t)nl + 2;
    const int n2 = nk * nk;
    for (DevBuf* d : {&B.pkey, &B.skey, &B.perm, &B.k2, &B.v2}) VX_HIP(c, grow(*d, fN * 4));
    for (DevBuf* d : {&B.scnt, &B.pc, &B.pptr}) VX_HIP(c, grow(*d, lN * 4));
    for (DevBuf* d : {&B.kcnt, &B.oflag, &B.orank, &B.bidx}) VX_HIP(c, grow(*d, ((size_t)n2 + 1) * 4));
    VX_HIP(c, p->blk_ij.ensure(((size_t)n2 + nk + 1) * 8));
    VX_HIP(c, p->blk_ptr.ensure(((size_t)n2 + nk + 1) * 4));
    VX_HIP(c, p->obs_uv.ensure(fN * 16));
    VX_HIP(c, p->obs_lm.ensure(fN * 4));
    VX_HIP(c, p->obs_kf.ensure(fN * 4));
    VX_HIP(c, p->kf_obs.ensure(fN * 4));
    VX_HIP(c, p->lm_ptr.ensure(lN * 4));
    VX_HIP(c, hipMemsetAsync(B.scnt.p, 0, lN * 4, sm));
    VX_HIP(c, hipMemsetAsync(B.kcnt.p, 0, ((size_t)n2 + 1) * 4, sm));
    SbaArgs a{};
    a.nk = nk;
    a.nf = nf;
    a.nl = nl;
    a.pad_kf = (int)((1ll << bits_for(nk)) - 1);
    a.dyn = K.a.dyn;
    a.dyn_r = K.a.dyn;
    a.plm = K.a.plm;
    a.pkf = K.a.pkf;
    a.puv = K.a.puv;
    a.kflags = p->kf_flags.as<int>();
    a.pkey = B.pkey.as<int>();
    a.skey = B.skey.as<int>();
    a.perm = B.perm.as<int>();
    a.scnt = B.scnt.as<int>();
    a.lm_ptr = p->lm_ptr.as<int>();
    a.obs_uv = p->obs_uv.as<double2>();
    a.obs_lm = p->obs_lm.as<int>();
    a.obs_kf = p->obs_kf.as<int>();
    a.k2 = B.k2.as<int>();
    a.v2 = B.v2.as<int>();
    a.pc = B.pc.as<int>();
    a.pptr = B.pptr.as<int>();
    a.kcnt = B.kcnt.as<int>();
    a.oflag = B.oflag.as<int>();
    a.orank = B.orank.as<int>();
    a.bidx = B.bidx.as<int>();
    a.bij = p->blk_ij.as<int2>();
    // observations in stable (optimised slot | n_opt) order, landmark pointers
    hipLaunchKernelGGL(k_sb_keys, dim3(grid(nf)), dim3(kT), 0, sm, a);
    VX_LAUNCH_CHECK(c, "k_sb_keys");
    if ((rc = scan_ex<int>(c, L.tmp, a.scnt, p->lm_ptr.as<int>(), nl))) return rc;
    if ((rc = scan_ex<int>(c, L.tmp, a.pkey, B.skey.as<int>(), nf))) return rc;
    hipLaunchKernelGGL(k_sb_scatter, dim3(grid(nf)), dim3(kT), 0, sm, a);
    hipLaunchKernelGGL(k_sb_fix, dim3(grid(nl)), dim3(kT), 0, sm, a);
    VX_LAUNCH_CHECK(c, "k_sb_scatter / k_sb_fix");
    hipLaunchKernelGGL(k_sb_obs, dim3(grid(nf)), dim3(kT), 0, sm, a);
    VX_LAUNCH_CHECK(c, "k_sb_obs");
    // keyframe lists: observation indices by window row, ascending within a row
    if (nf && (rc = sort_pairs(c, B.tmp, a.k2, B.pkey.as<int>(), a.v2, p->kf_obs.as<int>(), (size_t)nf,
                               bits_for(a.pad_kf))))
        return rc;
    // pairs: counts per slot and per block key, block table
    hipLaunchKernelGGL(k_sb_pcount, dim3(grid((long long)nl + 1)), dim3(kT), 0, sm, a);
    VX_LAUNCH_CHECK(c, "k_sb_pcount");
    if ((rc = scan_ex<int>(c, L.tmp, a.pc, B.pptr.as<int>(), nl))) return rc;
    hipLaunchKernelGGL(k_sb_bflag, dim3(grid((long long)n2 + 1)), dim3(kT), 0, sm, a);
    if ((rc = scan_ex<int>(c, L.tmp, a.oflag, B.orank.as<int>(), n2))) return rc;
    hipLaunchKernelGGL(k_sb_btab, dim3(grid(n2)), dim3(kT), 0, sm, a);
    VX_LAUNCH_CHECK(c, "k_sb_btab");
    // ---- read-back 1: the counts
    VX_HIP(c, B.rb.ensure(kDynInts * 4 + ((size_t)n2 + nk + 1) * 8));
    int* H = static_cast<int*>(B.rb.p);
    VX_HIP(c, hipMemcpyAsync(H, a.dyn, kDynInts * 4, hipMemcpyDeviceToHost, sm));
    VX_HIP(c, hipStreamSynchronize(sm));
    clk.mark("sba read-back 1 (counts)");
    p->n_landmarks_global = H[kDynGlobal];
    if (H[kDynStatus]) return VX_OK;  // no optimisable landmark (local_ba.cpp:106-108)
    const int n_opt = H[kDynNOpt], n_lm = H[kDynNLm], n_obs = H[kDynPoseObs], n_oo = H[kDynSbaOo];
    const int64_t n_pairs = H[kDynSbaPairs];
    const int max_obs = H[kDynSbaMaxObs], n_blocks = H[kDynSbaBlocks];
    if (max_obs > kSbaLmThreads)
        return set_error(c, VX_ERR_INVALID, "landmark with %d observations in the window (max %d)", max_obs,
                         kSbaLmThreads);
    p->status = 0;
    p->nk = nk;
    p->n_opt = n_opt;
    p->n_lm = n_lm;
    p->n_oo = n_oo;
    p->n_obs = n_obs;
    p->n_pairs = n_pairs;
    p->n_blocks = n_blocks;
    p->kf_map_idx = win;
    p->lm_map_idx.clear();  // (on the device: lm_map_dev)
    // pairs: emitted in (slot, a1, a2) order, stably sorted by block
    for (DevBuf* d : {&B.ekey, &B.ekey2}) VX_HIP(c, grow(*d, ((size_t)n_pairs + 1) * 4));
    VX_HIP(c, grow(B.eval, ((size_t)n_pairs + 1) * 8));
    VX_HIP(c, p->pairs.ensure(((size_t)n_pairs + 1) * 8));
    a.ekey = B.ekey.as<int>();
    a.eval = B.eval.as<unsigned long long>();
    hipLaunchKernelGGL(k_sb_pemit, dim3(grid(n_opt)), dim3(kT), 0, sm, a);
    VX_LAUNCH_CHECK(c, "k_sb_pemit");
    if (n_pairs && (rc = sort_pairs(c, B.tmp, a.ekey, B.ekey2.as<int>(), a.eval, p->pairs.as<unsigned long long>(),
                                    (size_t)n_pairs, bits_for(n_blocks))))
        return rc;
    hipLaunchKernelGGL(k_sb_bptr, dim3(grid(n_pairs + 1)), dim3(kT), 0, sm, (const int*)B.ekey2.as<int>(),
                       (int)n_pairs, n_blocks, p->blk_ptr.as<int>());
    VX_LAUNCH_CHECK(c, "k_sb_bptr");
    // k_sba_lm workgroups
    a.q = kSbaLmThreads - max_obs;
    VX_HIP(c, p->lm_blk.ensure(((size_t)(n_oo + n_opt) / std::max(a.q, 1) + 3) * 4));
    a.lm_blk = p->lm_blk.as<int>();
    if (max_obs <= kSbaLmThreads / 2 - 1) {
        hipLaunchKernelGGL(k_sb_lmblk, dim3(grid(n_opt)), dim3(kT), 0, sm, a);
        VX_LAUNCH_CHECK(c, "k_sb_lmblk");
    }
    // tables the run reads from the core build: keyframe poses / intrinsics / observation pointers,
    // initial positions by slot, and the scatter tables
    VX_HIP(c, p->pose0.ensure((size_t)nk * 64));
    VX_HIP(c, p->intr.ensure((size_t)nk * 32));
    VX_HIP(c, p->kf_ptr.ensure(((size_t)nk + 1) * 4));
    VX_HIP(c, p->lm0.ensure((size_t)std::max(n_lm, 1) * 32));
    VX_HIP(c, p->lm_map_dev.ensure((size_t)std::max(n_lm, 1) * 4));
    VX_HIP(c, p->kf_map_dev.ensure((size_t)nk * 4));
    {  // (one launch for the six copies)
        MultiCopy mc;
        bool ok = mc.add(p->pose0.p, K.a.kf_pose0, (size_t)nk * 64) && mc.add(p->intr.p, K.a.kf_intr, (size_t)nk * 32) &&
                  mc.add(p->kf_ptr.p, K.a.kf_obs_ptr, ((size_t)nk + 1) * 4) &&
                  mc.add(p->lm0.p, K.a.lm_pos0, (size_t)n_lm * 32) && mc.add(p->lm_map_dev.p, K.a.inv, (size_t)n_lm * 4) &&
                  mc.add(p->kf_map_dev.p, K.a.win, (size_t)nk * 4);
        if (!ok) return set_error(c, VX_ERR_STATE, "sba plan: unaligned table copy");
        VX_HIP(c, mc.launch(sm));
    }
    // ---- read-back 2: the workgroup count and the block list (the host's components and symbolic
    // factorisation need it)
    int2* HB = reinterpret_cast<int2*>(H + kDynInts);
    VX_HIP(c, hipMemcpyAsync(H, a.dyn, kDynInts * 4, hipMemcpyDeviceToHost, sm));
    VX_HIP(c, hipMemcpyAsync(HB, p->blk_ij.p, (size_t)n_blocks * 8, hipMemcpyDeviceToHost, sm));
    std::vector<int> lptr_h;
    if (max_obs > kSbaLmThreads / 2 - 1) {  // (a landmark seen by more than 127 window keyframes)
        lptr_h.resize((size_t)n_opt + 1);
        VX_HIP(c, hipMemcpyAsync(lptr_h.data(), p->lm_ptr.p, lptr_h.size() * 4, hipMemcpyDeviceToHost, sm));
    }
    clk.mark("sba pairs enqueued");
    VX_HIP(c, hipStreamSynchronize(sm));
    clk.mark("sba read-back 2 (blocks)");
    if (!lptr_h.empty()) {  // greedy packing on the host, as build_sba_plan does
        std::vector<int> blk{0};
        int n_o = 0, n_l = 0;
        for (int sl = 0; sl < n_opt; ++sl) {
            const int cnt = lptr_h[sl + 1] - lptr_h[sl];
            if (n_l + 1 > kSbaLmThreads || n_o + cnt > kSbaLmThreads) {
                blk.push_back(sl);
                n_o = n_l = 0;
            }
            n_o += cnt;
            ++n_l;
        }
        blk.push_back(n_opt);
        VX_HIP(c, p->lm_blk.ensure(blk.size() * 4));
        VX_HIP(c, hipMemcpy(p->lm_blk.p, blk.data(), blk.size() * 4, hipMemcpyHostToDevice));
        p->n_lm_blocks = (int)blk.size() - 1;
    } else {
        p->n_lm_blocks = n_opt ? H[kDynSbaLmBlocks] : 0;
    }
    const std::vector<int2> bij(HB, HB + n_blocks);
    return sba_plan_finish(c, p, flags, bij, &clk);
}
}  // namespace vx

vx_dmap::~vx_dmap() {
    if (lean.fallback) vx_ba_plan_destroy(lean.fallback);
}

using namespace vx;

namespace vx {
namespace {
// obs_lm of a view: the landmark row of each observation, from the landmark-major CSR pointers
__global__ __launch_bounds__(kT) void k_view_obs_rows(const int64_t* __restrict__ optr, int64_t nl, int* __restrict__ obs_lm) {
    const int64_t l = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (l >= nl) return;
    for (int64_t o = optr[l]; o < optr[l + 1]; ++o) obs_lm[o] = (int)l;
}

template <class T>
int view_up(vx_ctx* c, vx::DevBuf& d, const T* h, size_t n) {
    VX_HIP(c, grow(d, std::max<size_t>(n, 1) * sizeof(T)));
    if (n) VX_HIP(c, hipMemcpyAsync(d.p, h, n * sizeof(T), hipMemcpyHostToDevice, c->stream));
    return VX_OK;
}
}  // namespace

// vx_ba_optimize_map through the lean one-call build (round 6): the view is loaded into the
// context's scratch vx_dmap — its arrays uploaded as they are (one DMA each when they are
// page-locked, as visionx::FlatMap's are), the observation rows expanded from the CSR on the device,
// the host mirrors the window selection reads copied — and lean_optimize runs on it with its single
// synchronisation, the results coming back in the same copy (prefetch).  The general plan build
// needs four synchronisations (ba_window.hip: counts, fused packing, fused entries; the fetch).
// *fallback: a window the lean build does not take (the caller then builds a plan).
int lean_optimize_view(vx_ctx* c, vx_map_view* v, uint64_t ref, int has_ref, const vx_ba_options& o, vx_ba_stats* st,
                       bool* fallback) {
    *fallback = false;
    if (!c->snap_map) {
        int rc = vx_dmap_create(c, &c->snap_map);
        if (rc) return rc;
    }
    vx_dmap* m = c->snap_map;
    const int nk = v->n_kf;
    if (nk < 2 || v->n_lm < 0) {  // (nothing to select: the plan path's checks and early exits)
        *fallback = true;
        return VX_ERR_STATE;
    }
    const int64_t nl = v->n_lm, nf = v->kf_feat_ptr[nk], nobs = nl > 0 ? v->lm_obs_ptr[nl] : 0;
    if (nl >= INT_MAX / 2 || nf >= INT_MAX / 2 || nobs >= INT_MAX / 2) {
        *fallback = true;
        return VX_ERR_STATE;
    }
    // host mirrors: keyframe ids / rows / cameras, every keyframe live; the valid-feature counts only
    // for the window keyframes (the only ones lean_window reads)
    m->kf_id.assign(v->kf_id, v->kf_id + nk);
    m->kf_feat_ptr.assign(v->kf_feat_ptr, v->kf_feat_ptr + nk + 1);
    m->kf_has_cam.resize(nk);
    for (int k = 0; k < nk; ++k) m->kf_has_cam[k] = v->kf_has_cam[k] ? 1 : 0;
    m->kf_alive.assign(nk, 1);
    m->kf_valid_cnt.assign(nk, 0);
    for (int k : dmap_select_window(m, ref, has_ref, o.window_size)) {
        int cnt = 0;
        for (int64_t f = v->kf_feat_ptr[k]; f < v->kf_feat_ptr[k + 1]; ++f) cnt += v->feat_flags[f] & 1;
        m->kf_valid_cnt[k] = cnt;
    }
    m->n_lm = nl;
    m->n_obs = nobs;
    // device arrays
    VX_HIP(c, hipSetDevice(c->device));
    int rc;
    if ((rc = view_up(c, m->kf_pose, v->kf_pose, 7 * (size_t)nk))) return rc;
    if ((rc = view_up(c, m->kf_intr, v->kf_intr, 4 * (size_t)nk))) return rc;
    if ((rc = view_up(c, m->feat_uv, v->feat_uv, 2 * (size_t)nf))) return rc;
    if ((rc = view_up(c, m->feat_lm, v->feat_lm_id, (size_t)nf))) return rc;
    if ((rc = view_up(c, m->feat_fl, v->feat_flags, (size_t)nf))) return rc;
    if ((rc = view_up(c, m->lm_id, v->lm_id, (size_t)nl))) return rc;
    if ((rc = view_up(c, m->lm_pos, v->lm_pos, 3 * (size_t)nl))) return rc;
    if ((rc = view_up(c, m->lm_bad, v->lm_bad, (size_t)nl))) return rc;
    if ((rc = view_up(c, m->obs_kf, v->obs_kf_id, (size_t)nobs))) return rc;
    if ((rc = view_up(c, m->obs_fi, v->obs_feat_idx, (size_t)nobs))) return rc;
    if ((rc = view_up(c, m->optr, v->lm_obs_ptr, (size_t)nl + 1))) return rc;
    VX_HIP(c, grow(m->obs_lm, (size_t)std::max<int64_t>(nobs, 1) * 4));
    if (nl) {
        hipLaunchKernelGGL(k_view_obs_rows, dim3(grid(nl)), dim3(kT), 0, c->stream, (const int64_t*)m->optr.as<int64_t>(),
                           nl, m->obs_lm.as<int>());
        VX_LAUNCH_CHECK(c, "k_view_obs_rows");
    }
    // the id table of the previous view is stale: emptied, then refilled from row 0 (ht_sync)
    if (m->ht_cap) {
        hipLaunchKernelGGL(k_ht_clear, dim3(grid(m->ht_cap)), dim3(kT), 0, c->stream, m->ht_key.as<uint64_t>(), m->ht_cap);
        VX_LAUNCH_CHECK(c, "k_ht_clear");
    }
    m->ht_rows = 0;
    auto& L = m->lean;
    L.ran = false;
    L.prefetched = false;
    L.prefetch = true;
    vx_ba_stats s{};
    rc = lean_optimize(c, m, ref, has_ref, o, &s, fallback);
    if (*fallback || rc) return rc;
    // the results into the view (Frame::SetPose / Landmark::SetPosition happen in the caller)
    const int32_t *kr = nullptr, *lr = nullptr;
    const double *kp = nullptr, *lp = nullptr;
    int n_k = 0, n_l = 0;
    if ((rc = vx_ba_dmap_results_view(c, m, &kr, &kp, &lr, &lp, &n_k, &n_l))) return rc;
    for (int i = 0; i < n_k; ++i)
        for (int j = 0; j < 7; ++j) v->kf_pose[7 * (size_t)kr[i] + j] = kp[8 * (size_t)i + j];
    for (int i = 0; i < n_l; ++i)
        for (int j = 0; j < 3; ++j) v->lm_pos[3 * (size_t)lr[i] + j] = lp[4 * (size_t)i + j];
    if (st) *st = s;
    return VX_OK;
}
}  // namespace vx

extern "C" {

int vx_ba_optimize_dmap(vx_ctx* c, vx_dmap* m, uint64_t ref, int has_ref, const vx_ba_options* opt, vx_ba_stats* st) {
    if (!c || !m || !opt || m->c != c)
        return c ? set_error(c, VX_ERR_INVALID, "vx_ba_optimize_dmap: bad arguments") : VX_ERR_INVALID;
    if (opt->max_iterations < 0 || opt->max_iterations > 64)
        return set_error(c, VX_ERR_INVALID, "max_iterations must be in [0, 64]");
    auto& L = m->lean;
    if (L.fallback) {
        vx_ba_plan_destroy(L.fallback);
        L.fallback = nullptr;
    }
    L.ran = false;
    L.prefetched = false;
    // $VX_LEAN=0: always the general build (ba_window.hip), for A/B runs
    const char* e = getenv("VX_LEAN");
    bool fb = e && e[0] == '0';
    if (!fb) {
        const int rc = lean_optimize(c, m, ref, has_ref, *opt, st, &fb);
        if (!fb) return rc;
    }
    // a window the lean build does not take: plan from the resident map, run, scatter
    vx_ba_plan* p = nullptr;
    int rc = vx_ba_plan_create_dmap(c, m, ref, has_ref, opt, 0, 1, &p);
    if (rc) return rc;
    rc = vx_ba_plan_run_async(c, p);
    if (!rc) rc = vx_ba_plan_apply_dmap(c, p, m);
    vx_ba_stats s{};
    if (!rc) rc = vx_ba_plan_fetch(c, p, nullptr, &s);
    if (rc) {
        vx_ba_plan_destroy(p);
        return rc;
    }
    L.fallback = p;
    L.nk = s.status == 0 ? (int)p->kf_map_idx.size() : 0;
    L.status = s.status;
    L.n_opt = s.status == 0 ? p->n_opt : 0;
    L.iterations = s.iterations;
    L.win_rows = p->kf_map_idx;
    L.ran = true;
    if (st) *st = s;
    return VX_OK;
}

int vx_dmap_prefetch_results(vx_dmap* m, int on) {
    if (!m) return VX_ERR_INVALID;
    m->lean.prefetch = on != 0;
    return VX_OK;
}

int vx_ba_dmap_results_view(vx_ctx* c, vx_dmap* m, const int32_t** kf_rows, const double** kf_pose8,
                            const int32_t** lm_rows, const double** lm_pos4, int* n_kf, int* n_lm) {
    if (!c || !m || m->c != c || !n_kf || !n_lm || !kf_rows || !kf_pose8 || !lm_rows || !lm_pos4)
        return c ? set_error(c, VX_ERR_INVALID, "vx_ba_dmap_results_view: bad arguments") : VX_ERR_INVALID;
    auto& L = m->lean;
    if (!L.ran) return set_error(c, VX_ERR_STATE, "no vx_ba_optimize_dmap to report");
    const bool changed = L.status == 0 && L.iterations > 0;
    *n_kf = changed ? L.nk : 0;
    *n_lm = changed ? L.n_opt : 0;
    *kf_rows = *lm_rows = nullptr;
    *kf_pose8 = *lm_pos4 = nullptr;
    if (!changed) return VX_OK;
    if (!L.prefetched || L.fallback || L.n_opt > L.pf_nl)
        return set_error(c, VX_ERR_STATE, "results not prefetched (vx_dmap_prefetch_results): use vx_ba_dmap_results");
    const double* base = reinterpret_cast<const double*>(static_cast<const uint8_t*>(L.res_host.p) + L.res_off);
    *kf_rows = L.win_rows.data();
    *kf_pose8 = base + (size_t)(L.iterations & 1) * L.nk * 8;
    *lm_pos4 = base + 2 * (size_t)L.nk * 8;
    *lm_rows = reinterpret_cast<const int32_t*>(*lm_pos4 + (size_t)L.pf_nl * 4);
    return VX_OK;
}

int vx_ba_dmap_results(vx_ctx* c, vx_dmap* m, int cap_kf, int64_t* kf_rows, double* kf_pose7, int cap_lm,
                       int64_t* lm_rows, double* lm_pos3, int* n_kf, int* n_lm) {
    if (!c || !m || m->c != c || !n_kf || !n_lm) return c ? set_error(c, VX_ERR_INVALID, "vx_ba_dmap_results: bad arguments") : VX_ERR_INVALID;
    auto& L = m->lean;
    if (!L.ran) return set_error(c, VX_ERR_STATE, "no vx_ba_optimize_dmap to report");
    const bool changed = L.status == 0 && L.iterations > 0;
    *n_kf = changed ? L.nk : 0;
    *n_lm = changed ? L.n_opt : 0;
    if (!changed) return VX_OK;
    if (cap_kf < *n_kf || cap_lm < *n_lm) return set_error(c, VX_ERR_CAPACITY, "need %d keyframes / %d landmarks", *n_kf, *n_lm);
    const int nk = L.nk, n = L.n_opt;
    if (L.prefetched && !L.fallback && n <= L.pf_nl) {  // (vx_dmap_prefetch_results: host copies only)
        const double* base = reinterpret_cast<const double*>(static_cast<const uint8_t*>(L.res_host.p) + L.res_off);
        const double* pose = base + (size_t)(L.iterations & 1) * nk * 8;
        const double* pos = base + 2 * (size_t)nk * 8;
        const int* rows = reinterpret_cast<const int*>(pos + (size_t)L.pf_nl * 4);
        for (int r = 0; r < nk; ++r) {
            if (kf_rows) kf_rows[r] = L.win_rows[r];
            if (kf_pose7)
                for (int j = 0; j < 7; ++j) kf_pose7[7 * r + j] = pose[8 * (size_t)r + j];
        }
        for (int i = 0; i < n; ++i) {
            if (lm_rows) lm_rows[i] = rows[i];
            if (lm_pos3)
                for (int j = 0; j < 3; ++j) lm_pos3[3 * (size_t)i + j] = pos[4 * (size_t)i + j];
        }
        return VX_OK;
    }
    VX_HIP(c, hipSetDevice(c->device));
    // one pinned staging block (poses, positions, landmark rows), one synchronisation
    const size_t pose_b = (size_t)nk * 64, pos_b = (size_t)n * 32, rows_b = (size_t)n * 4;
    VX_HIP(c, L.res_host.ensure(pose_b + pos_b + rows_b + 64, true));
    double* pose = reinterpret_cast<double*>(L.res_host.p);
    double* pos = pose + (size_t)nk * 8;
    int* rows = reinterpret_cast<int*>(pos + (size_t)n * 4);
    const double* dpose;
    const double* dpos;
    if (L.fallback) {
        vx_ba_plan* p = L.fallback;
        dpose = p->kf_pose.as<double>() + (size_t)(L.iterations & 1) * nk * 8;
        dpos = p->lm_pos.as<double>();
        std::copy(p->lm_map_idx.begin(), p->lm_map_idx.begin() + n, rows);
    } else {
        dpose = L.kf_pose.as<double>() + (size_t)(L.iterations & 1) * nk * 8;
        dpos = L.lm_pos.as<double>();
        if (n) VX_HIP(c, hipMemcpyAsync(rows, L.inv.p, rows_b, hipMemcpyDeviceToHost, c->stream));
    }
    VX_HIP(c, hipMemcpyAsync(pose, dpose, pose_b, hipMemcpyDeviceToHost, c->stream));
    if (n) VX_HIP(c, hipMemcpyAsync(pos, dpos, pos_b, hipMemcpyDeviceToHost, c->stream));
    VX_HIP(c, hipStreamSynchronize(c->stream));
    for (int r = 0; r < nk; ++r) {
        if (kf_rows) kf_rows[r] = L.win_rows[r];
        if (kf_pose7)
            for (int j = 0; j < 7; ++j) kf_pose7[7 * r + j] = pose[8 * (size_t)r + j];
    }
    for (int i = 0; i < n; ++i) {
        if (lm_rows) lm_rows[i] = rows[i];
        if (lm_pos3)
            for (int j = 0; j < 3; ++j) lm_pos3[3 * (size_t)i + j] = pos[4 * (size_t)i + j];
    }
    return VX_OK;
}

}  // extern "C"
