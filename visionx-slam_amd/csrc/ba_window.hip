// ba_window.hip — LocalBA window / landmark set / CSR build on the device.
//
// The host build of a vx_ba_plan (ba.hip, build_plan) restates local_ba.cpp:42-108 and the
// per-observation checks of :126-138 and :186-204 with hash maps over the snapshot: 7.4 ms at C3,
// 24 ms at C4 on one core — two orders of magnitude above the GPU frame.  Here the host only
// sorts the keyframe ids (SelectKeyFrames) and gathers the window keyframes' feature ranges; the
// landmark join, the optimised-landmark filter, the slot assignment and both CSRs are device
// kernels over the snapshot:
//   k_ht_insert    landmark id -> map index, open-addressing hash table (ids are unique)
//   k_feat_scan    per window feature: its landmark (hash probe), referenced-by-window mark,
//                  pose-stage validity (has_landmark, !is_outlier, exists, !bad, owned, camera)
//   k_lm_flags     per landmark: optimised = referenced && !bad && total observations >= min,
//                  owned by this shard (splitmix64(id) mod N)
//   (scan)         optimised owned landmarks -> slots 0.. in map-index order (std::sort order)
//   k_first_occ    first pose observation of each non-optimised landmark (atomicMin)
//   (scan)         those landmarks -> slots n_opt.. in first-occurrence order (the host build
//                  numbers them as its keyframe-major pose scan meets them)
//   (scan)         pose-stage CSR positions; k_pose_fill writes (uv, slot) and kf_obs_ptr
//   k_lobs_count / (scan) / k_lobs_fill   landmark-stage CSR: each optimised landmark's
//                  observations whose keyframe is in the window (binary search over the sorted
//                  window ids), with a camera, a feature index in range and a feature that is a
//                  non-outlier observation of this landmark — in observation order
//   k_lm_gather    initial positions by slot
// The result is the same plan, array for array, as the host build (tests compare the runs
// bitwise).  Scans are rocPRIM's device exclusive scan.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include <rocprim/rocprim.hpp>

#include "vx_internal.hpp"
#include "ba_common.hpp"
#include "ba_plan.hpp"
#include "dmap.hpp"

namespace vx {
namespace {

constexpr int kT = 256;
constexpr uint64_t kEmpty = ~0ull;

__device__ __forceinline__ uint64_t mix(uint64_t x) {  // splitmix64 (the shard hash as well)
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

struct WinArgs {
    // window features (keyframe rows in ascending id order, features concatenated)
    int nk, nf;
    const int* wptr;          // nk + 1
    const uint64_t* wlm;      // nf
    const uint8_t* wfl;       // nf
    const uint8_t* cam;       // nk
    const uint64_t* wid;      // nk: window keyframe ids, ascending
    // snapshot landmarks
    int nl;
    const uint64_t* lid;
    const uint8_t* bad;
    const int64_t* optr;      // nl + 1
    const uint64_t* okf;
    const uint64_t* ofi;
    // hash table
    uint64_t* hkey;
    int* hval;
    unsigned hmask;
    int min_point, shard_rank, shard_count;
    // per feature / per landmark scratch
    int* f_lm;                // landmark map index or -1
    int* f_pv;                // pose-stage valid (0/1)
    int* f_first;             // first pose observation of a non-optimised landmark (0/1)
    int* l_ref;
    int* l_opt;               // optimised and owned (0/1)
    int* l_slot;
    int* l_first;             // first pose observation index (or INT_MAX)
    unsigned* counts;         // [0] optimised landmarks over all shards
};

__device__ __forceinline__ int ht_find(const WinArgs& a, uint64_t key) {
    unsigned h = (unsigned)mix(key) & a.hmask;
    for (unsigned probe = 0; probe <= a.hmask; ++probe) {
        const uint64_t k = a.hkey[h];
        if (k == key) return a.hval[h];
        if (k == kEmpty) return -1;
        h = (h + 1) & a.hmask;
    }
    return -1;
}

__global__ __launch_bounds__(kT) void k_ht_insert(WinArgs a) {
    const int l = blockIdx.x * kT + threadIdx.x;
    if (l >= a.nl || a.bad[l] == kLmRemoved) return;  // Map::RemoveLandmark: GetLandmark() == nullptr
    const uint64_t key = a.lid[l];
    unsigned h = (unsigned)mix(key) & a.hmask;
    for (;;) {
        const unsigned long long prev = atomicCAS(reinterpret_cast<unsigned long long*>(&a.hkey[h]),
                                                  (unsigned long long)kEmpty, (unsigned long long)key);
        if (prev == kEmpty || prev == key) {
            a.hval[h] = l;
            return;
        }
        h = (h + 1) & a.hmask;
    }
}

__device__ __forceinline__ int row_of_feature(const WinArgs& a, int f) {
    int lo = 0, hi = a.nk - 1;  // last row with wptr[row] <= f
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (a.wptr[mid] <= f) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

__device__ __forceinline__ bool owned(const WinArgs& a, uint64_t id) {
    return a.shard_count <= 1 || (int)(mix(id) % (uint64_t)a.shard_count) == a.shard_rank;
}

__global__ __launch_bounds__(kT) void k_feat_scan(WinArgs a) {
    const int f = blockIdx.x * kT + threadIdx.x;
    if (f >= a.nf) return;
    const uint8_t fl = a.wfl[f];
    int l = -1;
    if (fl & 1) {
        l = ht_find(a, a.wlm[f]);
        if (l >= 0) a.l_ref[l] = 1;  // the window references it (local_ba.cpp:83-92)
    }
    a.f_lm[f] = l;
    const int r = row_of_feature(a, f);
    // pose-stage observation (local_ba.cpp:126-138)
    a.f_pv[f] = (a.cam[r] && (fl & 1) && !(fl & 2) && l >= 0 && !a.bad[l] && owned(a, a.lid[l])) ? 1 : 0;
}

__global__ __launch_bounds__(kT) void k_lm_flags(WinArgs a) {
    const int l = blockIdx.x * kT + threadIdx.x;
    if (l >= a.nl) return;
    const bool opt = a.l_ref[l] && !a.bad[l] && (a.optr[l + 1] - a.optr[l]) >= (int64_t)a.min_point;
    if (opt) atomicAdd(&a.counts[0], 1u);
    a.l_opt[l] = (opt && owned(a, a.lid[l])) ? 1 : 0;
    a.l_first[l] = 0x7fffffff;
}

__global__ __launch_bounds__(kT) void k_opt_slots(WinArgs a, const int* scan, int* inv) {
    const int l = blockIdx.x * kT + threadIdx.x;
    if (l >= a.nl) return;
    a.l_slot[l] = -1;
    if (a.l_opt[l]) {
        a.l_slot[l] = scan[l];
        inv[scan[l]] = l;
    }
}

__global__ __launch_bounds__(kT) void k_first_occ(WinArgs a) {
    const int f = blockIdx.x * kT + threadIdx.x;
    if (f >= a.nf || !a.f_pv[f]) return;
    const int l = a.f_lm[f];
    if (!a.l_opt[l]) atomicMin(&a.l_first[l], f);
}

__global__ __launch_bounds__(kT) void k_is_first(WinArgs a) {
    const int f = blockIdx.x * kT + threadIdx.x;
    if (f >= a.nf) return;
    const int l = a.f_lm[f];
    a.f_first[f] = (a.f_pv[f] && !a.l_opt[l] && a.l_first[l] == f) ? 1 : 0;
}

// (n_opt: the optimised-landmark scan's total, read on the device; thread 0 also records it and
// the fixed-landmark count for the build's single read-back: counts[4], counts[5])
__global__ __launch_bounds__(kT) void k_fixed_slots(WinArgs a, const int* scan, const int* n_opt_dev, int* inv) {
    const int f = blockIdx.x * kT + threadIdx.x;
    const int n_opt = *n_opt_dev;
    if (f == 0) {
        a.counts[4] = (unsigned)n_opt;
        a.counts[5] = (unsigned)scan[a.nf];
    }
    if (f >= a.nf || !a.f_first[f]) return;
    const int l = a.f_lm[f];
    a.l_slot[l] = n_opt + scan[f];
    inv[n_opt + scan[f]] = l;
}

__global__ __launch_bounds__(kT) void k_pose_fill(WinArgs a, const int* pscan, const double* wuv, double2* puv,
                                                  int* plm, int* kf_obs_ptr) {
    const int f = blockIdx.x * kT + threadIdx.x;
    if (f < a.nf && a.f_pv[f]) {
        const int o = pscan[f];
        puv[o] = make_double2(wuv[2 * f], wuv[2 * f + 1]);
        plm[o] = a.l_slot[a.f_lm[f]];
    }
    if (f <= a.nk) kf_obs_ptr[f] = pscan[a.wptr[f]];  // (wptr[nk] == nf: the total)
    if (f == 0) a.counts[6] = (unsigned)pscan[a.nf];  // pose-stage observations, for the read-back
}

// landmark-stage observation check (local_ba.cpp:186-204); returns the window feature or -1
__device__ __forceinline__ int lobs_feature(const WinArgs& a, int l, int64_t o, int& row) {
    const uint64_t kid = a.okf[o];
    int lo = 0, hi = a.nk - 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (a.wid[mid] < kid) lo = mid + 1;
        else hi = mid;
    }
    if (a.wid[lo] != kid) return -1;
    row = lo;
    if (!a.cam[lo]) return -1;
    const uint64_t fi = a.ofi[o];
    const int nfk = a.wptr[lo + 1] - a.wptr[lo];
    if (fi >= (uint64_t)nfk) return -1;
    const int f = a.wptr[lo] + (int)fi;
    const uint8_t fl = a.wfl[f];
    if (!(fl & 1) || (fl & 2) || a.wlm[f] != a.lid[l]) return -1;
    return f;
}

// One wave per slot, its lanes over the landmark's observations (each lane's check is a chain of
// dependent loads: a thread per slot walking them one after the other took 13 us at C3).
// Over the slots [0, cap) (cap: the map's landmark count, an upper bound of n_opt, which is read
// on the device): slots >= n_opt count 0, so the scan over cap + 1 elements agrees with one over
// n_opt + 1 on its first n_opt + 1 outputs
__global__ __launch_bounds__(kT) void k_lobs_count(WinArgs a, const int* inv, const int* n_opt_dev, int cap, int* cnt) {
    const int s = (int)((blockIdx.x * (unsigned)kT + threadIdx.x) >> 6), lane = threadIdx.x & 63;
    if (s == 0 && lane == 0) cnt[cap] = 0;  // (the scan's extra element)
    if (s >= cap) return;
    if (s >= *n_opt_dev) {
        if (lane == 0) cnt[s] = 0;
        return;
    }
    const int l = inv[s];
    const int64_t o0 = a.optr[l], o1 = a.optr[l + 1];
    int c = 0;
    for (int64_t base = o0; base < o1; base += 64) {
        const int64_t o = base + lane;
        int row;
        c += __popcll(__ballot(o < o1 && lobs_feature(a, l, o, row) >= 0));
    }
    if (lane == 0) cnt[s] = c;
}

// the build's scratch state in one launch: empty hash slots, zeroed per-landmark / per-feature
// flags (the scans' extra elements included) and counters
__global__ __launch_bounds__(kT) void k_build_init(uint64_t* hkey, size_t hcap, int* l_ref, int* l_opt, size_t lN,
                                                   int* f_pv, int* f_first, size_t fN, unsigned* counts) {
    const size_t i = (size_t)blockIdx.x * kT + threadIdx.x;
    if (i < hcap) hkey[i] = ~0ull;
    if (i < lN) {
        l_ref[i] = 0;
        l_opt[i] = 0;
    }
    if (i < fN) {
        f_pv[i] = 0;
        f_first[i] = 0;
    }
    if (i < 16) counts[i] = 0;
}

// one wave per slot as in k_lobs_count; the valid observations keep their CSR order (ballot ranks)
__global__ __launch_bounds__(kT) void k_lobs_fill(WinArgs a, const int* inv, int n_opt, const int* lptr,
                                                  const double* wuv, int* lkf, int* llm, double2* luv) {
    const int s = (int)((blockIdx.x * (unsigned)kT + threadIdx.x) >> 6), lane = threadIdx.x & 63;
    if (s >= n_opt) return;
    const int l = inv[s];
    const int64_t o0 = a.optr[l], o1 = a.optr[l + 1];
    int w = lptr[s];
    for (int64_t base = o0; base < o1; base += 64) {
        const int64_t o = base + lane;
        int row = 0, f = -1;
        if (o < o1) f = lobs_feature(a, l, o, row);
        const unsigned long long m = __ballot(f >= 0);
        if (f >= 0) {
            const int at = w + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
            lkf[at] = row;
            llm[at] = s;
            luv[at] = make_double2(wuv[2 * f], wuv[2 * f + 1]);
        }
        w += __popcll(m);
    }
}

__global__ __launch_bounds__(kT) void k_lm_gather(const int* inv, int n, const double* pos, double* lm0) {
    const int s = blockIdx.x * kT + threadIdx.x;
    if (s >= n) return;
    const int l = inv[s];
    lm0[4 * s] = pos[3 * l];
    lm0[4 * s + 1] = pos[3 * l + 1];
    lm0[4 * s + 2] = pos[3 * l + 2];
    lm0[4 * s + 3] = 0.0;
}

inline unsigned grid(long long n) { return (unsigned)std::max(1ll, (n + kT - 1) / kT); }

template <class T>
int up(vx_ctx* c, DevBuf& d, const T* h, size_t n) {
    VX_HIP(c, d.ensure(std::max<size_t>(1, n) * sizeof(T)));
    if (n) VX_HIP(c, hipMemcpyAsync(d.p, h, n * sizeof(T), hipMemcpyHostToDevice, c->stream));
    return VX_OK;
}

// exclusive scan of n ints (n + 1 outputs: the total at [n])
int scan(vx_ctx* c, DevBuf& tmp, const int* in, int* out, int n) {
    size_t bytes = 0;
    VX_HIP(c, rocprim::exclusive_scan(nullptr, bytes, in, out, 0, (size_t)n + 1, rocprim::plus<int>(), c->stream));
    VX_HIP(c, tmp.ensure(std::max<size_t>(bytes, 16)));
    VX_HIP(c, rocprim::exclusive_scan(tmp.p, bytes, in, out, 0, (size_t)n + 1, rocprim::plus<int>(), c->stream));
    return VX_OK;
}

}  // namespace

// device inputs of the build: the window's features (keyframe rows in ascending id order) and the
// map's landmarks with their landmark-major observation CSR
struct BuildInputs {
    int nk, nf, nl;
    const int* wptr;
    const uint64_t* wlm;
    const uint8_t* wfl;
    const uint8_t* cam;
    const uint64_t* wid;
    const double* wuv;
    const uint64_t* lid;
    const uint8_t* bad;
    const int64_t* optr;
    const uint64_t* okf;
    const uint64_t* ofi;
    const double* pos;
};

namespace {
int build_core(vx_ctx* c, const BuildInputs& in, const std::vector<int>& win, const std::vector<int>& kf_flags,
               vx_ba_plan* p);

// SelectKeyFrames (local_ba.cpp:42-62) over keyframe ids: newest `window` with id <= max_id, in
// ascending id order (as indices into `ids`); `alive` (may be null) masks out removed keyframes
std::vector<int> select_ids(const uint64_t* ids, int n, uint64_t ref_kf_id, int has_ref, int window_size,
                            const uint8_t* alive = nullptr) {
    std::vector<int> order;
    order.reserve(n);
    for (int i = 0; i < n; ++i)
        if (!alive || alive[i]) order.push_back(i);
    if (order.empty()) return {};
    std::sort(order.begin(), order.end(), [&](int x, int y) { return ids[x] < ids[y]; });
    n = (int)order.size();
    const int window = std::max(1, window_size);
    const uint64_t max_id = has_ref ? ref_kf_id : ids[order.back()];
    std::vector<int> win;
    for (int i = n - 1; i >= 0 && (int)win.size() < window; --i)
        if (ids[order[i]] <= max_id) win.push_back(order[i]);
    std::reverse(win.begin(), win.end());
    return win;
}
}  // namespace

int build_plan_device(vx_ctx* c, const vx_map_view* m, uint64_t ref_kf_id, int has_ref, vx_ba_plan* p) {
    const vx_ba_options& o = p->opt;
    p->status = 1;
    p->n_window_kf = 0;
    p->n_landmarks_global = 0;
    if (!m || m->n_kf <= 0) return VX_OK;
    // ---- SelectKeyFrames (local_ba.cpp:42-62): host, over the keyframe ids only
    const std::vector<int> win = select_ids(m->kf_id, m->n_kf, ref_kf_id, has_ref, o.window_size);
    const int nk = (int)win.size();
    p->n_window_kf = nk;
    if (nk < 2) return VX_OK;
    const PlanClock clk;
    // ---- window feature gather + keyframe tables (host: contiguous copies per keyframe).  A window
    // of consecutive view rows (a snapshot of the window alone: visionx::LocalBA::Flatten) is uploaded
    // straight from the view's arrays instead (page-locked there: one DMA each)
    std::vector<int> wptr(nk + 1, 0);
    for (int r = 0; r < nk; ++r) wptr[r + 1] = wptr[r] + (int)(m->kf_feat_ptr[win[r] + 1] - m->kf_feat_ptr[win[r]]);
    const int nf = wptr[nk];
    bool consecutive = true;
    for (int r = 1; r < nk; ++r) consecutive = consecutive && win[r] == win[0] + r;
    const int64_t f_first = m->kf_feat_ptr[win[0]];
    std::vector<double> wuv;
    std::vector<uint64_t> wlm, wid(nk);
    std::vector<uint8_t> wfl, cam(nk);
    if (!consecutive) {
        wuv.resize((size_t)nf * 2);
        wlm.resize(nf);
        wfl.resize(nf);
    }
    std::vector<double> pose0((size_t)nk * 8, 0.0), intr((size_t)nk * 4, 0.0);
    std::vector<int> kf_flags(nk);
    int64_t mx = 0;
    for (int r = 0; r < nk; ++r) {
        const int k = win[r];
        const int64_t f0 = m->kf_feat_ptr[k], n = m->kf_feat_ptr[k + 1] - f0;
        if (!consecutive) {
            std::memcpy(&wuv[2 * (size_t)wptr[r]], m->feat_uv + 2 * f0, (size_t)n * 2 * sizeof(double));
            std::memcpy(&wlm[wptr[r]], m->feat_lm_id + f0, (size_t)n * sizeof(uint64_t));
            std::memcpy(&wfl[wptr[r]], m->feat_flags + f0, (size_t)n);
        }
        wid[r] = m->kf_id[k];
        cam[r] = m->kf_has_cam[k] ? 1 : 0;
        kf_flags[r] = cam[r];
        for (int j = 0; j < 7; ++j) pose0[8 * r + j] = m->kf_pose[7 * k + j];
        for (int j = 0; j < 4; ++j) intr[4 * r + j] = m->kf_intr[4 * k + j];
        if (cam[r]) {
            int64_t cnt = 0;
            const uint8_t* fl = m->feat_flags + f0;
            for (int64_t f = 0; f < n; ++f) cnt += fl[f] & 1;
            mx = std::max(mx, cnt);
        }
    }
    p->n_split = ba_split(mx, p->shard_count);
    const int nl = m->n_lm;
    const int64_t nobs = nl > 0 ? m->lm_obs_ptr[nl] : 0;
    clk.mark("device: window gathered");
    VX_HIP(c, hipSetDevice(c->device));
    vx_ctx::PlanScratch& B = c->plan_scratch;  // reused across this context's plan builds
    int rc;
    // the keyframe-sized tables through one pinned block: ids, initial poses, intrinsics, feature
    // offsets, camera flags
    const size_t o_wid = 0, o_pose = o_wid + 8 * (size_t)nk, o_intr = o_pose + 64 * (size_t)nk,
                 o_wptr = o_intr + 32 * (size_t)nk, o_cam = o_wptr + 4 * ((size_t)nk + 2), o_end = o_cam + (size_t)nk + 8;
    VX_HIP(c, B.win_host.ensure(o_end, true));
    VX_HIP(c, B.win.ensure(o_end));
    {
        uint8_t* H = static_cast<uint8_t*>(B.win_host.p);
        std::memcpy(H + o_wid, wid.data(), 8 * (size_t)nk);
        std::memcpy(H + o_pose, pose0.data(), 64 * (size_t)nk);
        std::memcpy(H + o_intr, intr.data(), 32 * (size_t)nk);
        std::memcpy(H + o_wptr, wptr.data(), 4 * ((size_t)nk + 1));
        std::memcpy(H + o_cam, cam.data(), (size_t)nk);
    }
    VX_HIP(c, hipMemcpyAsync(B.win.p, B.win_host.p, o_end, hipMemcpyHostToDevice, c->stream));
    const uint8_t* WD = B.win.as<uint8_t>();
    VX_HIP(c, p->kf_pose0.ensure(64 * (size_t)nk));
    VX_HIP(c, p->kf_intr.ensure(32 * (size_t)nk));
    VX_HIP(c, hipMemcpyAsync(p->kf_pose0.p, WD + o_pose, 64 * (size_t)nk, hipMemcpyDeviceToDevice, c->stream));
    VX_HIP(c, hipMemcpyAsync(p->kf_intr.p, WD + o_intr, 32 * (size_t)nk, hipMemcpyDeviceToDevice, c->stream));
    if ((rc = up(c, B.wlm, consecutive ? m->feat_lm_id + f_first : wlm.data(), (size_t)nf))) return rc;
    if ((rc = up(c, B.wfl, consecutive ? m->feat_flags + f_first : wfl.data(), (size_t)nf))) return rc;
    if ((rc = up(c, B.wuv, consecutive ? m->feat_uv + 2 * f_first : wuv.data(), 2 * (size_t)nf))) return rc;
    if ((rc = up(c, B.lid, m->lm_id, (size_t)nl))) return rc;
    if ((rc = up(c, B.bad, m->lm_bad, (size_t)nl))) return rc;
    if ((rc = up(c, B.optr, m->lm_obs_ptr, (size_t)nl + 1))) return rc;
    if ((rc = up(c, B.okf, m->obs_kf_id, (size_t)nobs))) return rc;
    if ((rc = up(c, B.ofi, m->obs_feat_idx, (size_t)nobs))) return rc;
    if ((rc = up(c, B.pos, m->lm_pos, (size_t)nl * 3))) return rc;
    clk.mark("device: uploads queued");
    BuildInputs in{nk, nf, nl, reinterpret_cast<const int*>(WD + o_wptr), B.wlm.as<uint64_t>(), B.wfl.as<uint8_t>(),
                   WD + o_cam, reinterpret_cast<const uint64_t*>(WD + o_wid), B.wuv.as<double>(), B.lid.as<uint64_t>(), B.bad.as<uint8_t>(),
                   B.optr.as<int64_t>(), B.okf.as<uint64_t>(), B.ofi.as<uint64_t>(), B.pos.as<double>()};
    rc = build_core(c, in, win, kf_flags, p);
    VX_HIP(c, hipStreamSynchronize(c->stream));  // the host vectors above must outlive their async copies
    return rc;
}

namespace {
int build_core(vx_ctx* c, const BuildInputs& in, const std::vector<int>& win, const std::vector<int>& kf_flags,
               vx_ba_plan* p) {
    const vx_ba_options& o = p->opt;
    const int nk = in.nk, nf = in.nf, nl = in.nl;
    vx_ctx::PlanScratch& B = c->plan_scratch;
    const PlanClock clk;
    int rc;
    unsigned hcap = 1024;
    while (hcap < 2u * (unsigned)std::max(nl, 1)) hcap <<= 1;

    VX_HIP(c, B.hkey.ensure((size_t)hcap * 8));
    VX_HIP(c, B.hval.ensure((size_t)hcap * 4));
    const size_t fN = (size_t)std::max(nf, 1) + 1, lN = (size_t)std::max(nl, 1) + 1;
    for (DevBuf* d : {&B.f_lm, &B.f_pv, &B.f_first, &B.scan_b}) VX_HIP(c, d->ensure(fN * 4));
    for (DevBuf* d : {&B.l_ref, &B.l_opt, &B.l_slot, &B.l_first, &B.scan_a, &B.inv, &B.cnt, &B.scan_c})
        VX_HIP(c, d->ensure(lN * 4));
    VX_HIP(c, B.counts.ensure(64));
    hipLaunchKernelGGL(k_build_init, dim3(grid((int)std::max<size_t>(std::max<size_t>(hcap, lN), fN))), dim3(kT), 0,
                       c->stream, B.hkey.as<uint64_t>(), (size_t)hcap, B.l_ref.as<int>(), B.l_opt.as<int>(), lN,
                       B.f_pv.as<int>(), B.f_first.as<int>(), fN, B.counts.as<unsigned>());  // ([nf] = 0 for the scans)

    WinArgs a{};
    a.nk = nk;
    a.nf = nf;
    a.wptr = in.wptr;
    a.wlm = in.wlm;
    a.wfl = in.wfl;
    a.cam = in.cam;
    a.wid = in.wid;
    a.nl = nl;
    a.lid = in.lid;
    a.bad = in.bad;
    a.optr = in.optr;
    a.okf = in.okf;
    a.ofi = in.ofi;
    a.hkey = B.hkey.as<uint64_t>();
    a.hval = B.hval.as<int>();
    a.hmask = hcap - 1;
    a.min_point = o.min_point_observations;
    a.shard_rank = p->shard_rank;
    a.shard_count = p->shard_count;
    a.f_lm = B.f_lm.as<int>();
    a.f_pv = B.f_pv.as<int>();
    a.f_first = B.f_first.as<int>();
    a.l_ref = B.l_ref.as<int>();
    a.l_opt = B.l_opt.as<int>();
    a.l_slot = B.l_slot.as<int>();
    a.l_first = B.l_first.as<int>();
    a.counts = B.counts.as<unsigned>();
    hipStream_t s = c->stream;
    hipLaunchKernelGGL(k_ht_insert, dim3(grid(nl)), dim3(kT), 0, s, a);
    hipLaunchKernelGGL(k_feat_scan, dim3(grid(nf)), dim3(kT), 0, s, a);
    hipLaunchKernelGGL(k_lm_flags, dim3(grid(nl)), dim3(kT), 0, s, a);
    VX_LAUNCH_CHECK(c, "plan build kernels");
    // optimised owned landmarks -> slots 0.. (map-index order)
    int* opt_scan = B.scan_a.as<int>();
    if ((rc = scan(c, B.tmp, a.l_opt, opt_scan, nl))) return rc;
    int* inv = B.inv.as<int>();
    hipLaunchKernelGGL(k_opt_slots, dim3(grid(nl)), dim3(kT), 0, s, a, opt_scan, inv);
    hipLaunchKernelGGL(k_first_occ, dim3(grid(nf)), dim3(kT), 0, s, a);
    hipLaunchKernelGGL(k_is_first, dim3(grid(nf)), dim3(kT), 0, s, a);
    VX_LAUNCH_CHECK(c, "plan slot kernels");
    int* first_scan = B.scan_b.as<int>();
    if ((rc = scan(c, B.tmp, a.f_first, first_scan, nf))) return rc;
    // No read-back here: the counts stay on the device (n_opt = opt_scan[nl]) and every size below
    // is bounded by the map (n_opt, n_lm <= nl): one synchronisation for the whole core build.
    const int* n_opt_dev = opt_scan + nl;
    hipLaunchKernelGGL(k_fixed_slots, dim3(grid(nf)), dim3(kT), 0, s, a, (const int*)first_scan, n_opt_dev, inv);
    // pose-stage CSR
    int* pscan = B.scan_b.as<int>();  // (first_scan consumed by k_fixed_slots above, stream-ordered)
    if ((rc = scan(c, B.tmp, a.f_pv, pscan, nf))) return rc;
    // (sized for every window feature: the count arrives with the read-back)
    VX_HIP(c, p->pobs_uv.ensure((size_t)std::max(nf, 1) * sizeof(double2)));
    VX_HIP(c, p->pobs_lm.ensure((size_t)std::max(nf, 1) * 4));
    VX_HIP(c, p->kf_obs_ptr.ensure((size_t)(nk + 1) * 4));
    hipLaunchKernelGGL(k_pose_fill, dim3(grid(std::max(nf, nk + 1))), dim3(kT), 0, s, a, pscan,
                       in.wuv, p->pobs_uv.as<double2>(), p->pobs_lm.as<int>(), p->kf_obs_ptr.as<int>());
    // landmark-stage CSR over all nl slots (those past n_opt count 0)
    int* cnt = B.cnt.as<int>();
    hipLaunchKernelGGL(k_lobs_count, dim3(grid(64ll * std::max(nl, 1))), dim3(kT), 0, s, a, inv, n_opt_dev, nl, cnt);
    VX_LAUNCH_CHECK(c, "plan CSR kernels");
    VX_HIP(c, p->lobs_ptr.ensure((size_t)(nl + 1) * 4));
    if ((rc = scan(c, B.tmp, cnt, p->lobs_ptr.as<int>(), nl))) return rc;
    // the one read-back: counts (global optimised landmarks, n_opt, n_fixed, pose-stage
    // observations), the landmark-stage pointers, slot -> map index (pinned)
    VX_HIP(c, B.rb_host.ensure((size_t)(8 + 2 * (size_t)nl + 1) * 4, true));
    int* RB = static_cast<int*>(B.rb_host.p);
    VX_HIP(c, hipMemcpyAsync(RB, B.counts.p, 8 * sizeof(int), hipMemcpyDeviceToHost, s));
    VX_HIP(c, hipMemcpyAsync(RB + 8, p->lobs_ptr.p, (size_t)(nl + 1) * 4, hipMemcpyDeviceToHost, s));
    if (nl) VX_HIP(c, hipMemcpyAsync(RB + 8 + nl + 1, inv, (size_t)nl * 4, hipMemcpyDeviceToHost, s));
    clk.mark("core: counts + CSR requested");
    VX_HIP(c, hipStreamSynchronize(s));
    clk.mark("core: counts + CSR back");
    p->n_landmarks_global = RB[0];
    if (RB[0] == 0) return VX_OK;  // no optimised landmark anywhere (local_ba.cpp:106-108)
    p->status = 0;
    p->n_kf = nk;
    p->kf_map_idx = win;
    const int n_opt = RB[4], n_lm = RB[4] + RB[5];
    p->n_opt = n_opt;
    p->n_lm = n_lm;
    p->n_pose_obs = RB[6];
    const std::vector<int> lptr(RB + 8, RB + 8 + n_opt + 1);
    const int* inv_h = RB + 8 + nl + 1;
    const int n_lobs = lptr[n_opt];
    p->n_lm_obs = n_lobs;
    p->lm_map_idx.assign(inv_h, inv_h + n_lm);
    VX_HIP(c, p->lobs_kf.ensure((size_t)std::max(n_lobs, 1) * 4));
    VX_HIP(c, p->lobs_lm.ensure((size_t)std::max(n_lobs, 1) * 4));
    VX_HIP(c, p->lobs_uv.ensure((size_t)std::max(n_lobs, 1) * sizeof(double2)));
    hipLaunchKernelGGL(k_lobs_fill, dim3(grid(64ll * n_opt)), dim3(kT), 0, s, a, inv, n_opt, p->lobs_ptr.as<int>(),
                       in.wuv, p->lobs_kf.as<int>(), p->lobs_lm.as<int>(),
                       p->lobs_uv.as<double2>());
    VX_HIP(c, p->lm_pos0.ensure((size_t)std::max(n_lm, 1) * 4 * sizeof(double)));
    hipLaunchKernelGGL(k_lm_gather, dim3(grid(n_lm)), dim3(kT), 0, s, (const int*)inv, n_lm,
                       in.pos, p->lm_pos0.as<double>());
    VX_LAUNCH_CHECK(c, "plan fill kernels");
    const std::vector<int> blk = pack_lm_blocks(lptr, n_opt, &p->max_lm_obs);
    p->n_lm_blocks = (int)blk.size() / 2 - 1;
    // both tables through a pinned block (no synchronisation here: the fused build below reads back
    // and synchronises before the next plan build can reuse the block, and a plan without the fused
    // layout synchronises at the end)
    const size_t nblk = blk.size(), nflg = kf_flags.size();
    VX_HIP(c, B.up_host.ensure((nblk + nflg) * 4, true));
    int* UP = static_cast<int*>(B.up_host.p);
    std::copy(blk.begin(), blk.end(), UP);
    std::copy(kf_flags.begin(), kf_flags.end(), UP + nblk);
    VX_HIP(c, p->lm_blk.ensure(nblk * 4));
    VX_HIP(c, p->kf_flags.ensure(std::max<size_t>(nflg, 1) * 4));
    VX_HIP(c, hipMemcpyAsync(p->lm_blk.p, UP, nblk * 4, hipMemcpyHostToDevice, s));
    if (nflg) VX_HIP(c, hipMemcpyAsync(p->kf_flags.p, UP + nblk, nflg * 4, hipMemcpyHostToDevice, s));
    if ((rc = alloc_run_buffers(c, p))) return rc;
    clk.mark("core: fill launched");
    // the fused layout, on the device from the CSRs just built (every plan, sharded ones included)
    if ((rc = build_fused_device(c, p))) return rc;
    clk.mark("core: fused layout built");
    if (!p->fused) VX_HIP(c, hipStreamSynchronize(s));  // (the pinned block above)
    return VX_OK;
}
}  // namespace



// ---------------------------------------------------------------- plan from the resident map
namespace {
// window features out of the resident feature arrays: output feature f of window row r (found by
// binary search over wptr) is resident feature src[r] + (f - wptr[r])
__global__ __launch_bounds__(kT) void k_gather_window(int nk, int nf, const int* wptr, const int64_t* src,
                                                      const double* uv, const uint64_t* lm, const uint8_t* fl,
                                                      double* wuv, uint64_t* wlm, uint8_t* wfl) {
    const int f = blockIdx.x * kT + threadIdx.x;
    if (f >= nf) return;
    int lo = 0, hi = nk;  // largest r with wptr[r] <= f
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (wptr[mid] <= f) lo = mid;
        else hi = mid;
    }
    const int64_t g = src[lo] + (f - wptr[lo]);
    wuv[2 * f] = uv[2 * g];
    wuv[2 * f + 1] = uv[2 * g + 1];
    wlm[f] = lm[g];
    wfl[f] = fl[g];
}
// window keyframes' poses (8-double rows, last 0) and intrinsics
// the finished plan's slot -> map index tables for vx_ba_plan_apply_dmap, one launch
__global__ void k_map_tables(const int* inv, int n_lm, const int* win, int nk, int* lm_map, int* kf_map) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n_lm) lm_map[i] = inv[i];
    if (i < nk) kf_map[i] = win[i];
}
__global__ void k_gather_kf(int nk, const int* win, const double* pose, const double* intr, double* pose0,
                            double* intr0) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nk) return;
    const int k = win[r];
    for (int j = 0; j < 7; ++j) pose0[8 * r + j] = pose[7 * k + j];
    pose0[8 * r + 7] = 0.0;
    for (int j = 0; j < 4; ++j) intr0[4 * r + j] = intr[4 * k + j];
}
}  // namespace

std::vector<int> dmap_select_window(const vx_dmap* m, uint64_t ref_kf_id, int has_ref, int window_size) {
    return select_ids(m->kf_id.data(), (int)m->kf_id.size(), ref_kf_id, has_ref, window_size, m->kf_alive.data());
}

int build_plan_dmap(vx_ctx* c, vx_dmap* m, uint64_t ref_kf_id, int has_ref, vx_ba_plan* p) {
    const vx_ba_options& o = p->opt;
    p->status = 1;
    p->n_window_kf = 0;
    p->n_landmarks_global = 0;
    const int n_kf = (int)m->kf_id.size();
    if (n_kf <= 0) return VX_OK;
    const PlanClock clk;
    const std::vector<int> win = select_ids(m->kf_id.data(), n_kf, ref_kf_id, has_ref, o.window_size, m->kf_alive.data());
    const int nk = (int)win.size();
    p->n_window_kf = nk;
    if (nk < 2) return VX_OK;
    // host: the window's feature ranges and keyframe tables (keyframe-sized, from the mirrors)
    std::vector<int> wptr(nk + 1, 0), kf_flags(nk);
    std::vector<int64_t> src(nk);
    std::vector<uint64_t> wid(nk);
    std::vector<uint8_t> cam(nk);
    int64_t mx = 0;
    for (int r = 0; r < nk; ++r) {
        const int k = win[r];
        src[r] = m->kf_feat_ptr[k];
        wptr[r + 1] = wptr[r] + (int)(m->kf_feat_ptr[k + 1] - m->kf_feat_ptr[k]);
        wid[r] = m->kf_id[k];
        cam[r] = m->kf_has_cam[k];
        kf_flags[r] = cam[r];
        if (cam[r]) mx = std::max<int64_t>(mx, m->kf_valid_cnt[k]);
    }
    p->n_split = ba_split(mx, p->shard_count);
    const int nf = wptr[nk];
    VX_HIP(c, hipSetDevice(c->device));
    vx_ctx::PlanScratch& B = c->plan_scratch;
    int rc;
    // the window's keyframe tables in one pinned block, one upload: source offsets (i64), ids
    // (u64), rows (i32, nk + 1), map indices (i32), camera flags (u8)
    const size_t o_src = 0, o_wid = o_src + 8 * (size_t)nk, o_wptr = o_wid + 8 * (size_t)nk,
                 o_win = o_wptr + 4 * ((size_t)nk + 2), o_cam = o_win + 4 * ((size_t)nk + 2),
                 o_end = o_cam + (size_t)nk + 8;
    VX_HIP(c, B.win_host.ensure(o_end, true));
    VX_HIP(c, B.win.ensure(o_end));
    {
        uint8_t* H = static_cast<uint8_t*>(B.win_host.p);
        std::memcpy(H + o_src, src.data(), 8 * (size_t)nk);
        std::memcpy(H + o_wid, wid.data(), 8 * (size_t)nk);
        std::memcpy(H + o_wptr, wptr.data(), 4 * ((size_t)nk + 1));
        for (int r = 0; r < nk; ++r) reinterpret_cast<int*>(H + o_win)[r] = win[r];
        std::memcpy(H + o_cam, cam.data(), (size_t)nk);
    }
    VX_HIP(c, hipMemcpyAsync(B.win.p, B.win_host.p, o_end, hipMemcpyHostToDevice, c->stream));
    uint8_t* WD = B.win.as<uint8_t>();
    const int64_t* d_src = reinterpret_cast<const int64_t*>(WD + o_src);
    const uint64_t* d_wid = reinterpret_cast<const uint64_t*>(WD + o_wid);
    const int* d_wptr = reinterpret_cast<const int*>(WD + o_wptr);
    const int* d_win = reinterpret_cast<const int*>(WD + o_win);
    const uint8_t* d_cam = WD + o_cam;
    VX_HIP(c, B.wlm.ensure((size_t)std::max(nf, 1) * 8));
    VX_HIP(c, B.wfl.ensure((size_t)std::max(nf, 1)));
    VX_HIP(c, B.wuv.ensure((size_t)std::max(nf, 1) * 16));
    hipLaunchKernelGGL(k_gather_window, dim3(grid(nf)), dim3(kT), 0, c->stream, nk, nf, d_wptr,
                       d_src, (const double*)m->feat_uv.as<double>(),
                       (const uint64_t*)m->feat_lm.as<uint64_t>(), (const uint8_t*)m->feat_fl.as<uint8_t>(),
                       B.wuv.as<double>(), B.wlm.as<uint64_t>(), B.wfl.as<uint8_t>());
    VX_LAUNCH_CHECK(c, "k_gather_window");
    VX_HIP(c, p->kf_pose0.ensure((size_t)nk * 8 * sizeof(double)));
    VX_HIP(c, p->kf_intr.ensure((size_t)nk * 4 * sizeof(double)));
    hipLaunchKernelGGL(k_gather_kf, dim3(grid(nk)), dim3(kT), 0, c->stream, nk, d_win,
                       (const double*)m->kf_pose.as<double>(), (const double*)m->kf_intr.as<double>(),
                       p->kf_pose0.as<double>(), p->kf_intr.as<double>());
    VX_LAUNCH_CHECK(c, "k_gather_kf");
    clk.mark("dmap: window gathered");
    if ((rc = dmap_build_csr(c, m))) return rc;
    clk.mark("dmap: CSR ready");
    const int nl = (int)m->n_lm;
    BuildInputs in{nk, nf, nl, d_wptr, B.wlm.as<uint64_t>(), B.wfl.as<uint8_t>(), d_cam,
                   d_wid, B.wuv.as<double>(), m->lm_id.as<uint64_t>(), m->lm_bad.as<uint8_t>(),
                   m->optr.as<int64_t>(), m->okf.as<uint64_t>(), m->ofi.as<uint64_t>(), m->lm_pos.as<double>()};
    rc = build_core(c, in, win, kf_flags, p);
    if (rc) {
        (void)hipStreamSynchronize(c->stream);
        return rc;
    }
    // device copies of the slot -> map index tables for vx_ba_plan_apply_dmap (the landmark one is
    // still on the device: build_core's slot -> map index array)
    if (p->status == 0) {
        VX_HIP(c, p->lm_map_dev.ensure((size_t)std::max(p->n_lm, 1) * 4));
        VX_HIP(c, p->kf_map_dev.ensure((size_t)std::max(nk, 1) * 4));
        hipLaunchKernelGGL(k_map_tables, dim3(grid(std::max(p->n_lm, nk))), dim3(kT), 0, c->stream,
                           (const int*)B.inv.as<int>(), p->n_lm, d_win, nk, p->lm_map_dev.as<int>(),
                           p->kf_map_dev.as<int>());
        VX_LAUNCH_CHECK(c, "k_map_tables");
    }
    clk.mark("dmap: tables queued");
    VX_HIP(c, hipStreamSynchronize(c->stream));
    clk.mark("dmap: done");
    return VX_OK;
}

}  // namespace vx
