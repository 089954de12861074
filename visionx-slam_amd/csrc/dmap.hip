// dmap.hip — the device-resident map (vx_dmap_*).
//
// The reference rebuilds LocalBA's input from visionx::Map on every keyframe
// (local_ba.cpp:42-108: std::map / unordered_map walks under mutexes), and a snapshot-based drop-in
// still ships the whole map over PCIe per plan.  Here the map lives on the device and is updated by
// the same events that change the reference's Map (Map::InsertKeyFrame, Map::InsertLandmark,
// Landmark::AddObservation, Feature::landmark_id_, Landmark::SetBad, Frame::SetPose): each update
// is one small host-to-device copy of the new rows, appended (or scattered) into arrays grown by
// doubling.  Landmarks' observation lists are an append-only list; the landmark-major CSR the plan
// build reads is rebuilt lazily by a stable radix sort (rocPRIM) when it changed, which keeps each
// landmark's observations in insertion order.
#include <algorithm>
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "vx_sort.hpp"

#include "dmap.hpp"

namespace vx {
namespace {

constexpr int kT = 256;
inline unsigned grid(long long n) { return (unsigned)std::max(1ll, (n + kT - 1) / kT); }

// make room for `want` bytes keeping the first `used` bytes (doubling; device-to-device copy)
int grow(vx_ctx* c, DevBuf& d, size_t used, size_t want) {
    if (want <= d.bytes) return VX_OK;
    size_t cap = std::max<size_t>(d.bytes * 2, 4096);
    while (cap < want) cap *= 2;
    void* np = nullptr;
    VX_HIP(c, hipMalloc(&np, cap));
    if (used) VX_HIP(c, hipMemcpyAsync(np, d.p, used, hipMemcpyDeviceToDevice, c->stream));
    VX_HIP(c, hipStreamSynchronize(c->stream));
    d.release();
    d.p = np;
    d.bytes = cap;
    return VX_OK;
}

// append n elements of T (host) at element offset `at` of a device array
template <class T>
int append(vx_ctx* c, DevBuf& d, int64_t at, const T* h, int64_t n) {
    int rc;
    if ((rc = grow(c, d, (size_t)at * sizeof(T), (size_t)(at + n) * sizeof(T)))) return rc;
    if (n) {
        VX_HIP(c, hipMemcpyAsync(d.as<T>() + at, h, (size_t)n * sizeof(T), hipMemcpyHostToDevice, c->stream));
        VX_HIP(c, hipStreamSynchronize(c->stream));  // the caller's host rows may go away on return
    }
    return VX_OK;
}

// scatter rows of `width` elements: dst[r(i) * width + j] = src[i * width + j], r(i) = idx[i], or
// id_row[idx[i]] when idx holds observation ids
template <class T>
__global__ void k_scatter_rows(T* dst, const int64_t* idx, const int64_t* id_row, const T* src, int n, int width) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (int64_t)n * width) return;
    const int64_t i = e / width, j = e - i * width;
    const int64_t r = id_row ? id_row[idx[i]] : idx[i];
    dst[r * width + j] = src[e];
}

template <class T>
int scatter(vx_ctx* c, DevBuf& dst, const std::vector<int64_t>& idx, const T* src, int width,
            const DevBuf* id_row = nullptr) {
    const int n = (int)idx.size();
    if (!n) return VX_OK;
    // one staging allocation: indices then values
    const size_t ib = (size_t)n * sizeof(int64_t), vb = (size_t)n * width * sizeof(T);
    DevBuf tmp;
    VX_HIP(c, tmp.ensure(ib + vb));
    VX_HIP(c, hipMemcpyAsync(tmp.p, idx.data(), ib, hipMemcpyHostToDevice, c->stream));
    VX_HIP(c, hipMemcpyAsync(tmp.as<uint8_t>() + ib, src, vb, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(k_scatter_rows<T>, dim3(grid((long long)n * width)), dim3(kT), 0, c->stream, dst.as<T>(),
                       tmp.as<int64_t>(), id_row ? (const int64_t*)id_row->as<int64_t>() : nullptr,
                       reinterpret_cast<const T*>(tmp.as<uint8_t>() + ib), n, width);
    VX_LAUNCH_CHECK(c, "k_scatter_rows");
    VX_HIP(c, hipStreamSynchronize(c->stream));  // tmp is freed on return
    return VX_OK;
}

__global__ void k_iota(int* v, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = (int)i;
}
// observations per landmark row; removed observations (kDeadObs) are not counted
__global__ void k_count(const int* keys, int64_t n, int64_t nl, int* cnt) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && (unsigned)keys[i] < (unsigned long long)nl) atomicAdd(&cnt[keys[i]], 1);
}
// sorted order -> CSR payload; int32 prefix -> int64 pointers
__global__ void k_csr_fill(const int* perm, int64_t n, const uint64_t* okf_in, const uint64_t* ofi_in,
                           uint64_t* okf, uint64_t* ofi, const int* scan, int64_t n_lm, int64_t* optr) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const int j = perm[i];
        okf[i] = okf_in[j];
        ofi[i] = ofi_in[j];
    }
    if (i <= n_lm) optr[i] = scan[i];
}

// live row flags: not tombstoned (RemoveObservation) and its landmark not removed
__global__ void k_live_rows(const int* obs_lm, const uint8_t* lm_bad, int64_t n, int* flag) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int l = obs_lm[i];
    flag[i] = (l != kDeadObs && lm_bad[l] != kLmRemoved) ? 1 : 0;
}
// live row i -> row pos[i] of the target arrays (order kept); every id re-pointed (-1: dropped)
__global__ void k_compact_rows(const int* flag, const int* pos, int64_t n, const int* lm, const uint64_t* kf,
                               const uint64_t* fi, const int64_t* id, int* lm2, uint64_t* kf2, uint64_t* fi2,
                               int64_t* id2, int64_t* id_row) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t o = id[i];
    if (!flag[i]) {
        id_row[o] = -1;
        return;
    }
    const int64_t r = pos[i];
    lm2[r] = lm[i];
    kf2[r] = kf[i];
    fi2[r] = fi[i];
    id2[r] = o;
    id_row[o] = r;
}

// Drops the dead observation rows (RemoveObservation tombstones and the pairs of removed
// landmarks), keeping the live rows in order — so every landmark's list and the CSR stay as they
// were — on the device: flags, a scan, one gather into the second set of arrays, which are then
// swapped in; id_row re-points every observation id, so obs_index is untouched.  The live row
// count is the host's n_obs_live (no read-back).  Amortised: it runs once dead rows exceed a
// quarter of the list.
int dmap_compact(vx_ctx* c, vx_dmap* m) {
    const int64_t n = m->n_obs;
    hipStream_t s = c->stream;
    VX_HIP(c, m->cflag.ensure((size_t)std::max<int64_t>(n, 1) * 4));
    VX_HIP(c, m->cpos.ensure((size_t)std::max<int64_t>(n, 1) * 4));
    const int64_t k = m->n_obs_live;
    const size_t keep = (size_t)std::max<int64_t>(k, 1);
    VX_HIP(c, m->obs_lm2.ensure(keep * 4));
    VX_HIP(c, m->obs_kf2.ensure(keep * 8));
    VX_HIP(c, m->obs_fi2.ensure(keep * 8));
    VX_HIP(c, m->obs_id2.ensure(keep * 8));
    if (n > 0) {
        hipLaunchKernelGGL(k_live_rows, dim3(grid(n)), dim3(kT), 0, s, (const int*)m->obs_lm.as<int>(),
                           (const uint8_t*)m->lm_bad.as<uint8_t>(), n, m->cflag.as<int>());
        VX_LAUNCH_CHECK(c, "dmap compact flags");
        size_t bytes = 0;
        VX_HIP(c, rocprim::exclusive_scan(nullptr, bytes, m->cflag.as<int>(), m->cpos.as<int>(), 0, (size_t)n,
                                          rocprim::plus<int>(), s));
        VX_HIP(c, m->tmp.ensure(std::max<size_t>(bytes, 16)));
        VX_HIP(c, rocprim::exclusive_scan(m->tmp.p, bytes, m->cflag.as<int>(), m->cpos.as<int>(), 0, (size_t)n,
                                          rocprim::plus<int>(), s));
        hipLaunchKernelGGL(k_compact_rows, dim3(grid(n)), dim3(kT), 0, s, (const int*)m->cflag.as<int>(),
                           (const int*)m->cpos.as<int>(), n, (const int*)m->obs_lm.as<int>(),
                           (const uint64_t*)m->obs_kf.as<uint64_t>(), (const uint64_t*)m->obs_fi.as<uint64_t>(),
                           (const int64_t*)m->obs_id.as<int64_t>(), m->obs_lm2.as<int>(), m->obs_kf2.as<uint64_t>(),
                           m->obs_fi2.as<uint64_t>(), m->obs_id2.as<int64_t>(), m->id_row.as<int64_t>());
        VX_LAUNCH_CHECK(c, "dmap compact rows");
        // the host's live count must be the device's (8 bytes back; compaction is rare)
        int tail[2];
        VX_HIP(c, hipMemcpyAsync(&tail[0], m->cflag.as<int>() + n - 1, 4, hipMemcpyDeviceToHost, s));
        VX_HIP(c, hipMemcpyAsync(&tail[1], m->cpos.as<int>() + n - 1, 4, hipMemcpyDeviceToHost, s));
        VX_HIP(c, hipStreamSynchronize(s));
        if (tail[0] + tail[1] != k)
            return set_error(c, VX_ERR_STATE, "dmap compaction: %d live rows on the device, %lld on the host",
                             tail[0] + tail[1], (long long)k);
    }
    // (the pointers only: DevBuf frees on destruction, so no temporary DevBuf may hold one)
    for (auto pr : {std::make_pair(&m->obs_lm, &m->obs_lm2), std::make_pair(&m->obs_kf, &m->obs_kf2),
                    std::make_pair(&m->obs_fi, &m->obs_fi2), std::make_pair(&m->obs_id, &m->obs_id2)}) {
        std::swap(pr.first->p, pr.second->p);
        std::swap(pr.first->bytes, pr.second->bytes);
    }
    m->n_obs = k;
    m->csr_dirty = true;
    return VX_OK;
}

}  // namespace

int dmap_build_csr(vx_ctx* c, vx_dmap* m) {
    // $VX_DMAP_COMPACT_MIN: fewest rows worth compacting (default 4096; 0: compact whenever a dead
    // row exists — the tests' setting)
    const char* e = getenv("VX_DMAP_COMPACT_MIN");
    const int64_t kMin = e ? (int64_t)atoll(e) : (int64_t)4096;
    const int64_t dead = m->n_obs - m->n_obs_live;
    if (dead > 0 && (kMin == 0 || (m->n_obs >= kMin && 4 * dead > m->n_obs))) {
        const int rc = dmap_compact(c, m);
        if (rc) return rc;
    }
    if (!m->csr_dirty) return VX_OK;
    const int64_t n = m->n_obs, nl = m->n_lm;
    hipStream_t s = c->stream;
    VX_HIP(c, m->optr.ensure((size_t)(nl + 1) * sizeof(int64_t)));
    VX_HIP(c, m->okf.ensure((size_t)std::max<int64_t>(n, 1) * 8));
    VX_HIP(c, m->ofi.ensure((size_t)std::max<int64_t>(n, 1) * 8));
    VX_HIP(c, m->cnt.ensure((size_t)(nl + 1) * 4 * 2));
    int* cnt = m->cnt.as<int>();
    int* scn = cnt + (nl + 1);
    VX_HIP(c, hipMemsetAsync(cnt, 0, (size_t)(nl + 1) * 4, s));
    if (n > 0) {
        for (DevBuf* d : {&m->sort_keys, &m->sort_keys2, &m->sort_vals, &m->sort_vals2})
            VX_HIP(c, d->ensure((size_t)n * 4));
        hipLaunchKernelGGL(k_iota, dim3(grid(n)), dim3(kT), 0, s, m->sort_vals.as<int>(), n);
        hipLaunchKernelGGL(k_count, dim3(grid(n)), dim3(kT), 0, s, m->obs_lm.as<int>(), n, nl, cnt);
        VX_LAUNCH_CHECK(c, "dmap csr count");
        // (1 << bits) > nl: a removed observation's key (kDeadObs, all bits set) sorts after every
        // live landmark row, so the CSR's first optr[nl] entries are exactly the live observations
        unsigned bits = 1;
        while ((1ll << bits) <= nl) ++bits;
        size_t bytes = 0;
        VX_HIP(c, rocprim::radix_sort_pairs<OnesweepSort>(nullptr, bytes, m->obs_lm.as<int>(), m->sort_keys2.as<int>(),
                                            m->sort_vals.as<int>(), m->sort_vals2.as<int>(), (size_t)n, 0, bits, s));
        VX_HIP(c, m->tmp.ensure(std::max<size_t>(bytes, 16)));
        VX_HIP(c, rocprim::radix_sort_pairs<OnesweepSort>(m->tmp.p, bytes, m->obs_lm.as<int>(), m->sort_keys2.as<int>(),
                                            m->sort_vals.as<int>(), m->sort_vals2.as<int>(), (size_t)n, 0, bits, s));
    }
    size_t bytes = 0;
    VX_HIP(c, rocprim::exclusive_scan(nullptr, bytes, cnt, scn, 0, (size_t)nl + 1, rocprim::plus<int>(), s));
    VX_HIP(c, m->tmp.ensure(std::max<size_t>(bytes, 16)));
    VX_HIP(c, rocprim::exclusive_scan(m->tmp.p, bytes, cnt, scn, 0, (size_t)nl + 1, rocprim::plus<int>(), s));
    hipLaunchKernelGGL(k_csr_fill, dim3(grid(std::max<int64_t>(n, nl + 1))), dim3(kT), 0, s,
                       (const int*)m->sort_vals2.as<int>(), n, (const uint64_t*)m->obs_kf.as<uint64_t>(),
                       (const uint64_t*)m->obs_fi.as<uint64_t>(), m->okf.as<uint64_t>(), m->ofi.as<uint64_t>(),
                       (const int*)scn, nl, m->optr.as<int64_t>());
    VX_LAUNCH_CHECK(c, "dmap csr fill");
    m->csr_dirty = false;
    return VX_OK;
}

}  // namespace vx

using namespace vx;

extern "C" {

int vx_dmap_create(vx_ctx* c, vx_dmap** out) {
    if (!c || !out) return c ? set_error(c, VX_ERR_INVALID, "vx_dmap_create: bad arguments") : VX_ERR_INVALID;
    *out = new vx_dmap();
    (*out)->c = c;
    return VX_OK;
}

void vx_dmap_destroy(vx_dmap* m) { delete m; }

int vx_dmap_add_keyframe(vx_dmap* m, uint64_t kf_id, const double* pose7, const double* intr4, int has_cam,
                         int n_feat, const double* uv, const uint64_t* lm, const uint8_t* fl) {
    if (!m) return VX_ERR_INVALID;
    vx_ctx* c = m->c;
    if (!pose7 || n_feat < 0 || (n_feat > 0 && (!uv || !lm || !fl)) || (has_cam && !intr4))
        return set_error(c, VX_ERR_INVALID, "vx_dmap_add_keyframe: bad arguments");
    if (m->kf_index.count(kf_id)) return set_error(c, VX_ERR_INVALID, "keyframe %llu already in the map",
                                                   (unsigned long long)kf_id);
    VX_HIP(c, hipSetDevice(c->device));
    const int64_t k = (int64_t)m->kf_id.size(), f0 = m->kf_feat_ptr.back();
    const double zero4[4] = {0, 0, 0, 0};
    int rc;
    if ((rc = append(c, m->kf_pose, 7 * k, pose7, 7))) return rc;
    if ((rc = append(c, m->kf_intr, 4 * k, has_cam ? intr4 : zero4, 4))) return rc;
    if ((rc = append(c, m->feat_uv, 2 * f0, uv, 2 * (int64_t)n_feat))) return rc;
    if ((rc = append(c, m->feat_lm, f0, lm, n_feat))) return rc;
    if ((rc = append(c, m->feat_fl, f0, fl, n_feat))) return rc;
    int valid = 0;
    for (int i = 0; i < n_feat; ++i) valid += fl[i] & 1;
    m->kf_index[kf_id] = (int)k;
    m->kf_id.push_back(kf_id);
    m->kf_feat_ptr.push_back(f0 + n_feat);
    m->kf_has_cam.push_back(has_cam ? 1 : 0);
    m->kf_alive.push_back(1);
    ++m->n_kf_live;
    m->kf_valid_cnt.push_back(valid);
    m->feat_flags.insert(m->feat_flags.end(), fl, fl + n_feat);
    return VX_OK;
}

int vx_dmap_add_landmarks(vx_dmap* m, int n, const uint64_t* id, const double* pos3, const uint8_t* bad) {
    if (!m) return VX_ERR_INVALID;
    vx_ctx* c = m->c;
    if (n < 0 || (n > 0 && (!id || !pos3))) return set_error(c, VX_ERR_INVALID, "vx_dmap_add_landmarks: bad arguments");
    {
        std::unordered_map<uint64_t, int> batch;
        for (int i = 0; i < n; ++i)
            if (m->lm_index.count(id[i]) || !batch.emplace(id[i], i).second)
                return set_error(c, VX_ERR_INVALID, "landmark %llu already in the map", (unsigned long long)id[i]);
    }
    VX_HIP(c, hipSetDevice(c->device));
    std::vector<uint8_t> b(bad ? bad : nullptr, bad ? bad + n : nullptr);
    if (!bad) b.assign(n, 0);
    int rc;
    if ((rc = append(c, m->lm_id, m->n_lm, id, n))) return rc;
    if ((rc = append(c, m->lm_pos, 3 * m->n_lm, pos3, 3 * (int64_t)n))) return rc;
    if ((rc = append(c, m->lm_bad, m->n_lm, b.data(), n))) return rc;
    for (int i = 0; i < n; ++i) m->lm_index[id[i]] = (int)(m->n_lm + i);
    m->n_lm += n;
    m->n_lm_live += n;
    m->lm_obs_live.resize(m->n_lm, 0);
    m->lm_removed.resize(m->n_lm, 0);
    m->csr_dirty = true;
    return VX_OK;
}

int vx_dmap_add_observations(vx_dmap* m, int n, const uint64_t* lm_id, const uint64_t* kf_id, const uint64_t* fi) {
    if (!m) return VX_ERR_INVALID;
    vx_ctx* c = m->c;
    if (n < 0 || (n > 0 && (!lm_id || !kf_id || !fi)))
        return set_error(c, VX_ERR_INVALID, "vx_dmap_add_observations: bad arguments");
    std::vector<int> li(n);
    for (int i = 0; i < n; ++i) {
        auto it = m->lm_index.find(lm_id[i]);
        if (it == m->lm_index.end())
            return set_error(c, VX_ERR_INVALID, "observation of unknown landmark %llu", (unsigned long long)lm_id[i]);
        li[i] = it->second;
    }
    // observations_[keyframe_id] = feature_idx (landmark.h:32-35): a new pair is appended (in
    // call order), a present one -- from an earlier call or earlier in this batch -- keeps its row
    // and takes the new feature index
    std::vector<int> a_lm;
    std::vector<uint64_t> a_kf, a_fi;
    std::vector<int64_t> w_row;  // (observation ids)
    std::vector<uint64_t> w_fi;
    // pairs first seen in this batch -> their new rows / ids; entered into obs_index (and the live counts)
    // only once the device rows are written (a failed append leaves the map unchanged)
    std::unordered_map<std::pair<int, uint64_t>, int64_t, vx_dmap::PairHash> fresh;
    std::vector<std::pair<int, uint64_t>> fresh_order;
    for (int i = 0; i < n; ++i) {
        const auto key = std::make_pair(li[i], kf_id[i]);
        auto it = m->obs_index.find(key);
        if (it != m->obs_index.end()) {
            w_row.push_back(it->second);
            w_fi.push_back(fi[i]);
            continue;
        }
        auto f = fresh.find(key);
        if (f != fresh.end()) {
            a_fi[f->second] = fi[i];
        } else {
            fresh.emplace(key, (int64_t)a_lm.size());
            fresh_order.push_back(key);
            a_lm.push_back(li[i]);
            a_kf.push_back(kf_id[i]);
            a_fi.push_back(fi[i]);
        }
    }
    VX_HIP(c, hipSetDevice(c->device));
    int rc;
    const int64_t na = (int64_t)a_lm.size();
    if ((rc = append(c, m->obs_lm, m->n_obs, a_lm.data(), na))) return rc;
    if ((rc = append(c, m->obs_kf, m->n_obs, a_kf.data(), na))) return rc;
    if ((rc = append(c, m->obs_fi, m->n_obs, a_fi.data(), na))) return rc;
    std::vector<int64_t> a_id(na), a_row(na);
    for (int64_t j = 0; j < na; ++j) {
        a_id[j] = m->n_ids + j;
        a_row[j] = m->n_obs + j;
    }
    if ((rc = append(c, m->obs_id, m->n_obs, a_id.data(), na))) return rc;
    if ((rc = append(c, m->id_row, m->n_ids, a_row.data(), na))) return rc;
    if ((rc = scatter(c, m->obs_fi, w_row, w_fi.data(), 1, &m->id_row))) return rc;
    for (const auto& key : fresh_order) {
        m->obs_index.emplace(key, m->n_ids + fresh[key]);
        ++m->lm_obs_live[key.first];
        ++m->n_obs_live;
    }
    m->n_obs += na;
    m->n_ids += na;
    if (na || !w_row.empty()) m->csr_dirty = true;
    return VX_OK;
}

int vx_dmap_remove_observations(vx_dmap* m, int n, const uint64_t* lm_id, const uint64_t* kf_id) {
    if (!m) return VX_ERR_INVALID;
    vx_ctx* c = m->c;
    if (n < 0 || (n > 0 && (!lm_id || !kf_id)))
        return set_error(c, VX_ERR_INVALID, "vx_dmap_remove_observations: bad arguments");
    std::vector<int> li(n);
    for (int i = 0; i < n; ++i) {
        auto it = m->lm_index.find(lm_id[i]);
        if (it == m->lm_index.end())
            return set_error(c, VX_ERR_INVALID, "unknown landmark %llu", (unsigned long long)lm_id[i]);
        li[i] = it->second;
    }
    std::vector<int64_t> rows;  // (observation ids)
    for (int i = 0; i < n; ++i) {
        auto it = m->obs_index.find(std::make_pair(li[i], kf_id[i]));
        if (it == m->obs_index.end()) continue;  // unordered_map::erase of an absent key
        rows.push_back(it->second);
        m->obs_index.erase(it);
        --m->lm_obs_live[li[i]];
        --m->n_obs_live;
    }
    if (rows.empty()) return VX_OK;
    const std::vector<int> dead(rows.size(), kDeadObs);
    VX_HIP(c, hipSetDevice(c->device));
    int rc;
    if ((rc = scatter(c, m->obs_lm, rows, dead.data(), 1, &m->id_row))) return rc;
    m->csr_dirty = true;
    return VX_OK;
}

int vx_dmap_remove_keyframe(vx_dmap* m, uint64_t kf_id) {
    if (!m) return VX_ERR_INVALID;
    auto it = m->kf_index.find(kf_id);
    if (it == m->kf_index.end()) return set_error(m->c, VX_ERR_INVALID, "unknown keyframe %llu", (unsigned long long)kf_id);
    m->kf_alive[it->second] = 0;
    m->kf_index.erase(it);
    --m->n_kf_live;
    return VX_OK;
}

int vx_dmap_remove_landmarks(vx_dmap* m, int n, const uint64_t* lm_id) {
    if (!m) return VX_ERR_INVALID;
    vx_ctx* c = m->c;
    if (n < 0 || (n > 0 && !lm_id)) return set_error(c, VX_ERR_INVALID, "vx_dmap_remove_landmarks: bad arguments");
    std::vector<int64_t> rows;
    for (int i = 0; i < n; ++i) {
        auto it = m->lm_index.find(lm_id[i]);
        if (it == m->lm_index.end()) continue;  // unordered_map::erase of an absent key
        rows.push_back(it->second);
        m->n_obs_live -= m->lm_obs_live[it->second];  // (its pairs can no longer be named: lm_index)
        m->lm_obs_live[it->second] = 0;
        m->lm_removed[it->second] = 1;                // (its observation rows go at the next compaction)
        m->lm_index.erase(it);
    }
    if (rows.empty()) return VX_OK;
    m->n_lm_live -= (int64_t)rows.size();
    // the removed landmarks' pairs left in obs_index: purged once they outnumber the live ones
    // (amortised host work, off the plan build)
    if ((int64_t)m->obs_index.size() > 2 * m->n_obs_live + 4096)
        for (auto it = m->obs_index.begin(); it != m->obs_index.end();)
            it = m->lm_removed[it->first.first] ? m->obs_index.erase(it) : std::next(it);
    const std::vector<uint8_t> removed(rows.size(), kLmRemoved);
    VX_HIP(c, hipSetDevice(c->device));
    return scatter(c, m->lm_bad, rows, removed.data(), 1);
}

int vx_dmap_set_features(vx_dmap* m, uint64_t kf_id, int n, const int32_t* idx, const uint64_t* lm,
                         const uint8_t* fl) {
    if (!m) return VX_ERR_INVALID;
    vx_ctx* c = m->c;
    if (n < 0 || (n > 0 && (!idx || !lm || !fl))) return set_error(c, VX_ERR_INVALID, "vx_dmap_set_features: bad arguments");
    auto it = m->kf_index.find(kf_id);
    if (it == m->kf_index.end()) return set_error(c, VX_ERR_INVALID, "unknown keyframe %llu", (unsigned long long)kf_id);
    const int k = it->second;
    const int64_t f0 = m->kf_feat_ptr[k], nf = m->kf_feat_ptr[k + 1] - f0;
    std::vector<int64_t> g(n);
    for (int i = 0; i < n; ++i) {
        if (idx[i] < 0 || idx[i] >= nf) return set_error(c, VX_ERR_INVALID, "feature index %d out of range", idx[i]);
        g[i] = f0 + idx[i];
        m->kf_valid_cnt[k] += (fl[i] & 1) - (m->feat_flags[g[i]] & 1);
        m->feat_flags[g[i]] = fl[i];
    }
    VX_HIP(c, hipSetDevice(c->device));
    int rc;
    if ((rc = scatter(c, m->feat_lm, g, lm, 1))) return rc;
    if ((rc = scatter(c, m->feat_fl, g, fl, 1))) return rc;
    return VX_OK;
}

int vx_dmap_set_landmark_bad(vx_dmap* m, int n, const uint64_t* id, const uint8_t* bad) {
    if (!m) return VX_ERR_INVALID;
    vx_ctx* c = m->c;
    if (n < 0 || (n > 0 && (!id || !bad))) return set_error(c, VX_ERR_INVALID, "vx_dmap_set_landmark_bad: bad arguments");
    std::vector<int64_t> g(n);
    for (int i = 0; i < n; ++i) {
        auto it = m->lm_index.find(id[i]);
        if (it == m->lm_index.end()) return set_error(c, VX_ERR_INVALID, "unknown landmark %llu", (unsigned long long)id[i]);
        g[i] = it->second;
    }
    VX_HIP(c, hipSetDevice(c->device));
    return scatter(c, m->lm_bad, g, bad, 1);
}

int vx_dmap_set_poses(vx_dmap* m, int n, const uint64_t* id, const double* pose7) {
    if (!m) return VX_ERR_INVALID;
    vx_ctx* c = m->c;
    if (n < 0 || (n > 0 && (!id || !pose7))) return set_error(c, VX_ERR_INVALID, "vx_dmap_set_poses: bad arguments");
    std::vector<int64_t> g(n);
    for (int i = 0; i < n; ++i) {
        auto it = m->kf_index.find(id[i]);
        if (it == m->kf_index.end()) return set_error(c, VX_ERR_INVALID, "unknown keyframe %llu", (unsigned long long)id[i]);
        g[i] = it->second;
    }
    VX_HIP(c, hipSetDevice(c->device));
    return scatter(c, m->kf_pose, g, pose7, 7);
}

int vx_dmap_counts(const vx_dmap* m, int64_t* out4) {
    if (!m || !out4) return VX_ERR_INVALID;
    out4[0] = (int64_t)m->kf_id.size();
    out4[1] = m->kf_feat_ptr.back();
    out4[2] = m->n_lm;
    out4[3] = m->n_obs;
    return VX_OK;
}

int vx_dmap_live_counts(const vx_dmap* m, int64_t* out4) {
    if (!m || !out4) return VX_ERR_INVALID;
    out4[0] = m->n_kf_live;
    out4[1] = m->n_lm_live;
    out4[2] = m->n_obs_live;
    out4[3] = 0;
    return VX_OK;
}

int vx_dmap_download(vx_dmap* m, double* kf_pose, double* lm_pos) {
    if (!m) return VX_ERR_INVALID;
    vx_ctx* c = m->c;
    VX_HIP(c, hipSetDevice(c->device));
    VX_HIP(c, hipStreamSynchronize(c->stream));
    const size_t nk = m->kf_id.size();
    if (kf_pose && nk) VX_HIP(c, hipMemcpy(kf_pose, m->kf_pose.p, nk * 7 * sizeof(double), hipMemcpyDeviceToHost));
    if (lm_pos && m->n_lm)
        VX_HIP(c, hipMemcpy(lm_pos, m->lm_pos.p, (size_t)m->n_lm * 3 * sizeof(double), hipMemcpyDeviceToHost));
    return VX_OK;
}

}  // extern "C"
