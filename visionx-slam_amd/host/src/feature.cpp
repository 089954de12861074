// feature.cpp — ORBExtractor / ORBMatcher / LocalBA adapters over the C ABI (see feature.h).
#include "visionx/feature.h"

#include "visionx/device_map.h"
#include "host_pool.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>

namespace visionx {

namespace vxhost {
namespace {
struct CtxHolder {
    vx_ctx* ctx = nullptr;
    ~CtxHolder() {
        if (ctx) vx_destroy(ctx);
    }
};
}  // namespace

vx_ctx* ThreadContext() {
    thread_local CtxHolder h;
    if (!h.ctx) {
        const char* env = std::getenv("VX_DEVICE");
        const int dev = env ? std::atoi(env) : 0;
        const int rc = vx_create(dev, &h.ctx);
        if (rc != VX_OK) throw std::runtime_error("vx_create failed: " + std::to_string(rc));
    }
    return h.ctx;
}
}  // namespace vxhost

// the landmark write-back's software prefetch: distance in landmarks, and the object's three lines
// (shared_ptr control block + id / position, then the observation map and the mutex)
// ($VX_WB_PREFETCH=0: none, for A/B runs)
static size_t LmAhead() {
    static const size_t d = [] {
        const char* e = std::getenv("VX_WB_PREFETCH");
        return e && e[0] == '0' ? (size_t)0 : (size_t)16;
    }();
    return d;
}
static inline void PrefetchObject(const void* p) {
    if (!p) return;
    const char* c = static_cast<const char*>(p);
    __builtin_prefetch(c, 1);
    __builtin_prefetch(c + 64, 1);
    __builtin_prefetch(c + 128, 1);
}

static void check(vx_ctx* c, int rc, const char* what) {
    if (rc != VX_OK) throw std::runtime_error(std::string(what) + ": " + vx_last_error(c));
}

// ------------------------------------------------------------------ ORBExtractor
ORBExtractor::ORBExtractor(int n_features, float scale_factor, int n_levels) {
    vx_orb_default_params(&params_);  // OpenCV ORB defaults (orb_extractor.cpp:6)
    params_.n_features = n_features;
    params_.scale_factor = scale_factor;
    params_.n_levels = n_levels;
}

void ORBExtractor::Extract(Frame& frame) {
    // orb_extractor.cpp:9-27: detectAndCompute, then features.clear() + one Feature per keypoint
    // (position, response) and Descriptors() = desc.clone().
    auto& features = frame.Features();
    const ImageU8& img = frame.Image();
    features.clear();
    frame.Descriptors() = DescriptorMat{};
    if (img.empty()) return;  // detectAndCompute returns early on an empty image
    vx_ctx* c = vxhost::ThreadContext();
    int cap = 2 * params_.n_features + 256;
    int n = 0;
    for (int attempt = 0; attempt < 2; ++attempt) {
        kp_.resize(cap);
        desc_.resize((size_t)cap * 32);
        const int rc = vx_orb_extract(c, &params_, img.ptr(), img.cols, img.rows, img.channels,
                                      (int64_t)img.step(), kp_.data(), desc_.data(), cap, &n);
        if (rc == VX_ERR_CAPACITY && n > cap) {
            cap = n;
            continue;
        }
        check(c, rc, "vx_orb_extract");
        break;
    }
    features.reserve(n);
    for (int i = 0; i < n; ++i) {
        Feature f;
        f.position = Vec2d(kp_[i].x, kp_[i].y);
        f.response = kp_[i].response;
        features.emplace_back(f);
    }
    DescriptorMat d;
    d.rows = n;
    d.data.assign(desc_.begin(), desc_.begin() + (size_t)n * 32);
    frame.Descriptors() = std::move(d);
}

void ORBExtractor::ExtractBatch(const std::vector<Frame::Ptr>& frames) {
    if (frames.empty()) return;
    const ImageU8& i0 = frames[0]->Image();
    bool uniform = (int)frames.size() <= VX_MAX_BATCH && !i0.empty();
    for (const auto& f : frames)
        uniform = uniform && f->Image().rows == i0.rows && f->Image().cols == i0.cols &&
                  f->Image().channels == i0.channels && f->Image().step() == i0.step() && !f->Image().empty();
    if (!uniform) {
        for (const auto& f : frames) Extract(*f);
        return;
    }
    vx_ctx* c = vxhost::ThreadContext();
    std::vector<const uint8_t*> imgs;
    for (const auto& f : frames) imgs.push_back(f->Image().ptr());
    check(c, vx_orb_extract_batch(c, &params_, imgs.data(), (int)frames.size(), i0.cols, i0.rows, i0.channels,
                                  (int64_t)i0.step(), 0),
          "vx_orb_extract_batch");
    for (size_t b = 0; b < frames.size(); ++b) {
        Frame& frame = *frames[b];
        int cap = 2 * params_.n_features + 256, n = 0;
        for (int attempt = 0; attempt < 2; ++attempt) {  // as Extract(): resize to the count and fetch again
            kp_.resize(cap);
            desc_.resize((size_t)cap * 32);
            const int rc = vx_orb_batch_fetch(c, 0, (int)b, kp_.data(), desc_.data(), cap, &n);
            if (rc == VX_ERR_CAPACITY && n > cap) {
                cap = n;
                continue;
            }
            check(c, rc, "vx_orb_batch_fetch");
            break;
        }
        auto& features = frame.Features();
        features.clear();
        features.reserve(n);
        for (int i = 0; i < n; ++i) {
            Feature f;
            f.position = Vec2d(kp_[i].x, kp_[i].y);
            f.response = kp_[i].response;
            features.emplace_back(f);
        }
        DescriptorMat d;
        d.rows = n;
        d.data.assign(desc_.begin(), desc_.begin() + (size_t)n * 32);
        frame.Descriptors() = std::move(d);
    }
}

// ------------------------------------------------------------------ ORBMatcher
ORBMatcher::ORBMatcher(const Options& options) : options_(options) {}

void ORBMatcher::Finish(std::vector<DMatch>& matches, int n) {
    matches.reserve(n);
    for (int i = 0; i < n; ++i) {
        DMatch m;
        m.queryIdx = buf_[i].query_idx;
        m.trainIdx = buf_[i].train_idx;
        m.imgIdx = 0;
        m.distance = buf_[i].distance;
        matches.push_back(m);
    }
    if (matches.size() < (size_t)options_.min_matches)          // orb_matcher.cpp:38-40
        std::fprintf(stderr, "W [ORBMatcher] Too few matches: %zu\n", matches.size());
}

std::vector<int> ORBMatcher::MatchBatch(const std::vector<std::pair<Frame::Ptr, Frame::Ptr>>& pairs,
                                        std::vector<std::vector<DMatch>>& matches) {
    matches.assign(pairs.size(), {});
    std::vector<int> counts(pairs.size(), 0);
    vx_ctx* c = vxhost::ThreadContext();
    for (size_t p0 = 0; p0 < pairs.size(); p0 += VX_MAX_MATCH_PAIRS) {
        const int np = (int)std::min<size_t>(VX_MAX_MATCH_PAIRS, pairs.size() - p0);
        std::vector<const uint8_t*> q(np), t(np);
        std::vector<int32_t> nq(np), nt(np);
        int cap = 1;
        for (int i = 0; i < np; ++i) {
            const DescriptorMat& d1 = pairs[p0 + i].first->Descriptors();
            const DescriptorMat& d2 = pairs[p0 + i].second->Descriptors();
            q[i] = d1.empty() ? nullptr : d1.ptr();
            t[i] = d2.empty() ? nullptr : d2.ptr();
            nq[i] = d1.empty() ? 0 : d1.rows;                    // orb_matcher.cpp:18-20
            nt[i] = d2.empty() ? 0 : d2.rows;
            cap = std::max(cap, nq[i]);
        }
        check(c, vx_match_knn2_ratio_batch(c, np, q.data(), nq.data(), t.data(), nt.data(), options_.nn_ratio),
              "vx_match_knn2_ratio_batch");
        buf_.resize(cap);
        for (int i = 0; i < np; ++i) {
            if (nq[i] == 0 || nt[i] == 0) continue;              // Match() returns 0 before warning
            int n = 0;
            check(c, vx_match_batch_fetch(c, i, buf_.data(), cap, &n), "vx_match_batch_fetch");
            Finish(matches[p0 + i], n);
            counts[p0 + i] = (int)matches[p0 + i].size();
        }
    }
    return counts;
}

int ORBMatcher::Match(const Frame::Ptr& last, const Frame::Ptr& curr, std::vector<DMatch>& matches) {
    matches.clear();                                             // orb_matcher.cpp:13
    const DescriptorMat& d1 = last->Descriptors();
    const DescriptorMat& d2 = curr->Descriptors();
    if (d1.empty() || d2.empty()) return 0;                      // orb_matcher.cpp:18-20
    vx_ctx* c = vxhost::ThreadContext();
    buf_.resize(d1.rows);
    int n = 0;
    check(c, vx_match_knn2_ratio(c, d1.ptr(), d1.rows, d2.ptr(), d2.rows, options_.nn_ratio, buf_.data(),
                                 (int)buf_.size(), &n),
          "vx_match_knn2_ratio");
    Finish(matches, n);
    return (int)matches.size();
}

// ------------------------------------------------------------------ LocalBA
vx_map_view FlatMap::view() {
    vx_map_view v{};
    v.n_kf = (int32_t)kf_id.size();
    v.kf_id = kf_id.data();
    v.kf_pose = kf_pose.data();
    v.kf_intr = kf_intr.data();
    v.kf_has_cam = kf_has_cam.data();
    v.kf_feat_ptr = kf_feat_ptr.data();
    v.feat_uv = feat_uv.data();
    v.feat_lm_id = feat_lm_id.data();
    v.feat_flags = feat_flags.data();
    v.n_lm = (int32_t)lm_id.size();
    v.lm_id = lm_id.data();
    v.lm_pos = lm_pos.data();
    v.lm_bad = lm_bad.data();
    v.lm_obs_ptr = lm_obs_ptr.data();
    v.obs_kf_id = obs_kf_id.data();
    v.obs_feat_idx = obs_feat_idx.data();
    return v;
}

// Distinct landmark ids of the window's features in first-occurrence order (the order of the first
// feature referencing each: deterministic, like the device plan's fixed-landmark numbering).  The
// hash space is split into one region per part, so every part dedupes its own ids in its own table
// without atomics.  The features pass (Flatten) counted each keyframe's features per region (kreg,
// nk x parts); here they are bucketed by region in feature order (a parallel scatter over the
// keyframes), so part t walks only its own bucket — ~1/parts of the features, not all of them — and
// the first insert of an id is its first occurrence, which it marks.  Then the ids in feature order,
// keyframe by keyframe in parallel.  `hash` = the features' id hashes; `reg` = their regions (0xff: no
// landmark).
static uint64_t mix64(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

static inline uint8_t id_region(uint64_t hash, int parts) {  // the high hash bits scaled to [0, parts)
    return (uint8_t)(((hash >> 32) * (uint64_t)parts) >> 32);
}

static int id_parts() { return std::min(std::max(1, vxhost::Pool::Get().Threads()), 64); }

static void distinct_ids(const pinned_vector<uint64_t>& feat_lm, const std::vector<uint8_t>& reg,
                         const std::vector<uint64_t>& hash, std::vector<uint8_t>& firstocc, FlatMap& f,
                         std::vector<uint64_t>& ids) {
    auto& pool = vxhost::Pool::Get();
    static const bool timing = std::getenv("VX_FLATTEN_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    auto lap = [&](const char* w) {
        if (timing)
            std::fprintf(stderr, "[flatten-ids] %s %.3f ms\n", w,
                         std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    };
    const size_t nk = f.kf_feat_ptr.size() - 1;
    const int parts = id_parts();
    // bucket offsets: region-major, keyframe-minor (so each bucket lists its features in order)
    std::vector<int64_t>& kr = f.scratch_kreg;  // [k * parts + r]: count in, offset out
    std::vector<int64_t> rbeg((size_t)parts + 1, 0);
    {
        int64_t at = 0;
        for (int r = 0; r < parts; ++r) {
            rbeg[(size_t)r] = at;
            for (size_t k = 0; k < nk; ++k) {
                const int64_t c = kr[k * parts + r];
                kr[k * parts + r] = at;
                at += c;
            }
        }
        rbeg[(size_t)parts] = at;
    }
    f.scratch_bucket.resize((size_t)rbeg[(size_t)parts]);
    uint32_t* bucket = f.scratch_bucket.data();
    pool.For(nk, 1, [&](size_t k0, size_t k1) {
        for (size_t k = k0; k < k1; ++k) {
            int64_t* off = &kr[k * parts];
            for (int64_t o = f.kf_feat_ptr[k]; o < f.kf_feat_ptr[k + 1]; ++o)
                if (reg[o] != 0xff) bucket[off[reg[o]]++] = (uint32_t)o;
        }
    });
    lap("scatter");
    // slots per region: ~2 x its bucket.  (A region whose ids outgrow half its slots — every feature
    // its own landmark — moves to a private table of twice the size, its keys re-inserted.)
    size_t per = 64;
    int64_t most = 0;
    for (int r = 0; r < parts; ++r) most = std::max(most, rbeg[(size_t)r + 1] - rbeg[(size_t)r]);
    while (per < 2 * (size_t)most / 4 + 64) per <<= 1;  // (ids <= features; a quarter as a first guess)
    f.scratch_key.resize(per * (size_t)parts);
    f.scratch_first.resize(per * (size_t)parts);  // (occupancy flags)
    pool.For((size_t)parts, 1, [&](size_t a, size_t b) {
        std::vector<uint64_t> own_key;  // a grown region's table
        std::vector<uint32_t> own_used;
        for (size_t t = a; t < b; ++t) {
            uint64_t* key = f.scratch_key.data() + t * per;
            uint32_t* used = f.scratch_first.data() + t * per;
            size_t cap = per;
            std::fill(used, used + cap, 0u);
            size_t n_in = 0;
            for (int64_t q = rbeg[t]; q < rbeg[t + 1]; ++q) {
                const uint32_t o = bucket[q];
                const uint64_t id = feat_lm[o];
                size_t h = (size_t)hash[o] & (cap - 1);
                for (;;) {
                    if (!used[h]) {  // first occurrence
                        used[h] = 1;
                        key[h] = id;
                        firstocc[o] = 1;
                        ++n_in;
                        break;
                    }
                    if (key[h] == id) break;
                    h = (h + 1) & (cap - 1);
                }
                if (2 * n_in > cap) {  // keep the load <= 1/2: double the table, re-insert its keys
                    std::vector<uint64_t> nk2(2 * cap);
                    std::vector<uint32_t> nu(2 * cap, 0u);
                    for (size_t s = 0; s < cap; ++s) {
                        if (!used[s]) continue;
                        size_t g = (size_t)mix64(key[s]) & (2 * cap - 1);
                        while (nu[g]) g = (g + 1) & (2 * cap - 1);
                        nu[g] = 1;
                        nk2[g] = key[s];
                    }
                    own_key.swap(nk2);
                    own_used.swap(nu);
                    key = own_key.data();
                    used = own_used.data();
                    cap *= 2;
                }
            }
        }
    });
    lap("dedup");
    // the ids in feature order: per keyframe counts, their prefix, then each keyframe's ids in place
    std::vector<int64_t> kc(nk + 1, 0);
    pool.For(nk, 1, [&](size_t k0, size_t k1) {
        for (size_t k = k0; k < k1; ++k) {
            int64_t c = 0;
            for (int64_t o = f.kf_feat_ptr[k]; o < f.kf_feat_ptr[k + 1]; ++o) c += firstocc[o];
            kc[k + 1] = c;
        }
    });
    for (size_t k = 0; k < nk; ++k) kc[k + 1] += kc[k];
    ids.resize((size_t)kc[nk]);
    pool.For(nk, 1, [&](size_t k0, size_t k1) {
        for (size_t k = k0; k < k1; ++k) {
            int64_t at = kc[k];
            for (int64_t o = f.kf_feat_ptr[k]; o < f.kf_feat_ptr[k + 1]; ++o)
                if (firstocc[o]) ids[(size_t)at++] = feat_lm[o];
        }
    });
}

FlatMap LocalBA::Flatten(const Map& map, const Frame::Ptr& ref_kf, int window_size) {
    FlatMap f;
    Flatten(map, ref_kf, window_size, f);
    return f;
}

// The snapshot gather (local_ba.cpp:42-104 walks the same objects): keyframes by SelectKeyFrames,
// their features copied to per-keyframe offsets in parallel, the referenced landmark ids made
// distinct (first-occurrence order), then each landmark's position, bad flag and observation map read in parallel
// (two passes: counts, then the observation rows at their prefix offsets).  `f` keeps its
// capacity from call to call.  Landmarks are found in Map::Landmarks() (read-only; the reference's
// LocalBA runs on the tracking thread, which is also the one that edits the map).
void LocalBA::Flatten(const Map& map, const Frame::Ptr& ref_kf, int window_size, FlatMap& f) {
    auto& pool = vxhost::Pool::Get();
    static const bool timing = std::getenv("VX_FLATTEN_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    auto lap = [&](const char* w) {
        if (timing)
            std::fprintf(stderr, "[flatten] %s %.3f ms\n", w,
                         std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    };
    // (every array below is resized to this call's sizes and then fully written: resizing without
    // clearing first keeps the elements of the previous call instead of zero-filling them)
    f.frames.clear();
    const auto& all = map.KeyFrames();
    if (all.empty()) {
        f.landmarks.clear();
        f.kf_id.clear();
        f.kf_pose.clear();
        f.kf_intr.clear();
        f.kf_has_cam.clear();
        f.kf_feat_ptr.clear();
        f.feat_uv.clear();
        f.feat_lm_id.clear();
        f.feat_flags.clear();
        f.lm_id.clear();
        f.lm_pos.clear();
        f.lm_bad.clear();
        f.lm_obs_ptr.clear();
        f.obs_kf_id.clear();
        f.obs_feat_idx.clear();
        return;
    }
    // SelectKeyFrames (local_ba.cpp:42-62)
    const uint64_t max_id = ref_kf ? ref_kf->Id() : all.rbegin()->first;
    const int window = std::max(1, window_size);
    for (auto it = all.rbegin(); it != all.rend() && (int)f.frames.size() < window; ++it) {
        if (it->first > max_id) continue;
        f.frames.push_back(it->second);
    }
    std::reverse(f.frames.begin(), f.frames.end());
    const size_t nk = f.frames.size();
    f.kf_feat_ptr.assign(nk + 1, 0);
    f.kf_id.resize(nk);
    f.kf_pose.resize(7 * nk);
    f.kf_intr.resize(4 * nk);
    f.kf_has_cam.resize(nk);
    for (size_t k = 0; k < nk; ++k) f.kf_feat_ptr[k + 1] = f.kf_feat_ptr[k] + (int64_t)f.frames[k]->Features().size();
    const size_t nf = (size_t)f.kf_feat_ptr[nk];
    f.feat_uv.resize(2 * nf);
    f.feat_lm_id.resize(nf);
    f.feat_flags.resize(nf);
    std::vector<uint8_t>& reg = f.scratch_has;  // (the feature's id hash region, 0xff: no landmark)
    reg.resize(nf);
    std::vector<uint8_t>& firstocc = f.scratch_firstocc;
    firstocc.resize(nf);
    std::vector<uint64_t>& hash = f.scratch_hash;
    hash.resize(nf);
    const int parts = id_parts();
    f.scratch_kreg.assign(nk * (size_t)parts, 0);
    pool.For(nk, 1, [&](size_t k0, size_t k1) {
        for (size_t k = k0; k < k1; ++k) {
            const auto& kf = f.frames[k];
            const SE3d T = kf->Pose();
            f.kf_id[k] = kf->Id();
            const double pose[7] = {T.qx, T.qy, T.qz, T.qw, T.tx, T.ty, T.tz};
            std::copy(pose, pose + 7, &f.kf_pose[7 * k]);
            const auto cam = kf->GetCamera();
            f.kf_has_cam[k] = cam ? 1 : 0;
            const double intr[4] = {cam ? cam->fx() : 0.0, cam ? cam->fy() : 0.0, cam ? cam->cx() : 0.0,
                                    cam ? cam->cy() : 0.0};
            std::copy(intr, intr + 4, &f.kf_intr[4 * k]);
            size_t o = (size_t)f.kf_feat_ptr[k];
            for (const auto& feat : kf->Features()) {
                f.feat_uv[2 * o] = feat.position.x;
                f.feat_uv[2 * o + 1] = feat.position.y;
                f.feat_lm_id[o] = feat.landmark_id_;
                f.feat_flags[o] = (feat.has_landmark ? 1 : 0) | (feat.is_outlier ? 2 : 0);
                hash[o] = feat.has_landmark ? mix64(feat.landmark_id_) : 0ull;
                reg[o] = feat.has_landmark ? id_region(hash[o], parts) : (uint8_t)0xff;
                if (feat.has_landmark) ++f.scratch_kreg[k * (size_t)parts + reg[o]];
                firstocc[o] = 0;
                ++o;
            }
        }
    });
    lap("features");
    // the landmark ids the window's features reference, distinct, in first-occurrence order
    std::vector<uint64_t>& ids = f.scratch_ids;
    distinct_ids(f.feat_lm_id, reg, hash, firstocc, f, ids);
    lap("ids");
    // per landmark: the object (absent ids are skipped, as GetLandmark -> nullptr in
    // local_ba.cpp:96-97,135-136), position, bad flag, observation count
    const size_t nid = ids.size();
    const auto& lms = map.Landmarks();
    std::vector<Landmark*>& obj = f.scratch_obj;
    std::vector<int64_t>& cnt = f.scratch_cnt;
    obj.assign(nid, nullptr);
    cnt.assign(nid + 1, 0);
    f.landmarks.resize(nid);
    pool.For(nid, 512, [&](size_t a, size_t b) {
        for (size_t i = a; i < b; ++i) {
            auto it = lms.find(ids[i]);
            if (it == lms.end() || !it->second) {
                f.landmarks[i].reset();
                continue;
            }
            obj[i] = it->second.get();
            f.landmarks[i] = it->second;
            cnt[i + 1] = (int64_t)it->second->Observations().size();
        }
    });
    lap("lookups");
    size_t nl = 0;
    for (size_t i = 0; i < nid; ++i)  // (compact the found ones, keep first-occurrence order)
        if (obj[i]) {
            ids[nl] = ids[i];
            obj[nl] = obj[i];
            f.landmarks[nl] = std::move(f.landmarks[i]);
            cnt[nl + 1] = cnt[i + 1];
            ++nl;
        }
    f.landmarks.resize(nl);
    f.lm_obs_ptr.resize(nl + 1);
    f.lm_obs_ptr[0] = 0;
    for (size_t i = 0; i < nl; ++i) f.lm_obs_ptr[i + 1] = f.lm_obs_ptr[i] + cnt[i + 1];
    f.lm_id.assign(ids.begin(), ids.begin() + (std::ptrdiff_t)nl);
    f.lm_pos.resize(3 * nl);
    f.lm_bad.resize(nl);
    f.obs_kf_id.resize((size_t)f.lm_obs_ptr[nl]);
    f.obs_feat_idx.resize((size_t)f.lm_obs_ptr[nl]);
    pool.For(nl, 512, [&](size_t a, size_t b) {
        for (size_t i = a; i < b; ++i) {
            if (i + 8 < b) PrefetchObject(obj[i + 8]);
            if (i + 4 < b) {  // (the observation map's first node: its pointer is in the object, 4 later)
                const auto& ob4 = obj[i + 4]->Observations();
                if (!ob4.empty()) __builtin_prefetch(&*ob4.begin());
            }
            const Landmark* lm = obj[i];
            const Vec3d p = lm->Position();
            f.lm_pos[3 * i] = p.x;
            f.lm_pos[3 * i + 1] = p.y;
            f.lm_pos[3 * i + 2] = p.z;
            f.lm_bad[i] = lm->IsBad() ? 1 : 0;
            size_t o = (size_t)f.lm_obs_ptr[i];
            for (const auto& [kid, fidx] : lm->Observations()) {
                f.obs_kf_id[o] = kid;
                f.obs_feat_idx[o] = (uint64_t)fidx;
                ++o;
            }
        }
    });
    lap("landmarks");
}

vx_ba_options LocalBA::VxOptions() const {
    vx_ba_options o;
    o.window_size = options_.window_size;
    o.max_iterations = options_.max_iterations;
    o.min_pose_observations = options_.min_pose_observations;
    o.min_point_observations = options_.min_point_observations;
    o.huber_delta = options_.huber_delta;
    o.max_reproj_error = options_.max_reproj_error;
    return o;
}

void LocalBA::UseDeviceMap(std::shared_ptr<DeviceMap> dm) {
    dmap_ = std::move(dm);
    if (dmap_) check(dmap_->context(), vx_dmap_prefetch_results(dmap_->handle(), 1), "vx_dmap_prefetch_results");
}

void LocalBA::OptimizeResident(const Frame::Ptr& ref_kf) {
    DeviceMap& dm = *dmap_;
    static const bool timing = std::getenv("VX_RESIDENT_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (timing)
            fprintf(stderr, "[vx resident] %s %.1f us\n", what,
                    std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    };
    dm.Flush();
    lap("flush");
    vx_ctx* c = dm.context();
    const vx_ba_options o = VxOptions();
    check(c, vx_ba_optimize_dmap(c, dm.handle(), ref_kf ? ref_kf->Id() : 0, ref_kf ? 1 : 0, &o, &stats_),
          "vx_ba_optimize_dmap");
    lap("optimize");
    // the results in place in the pinned block the call filled (vx_ba_dmap_results_view; prefetching
    // is on from UseDeviceMap), the copying vx_ba_dmap_results otherwise
    const int32_t *kr = nullptr, *lr = nullptr;
    const double *kp = nullptr, *lp = nullptr;
    int nk = 0, nl = 0, ks = 8, ls = 4;
    int rc = vx_ba_dmap_results_view(c, dm.handle(), &kr, &kp, &lr, &lp, &nk, &nl);
    if (rc == VX_ERR_STATE) {
        rc = vx_ba_dmap_results(c, dm.handle(), (int)kf_rows_.size(), kf_rows_.data(), kf_out_.data(),
                                (int)lm_rows_.size(), lm_rows_.data(), lm_out_.data(), &nk, &nl);
        if (rc == VX_ERR_CAPACITY) {  // (the buffers keep the largest window seen)
            kf_rows_.resize(nk);
            kf_out_.resize(7 * (size_t)nk);
            lm_rows_.resize(nl);
            lm_out_.resize(3 * (size_t)nl);
            rc = vx_ba_dmap_results(c, dm.handle(), nk, kf_rows_.data(), kf_out_.data(), nl, lm_rows_.data(),
                                    lm_out_.data(), &nk, &nl);
        }
        check(c, rc, "vx_ba_dmap_results");
        kr32_.assign(kf_rows_.begin(), kf_rows_.begin() + nk);
        lr32_.assign(lm_rows_.begin(), lm_rows_.begin() + nl);
        kr = kr32_.data(), kp = kf_out_.data(), lr = lr32_.data(), lp = lm_out_.data(), ks = 7, ls = 3;
    }
    check(c, rc, "vx_ba_dmap_results_view");
    lap("results");
    // Frame::SetPose / Landmark::SetPosition (local_ba.cpp:173,237) on the host objects (the
    // landmarks over the host pool: each SetPosition takes only that landmark's mutex)
    for (int i = 0; i < nk; ++i) {
        const double* p = kp + (size_t)ks * i;
        SE3d T;
        T.qx = p[0]; T.qy = p[1]; T.qz = p[2]; T.qw = p[3];
        T.tx = p[4]; T.ty = p[5]; T.tz = p[6];
        if (const auto& fr = dm.FrameAt(kr[i])) fr->SetPose(T);
    }
    // (software prefetch LmAhead() / twice that landmarks ahead: each SetPosition's lock is a
    // serialising instruction, so without it every landmark object's cache misses are paid one
    // after the other — 2.4x on a cold 20k-landmark loop, scripts/probe/writeback_prefetch.cpp)
    const size_t ahead = LmAhead();
    vxhost::Pool::Get().For((size_t)nl, 1024, [&](size_t a, size_t b) {
        for (size_t i = a; i < b; ++i) {
            if (ahead && i + 2 * ahead < b) __builtin_prefetch(&dm.LandmarkAt(lr[i + 2 * ahead]));
            if (ahead && i + ahead < b) PrefetchObject(dm.LandmarkAt(lr[i + ahead]).get());
            if (const auto& lm = dm.LandmarkAt(lr[i]))
                lm->SetPosition(Vec3d(lp[ls * i], lp[ls * i + 1], lp[ls * i + 2]));
        }
    });
    lap("write-back");
}

void LocalBA::Optimize(const Map::Ptr& map, const Frame::Ptr& ref_kf) {
    stats_ = vx_ba_stats{};
    stats_.status = 1;
    if (!map) return;                                            // local_ba.cpp:67-69
    if (dmap_) {
        OptimizeResident(ref_kf);
        return;
    }
    // ($VX_RESIDENT_TIMING=1: the snapshot call's phases on stderr too, scripts/adapter_timing.py)
    static const bool timing = std::getenv("VX_RESIDENT_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (timing)
            fprintf(stderr, "[vx snapshot] %s %.1f us\n", what,
                    std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    };
    FlatMap& f = flat_;
    Flatten(*map, ref_kf, options_.window_size, f);
    lap("flatten");
    if (f.frames.size() < 2) return;                            // local_ba.cpp:73-75
    const vx_ba_options o = VxOptions();
    vx_map_view v = f.view();
    vx_ctx* c = vxhost::ThreadContext();
    check(c, vx_ba_optimize_map(c, &v, ref_kf ? ref_kf->Id() : 0, ref_kf ? 1 : 0, &o, &stats_), "vx_ba_optimize_map");
    lap("optimize_map");
    if (stats_.status != 0) return;
    // scatter: Frame::SetPose / Landmark::SetPosition (local_ba.cpp:173,237)
    for (size_t i = 0; i < f.frames.size(); ++i) {
        const double* p = &f.kf_pose[7 * i];
        SE3d T;
        T.qx = p[0]; T.qy = p[1]; T.qz = p[2]; T.qw = p[3];
        T.tx = p[4]; T.ty = p[5]; T.tz = p[6];
        f.frames[i]->SetPose(T);
    }
    const size_t ahead = LmAhead();
    vxhost::Pool::Get().For(f.landmarks.size(), 1024, [&](size_t a, size_t b) {
        for (size_t i = a; i < b; ++i) {
            if (ahead && i + ahead < b) PrefetchObject(f.landmarks[i + ahead].get());
            f.landmarks[i]->SetPosition(Vec3d(f.lm_pos[3 * i], f.lm_pos[3 * i + 1], f.lm_pos[3 * i + 2]));
        }
    });
    lap("write-back");
}

}  // namespace visionx
