// feature.cpp — ORBExtractor / ORBMatcher / LocalBA adapters over the C ABI (see feature.h).
#include "visionx/feature.h"

#include "visionx/device_map.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <unordered_set>

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

FlatMap LocalBA::Flatten(const Map& map, const Frame::Ptr& ref_kf, int window_size) {
    FlatMap f;
    const auto& all = map.KeyFrames();
    if (all.empty()) return f;
    // SelectKeyFrames (local_ba.cpp:42-62)
    const uint64_t max_id = ref_kf ? ref_kf->Id() : all.rbegin()->first;
    const int window = std::max(1, window_size);
    for (auto it = all.rbegin(); it != all.rend() && (int)f.frames.size() < window; ++it) {
        if (it->first > max_id) continue;
        f.frames.push_back(it->second);
    }
    std::reverse(f.frames.begin(), f.frames.end());
    std::unordered_set<uint64_t> lm_ids;
    f.kf_feat_ptr.push_back(0);
    for (const auto& kf : f.frames) {
        const SE3d T = kf->Pose();
        f.kf_id.push_back(kf->Id());
        f.kf_pose.insert(f.kf_pose.end(), {T.qx, T.qy, T.qz, T.qw, T.tx, T.ty, T.tz});
        const auto cam = kf->GetCamera();
        f.kf_has_cam.push_back(cam ? 1 : 0);
        if (cam)
            f.kf_intr.insert(f.kf_intr.end(), {cam->fx(), cam->fy(), cam->cx(), cam->cy()});
        else
            f.kf_intr.insert(f.kf_intr.end(), {0.0, 0.0, 0.0, 0.0});
        for (const auto& feat : kf->Features()) {
            f.feat_uv.push_back(feat.position.x);
            f.feat_uv.push_back(feat.position.y);
            f.feat_lm_id.push_back(feat.landmark_id_);
            f.feat_flags.push_back((feat.has_landmark ? 1 : 0) | (feat.is_outlier ? 2 : 0));
            if (feat.has_landmark) lm_ids.insert(feat.landmark_id_);
        }
        f.kf_feat_ptr.push_back((int64_t)f.feat_uv.size() / 2);
    }
    std::vector<uint64_t> ids(lm_ids.begin(), lm_ids.end());
    std::sort(ids.begin(), ids.end());
    f.lm_obs_ptr.push_back(0);
    for (uint64_t id : ids) {
        auto lm = map.GetLandmark(id);
        if (!lm) continue;  // GetLandmark -> nullptr: treated as absent, like local_ba.cpp:96-97,135-136
        const Vec3d p = lm->Position();
        f.landmarks.push_back(lm);
        f.lm_id.push_back(id);
        f.lm_pos.insert(f.lm_pos.end(), {p.x, p.y, p.z});
        f.lm_bad.push_back(lm->IsBad() ? 1 : 0);
        for (const auto& [kid, fidx] : lm->Observations()) {
            f.obs_kf_id.push_back(kid);
            f.obs_feat_idx.push_back((uint64_t)fidx);
        }
        f.lm_obs_ptr.push_back((int64_t)f.obs_kf_id.size());
    }
    return f;
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

void LocalBA::OptimizeResident(const Frame::Ptr& ref_kf) {
    DeviceMap& dm = *dmap_;
    dm.Flush();
    vx_ctx* c = dm.context();
    const vx_ba_options o = VxOptions();
    check(c, vx_ba_optimize_dmap(c, dm.handle(), ref_kf ? ref_kf->Id() : 0, ref_kf ? 1 : 0, &o, &stats_),
          "vx_ba_optimize_dmap");
    int nk = 0, nl = 0;
    int rc = vx_ba_dmap_results(c, dm.handle(), (int)kf_rows_.size(), kf_rows_.data(), kf_out_.data(),
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
    // Frame::SetPose / Landmark::SetPosition (local_ba.cpp:173,237) on the host objects
    for (int i = 0; i < nk; ++i) {
        const double* p = &kf_out_[7 * (size_t)i];
        SE3d T;
        T.qx = p[0]; T.qy = p[1]; T.qz = p[2]; T.qw = p[3];
        T.tx = p[4]; T.ty = p[5]; T.tz = p[6];
        if (const auto& fr = dm.FrameAt(kf_rows_[i])) fr->SetPose(T);
    }
    for (int i = 0; i < nl; ++i)
        if (const auto& lm = dm.LandmarkAt(lm_rows_[i]))
            lm->SetPosition(Vec3d(lm_out_[3 * (size_t)i], lm_out_[3 * (size_t)i + 1], lm_out_[3 * (size_t)i + 2]));
}

void LocalBA::Optimize(const Map::Ptr& map, const Frame::Ptr& ref_kf) {
    stats_ = vx_ba_stats{};
    stats_.status = 1;
    if (!map) return;                                            // local_ba.cpp:67-69
    if (dmap_) {
        OptimizeResident(ref_kf);
        return;
    }
    FlatMap f = Flatten(*map, ref_kf, options_.window_size);
    if (f.frames.size() < 2) return;                            // local_ba.cpp:73-75
    const vx_ba_options o = VxOptions();
    vx_map_view v = f.view();
    vx_ctx* c = vxhost::ThreadContext();
    check(c, vx_ba_optimize_map(c, &v, ref_kf ? ref_kf->Id() : 0, ref_kf ? 1 : 0, &o, &stats_), "vx_ba_optimize_map");
    if (stats_.status != 0) return;
    // scatter: Frame::SetPose / Landmark::SetPosition (local_ba.cpp:173,237)
    for (size_t i = 0; i < f.frames.size(); ++i) {
        const double* p = &f.kf_pose[7 * i];
        SE3d T;
        T.qx = p[0]; T.qy = p[1]; T.qz = p[2]; T.qw = p[3];
        T.tx = p[4]; T.ty = p[5]; T.tz = p[6];
        f.frames[i]->SetPose(T);
    }
    for (size_t i = 0; i < f.landmarks.size(); ++i)
        f.landmarks[i]->SetPosition(Vec3d(f.lm_pos[3 * i], f.lm_pos[3 * i + 1], f.lm_pos[3 * i + 2]));
}

}  // namespace visionx
