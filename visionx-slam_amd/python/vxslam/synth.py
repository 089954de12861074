"""Seeded synthetic workloads shaped like the reference's inputs.

The TUM RGB-D sequences and real keyframe maps are not available offline, so every bench line
and parity test runs on data generated here:

* ``make_texture`` / ``make_frames`` — 640x480 (or any size) BGR8 frames cut from one textured
  plane with a small per-frame camera shift, uint16 depth (metres x 5000, tracking.cpp:603).
* ``make_ba_map`` — a flattened snapshot of ``visionx::Map`` (core/map/map.h:13-34,
  landmark.h:12-68, frame.h:16-64) holding a sliding BA window: keyframe poses ``T_cw`` on a
  smooth arc, landmarks observed by 2..5 consecutive keyframes, observations = true projection
  + N(0, 0.5 px) truncated at 1.5 px, poses perturbed by ~0.2 deg / 1 cm and landmarks by 1 cm.
  It also plants the corner cases LocalBA::Optimize handles (local_ba.cpp:66-249): older
  keyframes outside the window, single-observation landmarks (used by the pose stage only),
  bad landmarks, outlier features and features without a landmark.

Intrinsics default to 520.9/521.0/325.1/249.7 (apps/mono_demo.cpp:26-27).
"""
from __future__ import annotations

import numpy as np

FX, FY, CX, CY = 520.9, 521.0, 325.1, 249.7


# --------------------------------------------------------------------------- images
def _value_noise(rng, h, w, cell):
    gh, gw = h // cell + 3, w // cell + 3
    g = rng.random((gh, gw)).astype(np.float32)
    ys = np.arange(h, dtype=np.float32) / cell
    xs = np.arange(w, dtype=np.float32) / cell
    y0 = ys.astype(np.int64)
    x0 = xs.astype(np.int64)
    fy = (ys - y0)[:, None]
    fx = (xs - x0)[None, :]
    fy = fy * fy * (3 - 2 * fy)
    fx = fx * fx * (3 - 2 * fx)
    a = g[y0][:, x0]
    b = g[y0][:, x0 + 1]
    c = g[y0 + 1][:, x0]
    d = g[y0 + 1][:, x0 + 1]
    return (a * (1 - fx) + b * fx) * (1 - fy) + (c * (1 - fx) + d * fx) * fy


def make_texture(seed: int, h: int, w: int, n_rects: int | None = None) -> np.ndarray:
    """Gray uint8 texture: multi-octave value noise plus random rectangles (strong corners)."""
    rng = np.random.default_rng(seed)
    t = np.zeros((h, w), np.float32)
    for cell, amp in ((64, 0.45), (24, 0.3), (9, 0.2), (4, 0.12)):
        t += amp * _value_noise(rng, h, w, cell)
    t = (t - t.mean()) / (t.std() + 1e-6) * 38.0 + 110.0
    if n_rects is None:
        n_rects = max(8, (h * w) // 1500)
    for _ in range(n_rects):
        rh, rw = rng.integers(4, 40, size=2)
        y, x = rng.integers(0, h - rh), rng.integers(0, w - rw)
        t[y:y + rh, x:x + rw] += rng.choice([-1.0, 1.0]) * rng.uniform(35, 90)
    return np.clip(t, 0, 255).astype(np.uint8)


def make_frames(seed: int, n: int, h: int = 480, w: int = 640, step=(3, 2)) -> np.ndarray:
    """n BGR8 frames (n, h, w, 3) cut from one texture, shifted by ``step`` px per frame, with
    per-channel tint and per-frame noise."""
    rng = np.random.default_rng(seed + 1)
    sy, sx = step
    tex = make_texture(seed, h + abs(sy) * n + 8, w + abs(sx) * n + 8)
    out = np.empty((n, h, w, 3), np.uint8)
    for i in range(n):
        y0 = 4 + (sy * i if sy >= 0 else abs(sy) * (n - i))
        x0 = 4 + (sx * i if sx >= 0 else abs(sx) * (n - i))
        g = tex[y0:y0 + h, x0:x0 + w].astype(np.int16)
        noise = rng.integers(-2, 3, size=(h, w), dtype=np.int16)
        for c, tint in enumerate((-6, 0, 9)):
            out[i, :, :, c] = np.clip(g + noise + tint, 0, 255).astype(np.uint8)
    return out


def make_depth(seed: int, h: int = 480, w: int = 640) -> np.ndarray:
    """uint16 depth image, metres x 5000 in [0.5, 4] m (tracking.cpp:603 scale)."""
    rng = np.random.default_rng(seed + 7)
    d = 0.5 + 3.5 * _value_noise(rng, h, w, 80)
    return (d * 5000).astype(np.uint16)


# --------------------------------------------------------------------------- BA maps
def quat_from_rotvec(v):
    v = np.asarray(v, np.float64)
    th = np.linalg.norm(v, axis=-1, keepdims=True)
    half = 0.5 * th
    with np.errstate(invalid="ignore", divide="ignore"):
        k = np.where(th > 1e-12, np.sin(half) / th, 0.5)
    return np.concatenate([v * k, np.cos(half)], axis=-1)  # x y z w


def quat_to_mat(q):
    x, y, z, w = np.moveaxis(np.asarray(q, np.float64), -1, 0)
    return np.stack([
        np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)], -1),
        np.stack([2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)], -1),
        np.stack([2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)], -1),
    ], -2)


def quat_mul(a, b):
    ax, ay, az, aw = np.moveaxis(a, -1, 0)
    bx, by, bz, bw = np.moveaxis(b, -1, 0)
    return np.stack([aw * bx + ax * bw + ay * bz - az * by,
                     aw * by + ay * bw + az * bx - ax * bz,
                     aw * bz + az * bw + ax * by - ay * bx,
                     aw * bw - ax * bx - ay * by - az * bz], -1)


class BAMap(dict):
    """Flattened visionx::Map snapshot: a dict of numpy arrays plus scalars."""

    @property
    def n_kf(self):
        return int(self["kf_id"].shape[0])

    @property
    def n_lm(self):
        return int(self["lm_id"].shape[0])

    @property
    def n_obs(self):
        return int(self["obs_kf_id"].shape[0])

    def copy(self):
        return BAMap({k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in self.items()})


def make_ba_map(seed: int, n_kf: int = 10, n_lm: int = 2000, *, n_old_kf: int = 2,
                extra_feats_per_kf: int = 40, frac_single: float = 0.03, frac_bad: float = 0.01,
                frac_outlier: float = 0.01, noise_px: float = 0.5, noise_clip: float = 1.5,
                rot_deg: float = 0.2, trans_m: float = 0.01, lm_sigma: float = 0.01,
                width: int = 640, height: int = 480, intr=(FX, FY, CX, CY),
                n_streams: int = 1, cross_frac: float = 0.0) -> BAMap:
    """A BA window of ``n_kf`` keyframes (+ ``n_old_kf`` older keyframes outside the window) and
    ``n_lm`` landmarks.  ``n_streams`` > 1 builds a multi-camera rig (configs C5): keyframes are
    split into streams, each stream observing its own landmark subset.  ``cross_frac`` > 0 makes
    the rig one body: that fraction of the landmarks lies in the field of view the stream shares
    with its neighbour (the next camera, 360 / n_streams degrees further round the rig) and is
    observed by both, so the streams' keyframes form ONE covisibility component (config C5's
    global window; with 0 every stream is a component of its own).

    Returns a BAMap with the vx_map_view / orc_map_view fields.  Landmark ids are random uint64,
    keyframe ids increase with time but are not contiguous."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = intr
    K_all = n_kf + n_old_kf
    per_stream = K_all // n_streams
    assert per_stream * n_streams == K_all, "n_kf + n_old_kf must divide by n_streams"

    # ---- ground-truth camera trajectory (camera-to-world), per stream an offset arc
    idx = np.arange(K_all)
    stream = idx % n_streams
    tpos = idx // n_streams  # time index inside a stream
    yaw = np.deg2rad(0.35) * tpos + stream * (2 * np.pi / max(n_streams, 1))
    centres = np.stack([0.04 * tpos * np.cos(yaw) + 0.3 * stream,
                        0.01 * np.sin(tpos / 5.0),
                        0.04 * tpos * np.sin(yaw) * 0.2], -1)
    q_wc = quat_from_rotvec(np.stack([np.deg2rad(0.1) * np.sin(tpos / 7.0), yaw, np.zeros(K_all)], -1))
    R_wc = quat_to_mat(q_wc)
    R_cw = np.transpose(R_wc, (0, 2, 1))
    t_cw = -np.einsum("kij,kj->ki", R_cw, centres)
    q_cw = q_wc * np.array([-1, -1, -1, 1.0])

    # ---- landmarks: each observed by L in {2..5} consecutive KFs of one stream
    lm_stream = rng.integers(0, n_streams, size=n_lm)
    L = np.minimum(rng.integers(2, 6, size=n_lm), per_stream)
    n_single = int(round(frac_single * n_lm))
    L[:n_single] = 1  # depth landmarks observed once (pose stage only)
    start = rng.integers(0, per_stream, size=n_lm)
    start = np.minimum(start, per_stream - L)
    start = np.maximum(start, 0)
    anchor_t = start + L // 2
    anchor = anchor_t * n_streams + lm_stream
    u = rng.uniform(20, width - 20, size=n_lm)
    v = rng.uniform(20, height - 20, size=n_lm)
    z = rng.uniform(1.0, 5.0, size=n_lm)
    pc = np.stack([(u - cx) / fx * z, (v - cy) / fy * z, z], -1)
    p_true = np.einsum("nij,nj->ni", R_wc[anchor], pc) + centres[anchor]

    # observations
    obs_lm = np.repeat(np.arange(n_lm), L)
    within = np.arange(obs_lm.shape[0]) - np.repeat(np.cumsum(L) - L, L)
    obs_t = start[obs_lm] + within
    obs_kf = obs_t * n_streams + lm_stream[obs_lm]
    if cross_frac > 0 and n_streams > 1:
        # shared landmarks: 15-28 degrees off the anchor camera's axis towards the next camera
        # (its yaw is 360 / n_streams degrees larger), 2-5 m deep, observed by that camera too at
        # the same times wherever the point projects inside its image (separate generator, so the
        # maps of cross_frac = 0 are unchanged)
        rc = np.random.default_rng(seed ^ 0xC5C5C5)
        cand = np.nonzero(L >= 2)[0]
        sh = np.sort(rc.choice(cand, size=min(len(cand), int(round(cross_frac * n_lm))), replace=False))
        th = np.deg2rad(rc.uniform(15.0, 28.0, size=len(sh)))
        zs = rc.uniform(2.0, 5.0, size=len(sh))
        u[sh] = cx + np.tan(th) * fx
        v[sh] = rc.uniform(60, height - 60, size=len(sh))
        z[sh] = zs
        pcs_a = np.stack([(u[sh] - cx) / fx * zs, (v[sh] - cy) / fy * zs, zs], -1)
        p_true[sh] = np.einsum("nij,nj->ni", R_wc[anchor[sh]], pcs_a) + centres[anchor[sh]]
        x_lm = np.repeat(sh, L[sh])
        x_t = start[x_lm] + (np.arange(len(x_lm)) - np.repeat(np.cumsum(L[sh]) - L[sh], L[sh]))
        x_kf = x_t * n_streams + (lm_stream[x_lm] + 1) % n_streams
        pc2 = np.einsum("oij,oj->oi", R_cw[x_kf], p_true[x_lm]) + t_cw[x_kf]
        z2 = np.where(pc2[:, 2] > 0.3, pc2[:, 2], 1.0)
        u2, v2 = fx * pc2[:, 0] / z2 + cx, fy * pc2[:, 1] / z2 + cy
        vis = (pc2[:, 2] > 0.3) & (u2 > 20) & (u2 < width - 20) & (v2 > 20) & (v2 < height - 20)
        obs_lm = np.concatenate([obs_lm, x_lm[vis]])
        obs_t = np.concatenate([obs_t, x_t[vis]])
        obs_kf = np.concatenate([obs_kf, x_kf[vis]])
        L = np.bincount(obs_lm, minlength=n_lm)
    pcs = np.einsum("oij,oj->oi", R_cw[obs_kf], p_true[obs_lm]) + t_cw[obs_kf]
    uv = np.stack([fx * pcs[:, 0] / pcs[:, 2] + cx, fy * pcs[:, 1] / pcs[:, 2] + cy], -1)
    nz = np.clip(rng.normal(0, noise_px, size=uv.shape), -noise_clip, noise_clip)
    uv = uv + nz

    # ---- features per KF: observations (shuffled) + features without a landmark
    n_obs = obs_lm.shape[0]
    order = np.lexsort((rng.random(n_obs), obs_kf))
    feat_kf = obs_kf[order]
    feat_uv = uv[order]
    feat_lm = obs_lm[order]
    counts = np.bincount(feat_kf, minlength=K_all)
    extra = np.full(K_all, extra_feats_per_kf)
    # interleave: per KF, obs features then extra features
    tot = counts + extra
    feat_ptr = np.zeros(K_all + 1, np.int64)
    feat_ptr[1:] = np.cumsum(tot)
    nf = int(feat_ptr[-1])
    f_uv = rng.uniform([0, 0], [width, height], size=(nf, 2))
    f_lm_idx = np.full(nf, -1, np.int64)
    obs_start = np.zeros(K_all + 1, np.int64)
    obs_start[1:] = np.cumsum(counts)
    pos_in_kf = np.arange(n_obs) - obs_start[feat_kf]
    fpos = feat_ptr[feat_kf] + pos_in_kf
    f_uv[fpos] = feat_uv
    f_lm_idx[fpos] = feat_lm
    flags = (f_lm_idx >= 0).astype(np.uint8)
    n_out = int(round(frac_outlier * n_obs))
    if n_out:
        flags[rng.choice(fpos, size=n_out, replace=False)] |= 2
    # a few features pointing at ids that are not in the map (GetLandmark -> nullptr)
    lm_ids = rng.choice(np.iinfo(np.int64).max, size=n_lm + 16, replace=False).astype(np.uint64)
    missing_ids = lm_ids[n_lm:]
    lm_ids = lm_ids[:n_lm]
    f_lm_id = np.zeros(nf, np.uint64)
    f_lm_id[fpos] = lm_ids[feat_lm]
    no_lm = np.nonzero(f_lm_idx < 0)[0]
    if no_lm.size >= 8:
        ghosts = rng.choice(no_lm, size=8, replace=False)
        flags[ghosts] = 1
        f_lm_id[ghosts] = missing_ids[:8]

    # landmark observation lists (kf_id, feature idx) — ordered by KF
    kf_ids = (np.arange(K_all, dtype=np.uint64) * 3 + 7).astype(np.uint64)
    lm_order = np.lexsort((obs_kf, obs_lm))
    o_lm = obs_lm[lm_order]
    o_kf = obs_kf[lm_order]
    # feature index of each (lm, kf) observation
    inv = np.empty(n_obs, np.int64)
    inv[order] = np.arange(n_obs)  # obs -> position in sorted feature order
    o_feat = pos_in_kf[inv[lm_order]]
    lm_obs_ptr = np.zeros(n_lm + 1, np.int64)
    lm_obs_ptr[1:] = np.cumsum(L)

    lm_bad = np.zeros(n_lm, np.uint8)
    n_bad = int(round(frac_bad * n_lm))
    if n_bad:
        lm_bad[rng.choice(n_lm, size=n_bad, replace=False)] = 1

    # ---- perturbed initial state
    dq = quat_from_rotvec(rng.normal(0, np.deg2rad(rot_deg) / np.sqrt(3), size=(K_all, 3)))
    q0 = quat_mul(dq, q_cw)
    q0 /= np.linalg.norm(q0, axis=-1, keepdims=True)
    t0 = t_cw + rng.normal(0, trans_m / np.sqrt(3), size=(K_all, 3))
    p0 = p_true + rng.normal(0, lm_sigma / np.sqrt(3), size=(n_lm, 3))

    m = BAMap()
    m["kf_id"] = kf_ids
    m["kf_pose"] = np.ascontiguousarray(np.concatenate([q0, t0], -1))
    m["kf_intr"] = np.tile(np.array(intr, np.float64), (K_all, 1))
    m["kf_has_cam"] = np.ones(K_all, np.uint8)
    m["kf_feat_ptr"] = feat_ptr
    m["feat_uv"] = np.ascontiguousarray(f_uv)
    m["feat_lm_id"] = f_lm_id
    m["feat_flags"] = flags
    m["lm_id"] = lm_ids
    m["lm_pos"] = np.ascontiguousarray(p0)
    m["lm_bad"] = lm_bad
    m["lm_obs_ptr"] = lm_obs_ptr
    m["obs_kf_id"] = kf_ids[o_kf].astype(np.uint64)
    m["obs_feat_idx"] = o_feat.astype(np.uint64)
    m["ref_kf_id"] = int(kf_ids[-1])
    m["window"] = n_kf
    return m


def ba_config(name: str):
    """(n_kf, n_lm, n_streams) of the BASELINE.json configs."""
    return {"C2": (10, 2000, 1), "C3": (50, 20000, 1), "C4": (100, 50000, 1),
            "C5": (200, 100000, 8)}[name]


def make_keyframe_pair(seed: int, n: int = 2000, *, width: int = 640, height: int = 480, intr=(FX, FY, CX, CY),
                       baseline_m: float = 0.08, yaw_deg: float = 1.5, noise_px: float = 0.3,
                       frac_has: float = 0.1, frac_bad_match: float = 0.1, frac_dup_train: float = 0.03,
                       depth_type: str = "u16"):
    """Two keyframes seeing a common set of points, for Tracking::CreateKeyFrame's landmark
    creation (tracking.cpp:577-580): per frame Feature positions and has_landmark flags, T_cw poses,
    a depth image of the second frame (TUM u16 metres * 5000, with holes and out-of-range pixels)
    and the match list Match(last, curr) would return (query = last frame, unique queries; some
    wrong / duplicated train indices).  Returns a dict of numpy arrays."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = intr
    # points in front of camera 1
    u = rng.uniform(5, width - 5, n)
    v = rng.uniform(5, height - 5, n)
    z = rng.uniform(0.6, 6.0, n)
    pc1 = np.stack([(u - cx) / fx * z, (v - cy) / fy * z, z], -1)
    q1 = quat_from_rotvec(rng.normal(0, 0.02, 3))
    t1 = rng.normal(0, 0.1, 3)
    R1 = quat_to_mat(q1)
    pw = (pc1 - t1) @ R1  # R1^T (pc - t)
    q12 = quat_from_rotvec(np.array([0.0, np.deg2rad(yaw_deg), 0.0]))
    q2 = quat_mul(q12, q1)
    q2 /= np.linalg.norm(q2)
    R2 = quat_to_mat(q2)
    c1w = -R1.T @ t1
    c2w = c1w + np.array([baseline_m, 0.01, 0.005])
    t2 = -R2 @ c2w
    pc2 = pw @ R2.T + t2
    uv1 = np.stack([fx * pc1[:, 0] / pc1[:, 2] + cx, fy * pc1[:, 1] / pc1[:, 2] + cy], -1)
    uv2 = np.stack([fx * pc2[:, 0] / pc2[:, 2] + cx, fy * pc2[:, 1] / pc2[:, 2] + cy], -1)
    uv1 += rng.normal(0, noise_px, uv1.shape)
    uv2 += rng.normal(0, noise_px, uv2.shape)
    # frame 2 feature order is a permutation of frame 1's
    perm = rng.permutation(n)
    uv2 = uv2[perm]
    inv = np.empty(n, np.int64)
    inv[perm] = np.arange(n)  # point i is feature inv[i] of frame 2
    has1 = (rng.random(n) < frac_has).astype(np.uint8)
    has2 = (rng.random(n) < frac_has).astype(np.uint8)
    q_idx = np.sort(rng.choice(n, size=int(0.8 * n), replace=False))
    t_idx = inv[q_idx].copy()
    bad = rng.random(q_idx.size) < frac_bad_match
    t_idx[bad] = rng.integers(0, n, bad.sum())
    dup = rng.random(q_idx.size) < frac_dup_train
    dup_src = rng.integers(0, q_idx.size, dup.sum())
    t_idx[dup] = t_idx[dup_src]
    matches = np.zeros(q_idx.size, np.dtype([("query_idx", "<i4"), ("train_idx", "<i4"), ("distance", "<f4")]))
    matches["query_idx"] = q_idx
    matches["train_idx"] = t_idx
    matches["distance"] = rng.integers(0, 64, q_idx.size)
    # depth image of frame 2: smooth field, holes (0) and out-of-range pixels
    yy, xx = np.mgrid[0:height, 0:width]
    dm = 2.5 + 1.5 * np.sin(xx / 57.0) * np.cos(yy / 43.0) + 0.002 * xx
    dm[rng.random(dm.shape) < 0.05] = 0.0
    dm[rng.random(dm.shape) < 0.02] = 0.05
    dm[rng.random(dm.shape) < 0.02] = 12.0
    if depth_type == "u16":
        depth = np.round(dm * 5000.0).clip(0, 65535).astype(np.uint16)
    elif depth_type == "f32":
        depth = dm.astype(np.float32)
    else:
        depth = dm.astype(np.float64)
    pose1 = np.concatenate([q1, t1])
    pose2 = np.concatenate([q2, t2])
    return {"uv1": np.ascontiguousarray(uv1), "has1": has1, "uv2": np.ascontiguousarray(uv2), "has2": has2,
            "intr": np.array(intr, np.float64), "pose1": pose1, "pose2": pose2, "matches": matches,
            "depth": np.ascontiguousarray(depth), "pw_true": pw, "inv": inv}


def make_pnp_problem(seed: int, n: int = 1000, *, outlier_frac: float = 0.3, noise_px: float = 0.5,
                     width: int = 640, height: int = 480, intr=(FX, FY, CX, CY), z_range=(1.0, 6.0)):
    """3D-2D correspondences as Tracking::TrackWithPnP builds them (tracking.cpp:364-401:
    cv::Point3f landmark positions, cv::Point2f current-frame feature positions): points seen by a
    camera at a random T_cw, pixel noise, a fraction of wrong matches (random pixels).  Returns a
    dict: obj (n x 3 float32), img (n x 2 float32), intr, pose (T_cw qx qy qz qw tx ty tz),
    R, t, outlier (bool per correspondence)."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = intr
    u = rng.uniform(0, width, n)
    v = rng.uniform(0, height, n)
    z = rng.uniform(z_range[0], z_range[1], n)
    pc = np.stack([(u - cx) / fx * z, (v - cy) / fy * z, z], -1)
    q = quat_from_rotvec(rng.normal(0, 0.3, 3))
    R = quat_to_mat(q)
    t = rng.normal(0, 0.5, 3)
    pw = (pc - t) @ R  # R^T (pc - t)
    uv = np.stack([u, v], -1) + rng.normal(0, noise_px, (n, 2))
    out = rng.random(n) < outlier_frac
    uv[out] = np.stack([rng.uniform(0, width, out.sum()), rng.uniform(0, height, out.sum())], -1)
    if q[3] < 0:
        q = -q
    return {"obj": pw.astype(np.float32), "img": uv.astype(np.float32), "intr": np.array(intr, np.float64),
            "pose": np.concatenate([q, t]), "R": R, "t": t, "outlier": out}


def make_two_view(seed: int, n: int = 1000, *, outlier_frac: float = 0.3, noise_px: float = 0.5,
                  width: int = 640, height: int = 480, intr=(FX, FY, CX, CY), baseline_m: float = 0.15,
                  rot_deg: float = 3.0, z_range=(1.0, 6.0)):
    """Matched pixel pairs as Tracking::EstimatePoseByEssential builds them (tracking.cpp:506-514:
    cv::Point2f of the last and the current frame's features): points seen by both cameras, pixel
    noise, a fraction of wrong matches.  Returns pts_last, pts_curr (n x 2 float32), intr, the true
    T_cl (R, t with x_curr = R x_last + t; t unit-normalised copy in t_dir) and the outlier flags."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = intr
    q = quat_from_rotvec(rng.normal(0, 1, 3) * np.deg2rad(rot_deg) / np.sqrt(3))
    R = quat_to_mat(q)
    d = rng.normal(0, 1, 3)
    d[2] *= 0.3
    t = baseline_m * d / np.linalg.norm(d)
    pts_last, pts_curr = [], []
    while not pts_last or sum(len(a) for a in pts_last) < n:
        u = rng.uniform(0, width, 2 * n)
        v = rng.uniform(0, height, 2 * n)
        z = rng.uniform(z_range[0], z_range[1], 2 * n)
        p1 = np.stack([(u - cx) / fx * z, (v - cy) / fy * z, z], -1)
        p2 = p1 @ R.T + t
        u2 = fx * p2[:, 0] / p2[:, 2] + cx
        v2 = fy * p2[:, 1] / p2[:, 2] + cy
        ok = (p2[:, 2] > 0.1) & (u2 >= 0) & (u2 < width) & (v2 >= 0) & (v2 < height)
        pts_last.append(np.stack([u, v], -1)[ok])
        pts_curr.append(np.stack([u2, v2], -1)[ok])
    a = np.concatenate(pts_last)[:n] + rng.normal(0, noise_px, (n, 2))
    b = np.concatenate(pts_curr)[:n] + rng.normal(0, noise_px, (n, 2))
    out = rng.random(n) < outlier_frac
    b[out] = np.stack([rng.uniform(0, width, out.sum()), rng.uniform(0, height, out.sum())], -1)
    return {"pts_last": a.astype(np.float32), "pts_curr": b.astype(np.float32), "intr": np.array(intr, np.float64),
            "R": R, "t": t, "t_dir": t / np.linalg.norm(t), "outlier": out}
