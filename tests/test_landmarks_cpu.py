"""Keyframe-insertion landmark creation: CPU checks of the restatement
(oracle/landmark_oracle.cpp) of Tracking::CreateLandmarksFromDepth (tracking.cpp:586-650) and
TriangulateWithLastKeyFrame / TriangulatePoint (tracking.cpp:856-945).

TriangulatePoint's SVD is Eigen::JacobiSVD in the reference (not installed here): its point is
pinned against numpy's LAPACK SVD of the same 4x4 DLT matrix, and against ground truth on
noise-free data."""
import numpy as np

from vxslam import synth


def _R(q):
    return synth.quat_to_mat(np.asarray(q, float))


def _dlt_numpy(d, k):
    """Point of match k from numpy's SVD of the reference's DLT matrix (tracking.cpp:931-945)."""
    fx, fy, cx, cy = d["intr"]
    K = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1.0]])
    P1 = K @ np.hstack([_R(d["pose1"][:4]), d["pose1"][4:, None]])
    P2 = K @ np.hstack([_R(d["pose2"][:4]), d["pose2"][4:, None]])
    q, t = d["matches"]["query_idx"][k], d["matches"]["train_idx"][k]
    x1, x2 = d["uv1"][q], d["uv2"][t]
    A = np.stack([x1[0] * P1[2] - P1[0], x1[1] * P1[2] - P1[1], x2[0] * P2[2] - P2[0], x2[1] * P2[2] - P2[1]])
    X = np.linalg.svd(A)[2][3]
    return X[:3] / X[3]


def test_triangulated_points_match_lapack_svd(oracle):
    d = synth.make_keyframe_pair(3, 600)
    idx, pw = oracle.triangulate(d)
    ks = np.nonzero(idx >= 0)[0]
    assert len(ks) > 100
    for k in ks:
        ref = _dlt_numpy(d, k)
        assert np.abs(pw[idx[k]] - ref).max() <= 1e-9 * np.abs(ref).max()


def test_triangulation_noise_free_recovers_points(oracle):
    d = synth.make_keyframe_pair(4, 500, noise_px=0.0, frac_bad_match=0.0, frac_dup_train=0.0, frac_has=0.0)
    idx, pw = oracle.triangulate(d)
    q = d["matches"]["query_idx"][idx >= 0]
    assert len(q) > 50
    assert np.abs(pw - d["pw_true"][q]).max() <= 1e-7


def test_triangulation_sequential_semantics(oracle):
    """has_landmark features are skipped, and a train feature is used by its first passing match
    only (the reference marks features as it goes, tracking.cpp:917-925)."""
    d = synth.make_keyframe_pair(5, 800, frac_dup_train=0.2)
    idx, pw = oracle.triangulate(d)
    m = d["matches"]
    made = idx >= 0
    assert not d["has1"][m["query_idx"][made]].any() and not d["has2"][m["train_idx"][made]].any()
    t = m["train_idx"][made]
    assert len(np.unique(t)) == len(t)
    assert (idx[made] == np.arange(made.sum())).all()  # numbered in match order
    # angle gate: a huge minimum angle creates nothing, a zero one creates at least as many
    assert len(oracle.triangulate(d, min_angle_deg=90.0)[1]) == 0
    assert len(oracle.triangulate(d, min_angle_deg=0.0)[1]) >= len(pw)


def _depth_numpy(uv, has, depth, intr, pose):
    fx, fy, cx, cy = intr
    R, t = _R(pose[:4]), pose[4:]
    out = {}
    for i in range(len(has)):
        if has[i]:
            continue
        u, v = int(uv[i, 0] + 0.5), int(uv[i, 1] + 0.5)
        if not (0 <= u < depth.shape[1] and 0 <= v < depth.shape[0]):
            continue
        if depth.dtype == np.uint16:
            if depth[v, u] == 0:
                continue
            z = float(depth[v, u]) / 5000.0
        else:
            z = float(depth[v, u])
        if z < 0.1 or z > 10.0:
            continue
        pc = np.array([(uv[i, 0] - cx) / fx * z, (uv[i, 1] - cy) / fy * z, z])
        out[i] = R.T @ (pc - t)
    return out


def test_depth_landmarks_match_numpy(oracle):
    for dt in ("u16", "f32", "f64"):
        d = synth.make_keyframe_pair(6, 1500, depth_type=dt)
        uv = d["uv2"].copy()
        uv[:20] = [[-0.7, 10.0]] * 20  # (int)(x + 0.5) truncates toward zero: column 0 is valid
        uv[20:30] = [[700.0, 10.0]] * 10  # outside the image
        idx, pw = oracle.depth_landmarks(uv, d["has2"], d["depth"], d["intr"], d["pose2"])
        ref = _depth_numpy(uv, d["has2"], d["depth"], d["intr"], d["pose2"])
        assert sorted(ref) == list(np.nonzero(idx >= 0)[0])
        for i, p in ref.items():
            assert np.abs(pw[idx[i]] - p).max() <= 1e-12 * max(1.0, np.abs(p).max())
    idx, pw = oracle.depth_landmarks(d["uv2"], d["has2"], None, d["intr"], d["pose2"])  # Depth().empty()
    assert (idx == -1).all() and len(pw) == 0
