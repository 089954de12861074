"""ctypes binding of oracle/build/liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, as the
checker / CPU baseline.  See oracle.h for what is restated and how it is pinned.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# $VX_ORACLE_LIB: another build of the same sources (the ASan/UBSan one, tests/test_sanitizers.py)
LIB_PATH = os.environ.get("VX_ORACLE_LIB") or os.path.join(HERE, "build", "liboracle.so")
PATTERN_PATH = os.path.join(os.path.dirname(HERE), "tests", "golden", "orb_bit_pattern_31.txt")

ORDER_STL, ORDER_RASTER = 0, 1

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("response", "<f4"), ("angle", "<f4"),
                           ("octave", "<i4")])
MATCH_DTYPE = np.dtype([("query_idx", "<i4"), ("train_idx", "<i4"), ("distance", "<f4")])


def build():
    subprocess.run(["make", "-s", "-C", HERE, "asan" if os.environ.get("VX_ORACLE_LIB") else "all"], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _lib.orc_harris.restype = C.c_float
        _lib.orc_ic_angle.restype = C.c_float
        _lib.orc_fast_atan2.restype = C.c_float
        _lib.orc_fast_atan2.argtypes = [C.c_float, C.c_float]
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def load_pattern() -> np.ndarray:
    rows = [l.split() for l in open(PATTERN_PATH) if not l.startswith("#")]
    return np.array(rows, dtype=np.int32).reshape(-1)


def quotas(n, scale=1.2, levels=8):
    q = np.zeros(levels, np.int32)
    lib().orc_orb_quotas(n, C.c_float(scale), levels, _p(q))
    return q


def level_sizes(w, h, scale=1.2, levels=8):
    lw = np.zeros(levels, np.int32)
    lh = np.zeros(levels, np.int32)
    s = np.zeros(levels, np.float32)
    lib().orc_orb_level_sizes(w, h, C.c_float(scale), levels, _p(lw), _p(lh), _p(s))
    return lw, lh, s


def pyramid(img, scale=1.2, levels=8):
    img = np.ascontiguousarray(img)
    h, w = img.shape[:2]
    ch = 1 if img.ndim == 2 else img.shape[2]
    lw, lh, _ = level_sizes(w, h, scale, levels)
    tot = int((lw.astype(np.int64) * lh).sum())
    out = np.zeros(tot, np.uint8)
    rc = lib().orc_orb_pyramid(_p(img), w, h, ch, C.c_int64(img.strides[0]), C.c_float(scale),
                               levels, _p(out), C.c_int64(tot))
    assert rc == 0
    res, off = [], 0
    for a, b in zip(lw, lh):
        res.append(out[off:off + a * b].reshape(b, a))
        off += a * b
    return res


def fast_nms(level, threshold=20):
    level = np.ascontiguousarray(level, np.uint8)
    h, w = level.shape
    cap = w * h // 2 + 16
    xys = np.zeros((cap, 3), np.int32)
    n = C.c_int(0)
    rc = lib().orc_fast_nms(_p(level), w, h, threshold, _p(xys), cap, C.byref(n))
    assert rc == 0
    return xys[:n.value].copy()


def fast_scores(level, threshold=20):
    level = np.ascontiguousarray(level, np.uint8)
    out = np.zeros_like(level)
    lib().orc_fast_scores(_p(level), level.shape[1], level.shape[0], threshold, _p(out))
    return out


def harris(level, x, y):
    level = np.ascontiguousarray(level, np.uint8)
    return lib().orc_harris(_p(level), level.shape[1], level.shape[0], int(x), int(y))


def ic_angle(level, x, y):
    level = np.ascontiguousarray(level, np.uint8)
    return lib().orc_ic_angle(_p(level), level.shape[1], level.shape[0], int(x), int(y))


def fast_atan2(y, x):
    return lib().orc_fast_atan2(float(y), float(x))


def blur_level(level):
    level = np.ascontiguousarray(level, np.uint8)
    out = np.zeros_like(level)
    lib().orc_blur_level(_p(level), level.shape[1], level.shape[0], _p(out))
    return out


def orb_extract(img, n_features=1000, scale=1.2, levels=8, fast_threshold=20,
                order=ORDER_STL, pattern=None):
    img = np.ascontiguousarray(img)
    h, w = img.shape[:2]
    ch = 1 if img.ndim == 2 else img.shape[2]
    pat = load_pattern() if pattern is None else np.ascontiguousarray(pattern, np.int32)
    cap = 4 * n_features + 64
    kps = np.zeros(cap, KEYPOINT_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    n = C.c_int(0)
    rc = lib().orc_orb_extract(_p(img), w, h, ch, C.c_int64(img.strides[0]), n_features,
                               C.c_float(scale), levels, fast_threshold, _p(pat), order, _p(kps),
                               _p(desc), cap, C.byref(n))
    assert rc == 0, rc
    return kps[:n.value].copy(), desc[:n.value].copy()


def orb_stages(img, n_features=1000, scale=1.2, levels=8, fast_threshold=20, order=ORDER_STL):
    """Per-level stage lists of one extraction (orc_orb_stages): a list of dicts with keys
    fast (x, y, score; before runByImageBorder), cand (x, y, score, harris; raster order after the
    border), keep1 / fin (indices into cand: the two retainBest outputs, in output order)."""
    img = np.ascontiguousarray(img)
    h, w = img.shape[:2]
    ch = 1 if img.ndim == 2 else img.shape[2]
    cap = w * h // 2 + 64
    counts = np.zeros(4 * levels, np.int32)
    fast = np.zeros((cap, 3), np.int32)
    cand = np.zeros((cap, 4), np.float32)
    k1 = np.zeros(cap, np.int32)
    fin = np.zeros(cap, np.int32)
    rc = lib().orc_orb_stages(_p(img), w, h, ch, C.c_int64(img.strides[0]), n_features, C.c_float(scale), levels,
                              fast_threshold, order, _p(counts), _p(fast), _p(cand), _p(k1), _p(fin), C.c_int64(cap))
    assert rc == 0, rc
    out, o = [], np.zeros(4, np.int64)
    for l in range(levels):
        c = counts[4 * l:4 * l + 4]
        out.append(dict(fast=fast[o[0]:o[0] + c[0]].copy(), cand=cand[o[1]:o[1] + c[1]].copy(),
                        keep1=k1[o[2]:o[2] + c[2]].copy(), fin=fin[o[3]:o[3] + c[3]].copy()))
        o += c
    return out


def retain_best_keys(keys, npts):
    """retainBest over bare u32 keys with the real std::nth_element / std::partition: kept indices
    in the library's order."""
    keys = np.ascontiguousarray(keys, np.uint32)
    out = np.zeros(max(len(keys), 1), np.int32)
    n = C.c_int(0)
    assert lib().orc_retain_best_keys(_p(keys), len(keys), int(npts), _p(out), C.byref(n)) == 0
    return out[:n.value].copy()


def antiqsort(n, nth):
    """McIlroy's adversary against std::nth_element(.., nth, .., greater): killer keys (u32)."""
    out = np.zeros(n, np.uint32)
    assert lib().orc_antiqsort(int(n), int(nth), _p(out)) == 0
    return out


def knn2(q, t):
    q = np.ascontiguousarray(q, np.uint8)
    t = np.ascontiguousarray(t, np.uint8)
    idx = np.zeros((len(q), 2), np.int32)
    dist = np.zeros((len(q), 2), np.int32)
    lib().orc_knn2(_p(q), len(q), _p(t), len(t), _p(idx), _p(dist))
    return idx, dist


def match(q, t, ratio=0.8):
    q = np.ascontiguousarray(q, np.uint8)
    t = np.ascontiguousarray(t, np.uint8)
    out = np.zeros(max(len(q), 1), MATCH_DTYPE)
    n = C.c_int(0)
    rc = lib().orc_match_knn2_ratio(_p(q), len(q), _p(t), len(t), C.c_float(ratio), _p(out),
                                    len(out), C.byref(n))
    assert rc == 0
    return out[:n.value].copy()


# ---------------------------------------------------------------------------- LocalBA
class MapView(C.Structure):
    _fields_ = [("n_kf", C.c_int32), ("kf_id", C.c_void_p), ("kf_pose", C.c_void_p),
                ("kf_intr", C.c_void_p), ("kf_has_cam", C.c_void_p), ("kf_feat_ptr", C.c_void_p),
                ("feat_uv", C.c_void_p), ("feat_lm_id", C.c_void_p), ("feat_flags", C.c_void_p),
                ("n_lm", C.c_int32), ("lm_id", C.c_void_p), ("lm_pos", C.c_void_p),
                ("lm_bad", C.c_void_p), ("lm_obs_ptr", C.c_void_p), ("obs_kf_id", C.c_void_p),
                ("obs_feat_idx", C.c_void_p)]


class BAOptions(C.Structure):
    _fields_ = [("window_size", C.c_int32), ("max_iterations", C.c_int32),
                ("min_pose_observations", C.c_int32), ("min_point_observations", C.c_int32),
                ("huber_delta", C.c_double), ("max_reproj_error", C.c_double)]


class BAStats(C.Structure):
    _fields_ = [("iterations", C.c_int32), ("n_window_kf", C.c_int32), ("n_landmarks", C.c_int32),
                ("cost", C.c_double * 16), ("obs", C.c_int32 * 16), ("gate_margin", C.c_double),
                ("status", C.c_int32)]


def map_view(m, cls=MapView):
    """Build a MapView over the arrays of a synth.BAMap (kf_pose / lm_pos are updated in place)."""
    keys = [f[0] for f in cls._fields_]
    v = cls()
    for k in keys:
        if k in ("n_kf", "n_lm"):
            setattr(v, k, int(m["kf_id" if k == "n_kf" else "lm_id"].shape[0]))
        else:
            a = m[k]
            assert a.flags["C_CONTIGUOUS"], k
            setattr(v, k, a.ctypes.data)
    return v


def ba_options(window=5, iters=5, min_pose=20, min_point=2, huber=5.0, max_err=5.0):
    return BAOptions(window, iters, min_pose, min_point, huber, max_err)


def ba_optimize(m, opts=None, ref_kf_id=None):
    """Runs the oracle LocalBA on a synth.BAMap in place; returns BAStats."""
    if opts is None:
        opts = ba_options(window=m.get("window", 5))
    v = map_view(m)
    st = BAStats()
    ref = m.get("ref_kf_id") if ref_kf_id is None else ref_kf_id
    has_ref = 0 if ref is None else 1
    rc = lib().orc_ba_optimize_map(C.byref(v), C.c_uint64(0 if ref is None else int(ref)), has_ref,
                                   C.byref(opts), C.byref(st))
    assert rc == 0
    return st


def ba_last_timing():
    """(setup_s, iterations_s) of the last ba_optimize: window / landmark-set selection
    (local_ba.cpp:66-108) and the alternating iterations (:110-248)."""
    out = (C.c_double * 2)()
    lib().orc_ba_last_timing(out)
    return out[0], out[1]


# ---------------------------------------------------------------------------- Schur-complement BA
class SBAOptions(C.Structure):
    _fields_ = [("window_size", C.c_int32), ("max_iterations", C.c_int32),
                ("min_point_observations", C.c_int32), ("fixed_keyframes", C.c_int32),
                ("huber_delta", C.c_double), ("max_reproj_error", C.c_double),
                ("lambda_init", C.c_double), ("rel_tol", C.c_double)]


class SBAStats(C.Structure):
    _fields_ = [("iterations", C.c_int32), ("accepted", C.c_int32), ("n_window_kf", C.c_int32),
                ("n_landmarks", C.c_int32), ("cost", C.c_double * 16), ("obs", C.c_int32 * 16),
                ("step", C.c_int32 * 16), ("lambda_", C.c_double), ("initial_cost", C.c_double),
                ("final_cost", C.c_double), ("status", C.c_int32)]


def sba_options(window=5, iters=10, min_point=2, fixed=2, huber=5.0, max_err=5.0, lam=1e-4,
                rel_tol=1e-6):
    return SBAOptions(window, iters, min_point, fixed, huber, max_err, lam, rel_tol)


def _ref(m, ref_kf_id):
    ref = m.get("ref_kf_id") if ref_kf_id is None else ref_kf_id
    return C.c_uint64(0 if ref is None else int(ref)), (0 if ref is None else 1)


def sba_optimize(m, opts=None, ref_kf_id=None):
    """Runs the oracle Schur-complement BA on a synth.BAMap in place; returns SBAStats."""
    if opts is None:
        opts = sba_options(window=m.get("window", 5))
    v = map_view(m)
    st = SBAStats()
    ref, has_ref = _ref(m, ref_kf_id)
    assert lib().orc_sba_optimize_map(C.byref(v), ref, has_ref, C.byref(opts), C.byref(st)) == 0
    return st


def sba_system(m, opts=None, lam=None, ref_kf_id=None):
    """Reduced pose system (S, rhs) at the map's current state (None on an early return)."""
    if opts is None:
        opts = sba_options(window=m.get("window", 5))
    lam = opts.lambda_init if lam is None else lam
    v = map_view(m)
    ref, has_ref = _ref(m, ref_kf_id)
    nk = min(int(opts.window_size), m.n_kf)
    n = 6 * nk
    S = np.zeros((n, n))
    rhs = np.zeros(n)
    rc = lib().orc_sba_system(C.byref(v), ref, has_ref, C.byref(opts), C.c_double(lam), _p(S), _p(rhs), n)
    if rc == 1:
        return None
    assert rc == 0, rc
    return S, rhs


def sba_system_shard(m, shard_rank, shard_count, opts=None, lam=None, ref_kf_id=None):
    """One landmark shard's partial reduced system before the all-reduce (no pose damping, no gauge):
    (S_part, rhs_part, pose-block diagonals, cost, valid observations), or None on an early return."""
    if opts is None:
        opts = sba_options(window=m.get("window", 5))
    lam = opts.lambda_init if lam is None else lam
    v = map_view(m)
    ref, has_ref = _ref(m, ref_kf_id)
    nk = min(int(opts.window_size), m.n_kf)
    n = 6 * nk
    S, rhs, htd, cc = np.zeros((n, n)), np.zeros(n), np.zeros(n), np.zeros(2)
    rc = lib().orc_sba_system_shard(C.byref(v), ref, has_ref, C.byref(opts), C.c_double(lam), int(shard_rank),
                                    int(shard_count), _p(S), _p(rhs), _p(htd), _p(cc), n)
    if rc == 1:
        return None
    assert rc == 0, rc
    return S, rhs, htd, float(cc[0]), int(cc[1])


# ---------------------------------------------------------------------------- landmark creation
DEPTH_TYPES = {np.dtype(np.uint16): 0, np.dtype(np.float32): 1, np.dtype(np.float64): 2}


def depth_landmarks(uv, has, depth, intr, pose):
    """CreateLandmarksFromDepth restated: (index per feature, created points)."""
    uv = np.ascontiguousarray(uv, np.float64)
    has = np.ascontiguousarray(has, np.uint8)
    n = len(has)
    idx = np.full(max(n, 1), -1, np.int32)
    pw = np.zeros((max(n, 1), 3))
    cnt = C.c_int(0)
    if depth is None:
        dptr, dt, rows, cols, stride = None, 0, 0, 0, 0
    else:
        depth = np.ascontiguousarray(depth)
        dptr, dt, rows, cols, stride = _p(depth), DEPTH_TYPES[depth.dtype], depth.shape[0], depth.shape[1], depth.strides[0]
    intr = np.ascontiguousarray(intr, np.float64)
    pose = np.ascontiguousarray(pose, np.float64)
    assert lib().orc_depth_landmarks(_p(uv), _p(has), n, dptr, dt, rows, cols, C.c_int64(stride), _p(intr),
                                     _p(pose), _p(idx), _p(pw), C.byref(cnt)) == 0
    return idx[:n].copy(), pw[:cnt.value].copy()


def triangulate(d, min_angle_deg=1.0, max_err=5.0, intr1=None, intr2=None):
    """TriangulateWithLastKeyFrame restated on a synth.make_keyframe_pair dict."""
    m = np.ascontiguousarray(d["matches"])
    nm = len(m)
    idx = np.full(max(nm, 1), -1, np.int32)
    pw = np.zeros((max(nm, 1), 3))
    cnt = C.c_int(0)
    i1 = np.ascontiguousarray(d["intr"] if intr1 is None else intr1, np.float64)
    i2 = np.ascontiguousarray(d["intr"] if intr2 is None else intr2, np.float64)
    rc = lib().orc_triangulate(_p(d["uv1"]), _p(d["has1"]), len(d["has1"]), _p(i1), _p(d["pose1"]),
                               _p(d["uv2"]), _p(d["has2"]), len(d["has2"]), _p(i2), _p(d["pose2"]), _p(m), nm,
                               C.c_double(min_angle_deg), C.c_double(max_err), _p(idx), _p(pw), C.byref(cnt))
    assert rc == 0, rc
    return idx[:nm].copy(), pw[:cnt.value].copy()


# ---------------------------------------------------------------------------- PnP RANSAC
PNP_OPTIONS_DTYPE = np.dtype([("max_iterations", "<i4"), ("refine_iterations", "<i4"), ("reproj_error", "<f8"),
                              ("confidence", "<f8"), ("seed", "<u8")])
PNP_RESULT_DTYPE = np.dtype([("ok", "<i4"), ("n_inliers", "<i4"), ("best_hypothesis", "<i4"),
                             ("hypotheses_run", "<i4"), ("refine_iterations", "<i4"), ("reserved", "<i4"),
                             ("rvec", "<f8", 3), ("tvec", "<f8", 3), ("pose", "<f8", 7), ("cost0", "<f8"),
                             ("cost", "<f8")])


def pnp_options(n, max_iterations=None, reproj_error=2.0, confidence=0.99, seed=0x5EED, refine_iterations=20):
    """Tracking::TrackWithPnP's solvePnPRansac arguments (tracking.cpp:420-423)."""
    o = np.zeros((), PNP_OPTIONS_DTYPE)
    o["max_iterations"] = min(100, 2 * n) if max_iterations is None else max_iterations
    o["refine_iterations"] = refine_iterations
    o["reproj_error"] = reproj_error
    o["confidence"] = confidence
    o["seed"] = seed
    return o


def pnp_ransac_batch(offsets, obj, img, intr, opts):
    """Restated PnP RANSAC over independent problems: (results[P], mask[N])."""
    offsets = np.ascontiguousarray(offsets, np.int32)
    obj = np.ascontiguousarray(obj, np.float32)
    img = np.ascontiguousarray(img, np.float32)
    intr = np.ascontiguousarray(intr, np.float64)
    opts = np.ascontiguousarray(opts, PNP_OPTIONS_DTYPE)
    P = len(offsets) - 1
    out = np.zeros(P, PNP_RESULT_DTYPE)
    mask = np.zeros(max(int(offsets[-1]), 1), np.uint8)
    assert lib().orc_pnp_ransac_batch(P, _p(offsets), _p(obj), _p(img), _p(intr), _p(opts), _p(mask), _p(out)) == 0
    return out, mask[:offsets[-1]].copy()


def pnp_ransac(obj, img, intr, opt):
    out, mask = pnp_ransac_batch(np.array([0, len(obj)]), obj, img, intr, np.atleast_1d(opt))
    return out[0], mask


def pnp_hypothesis(obj, img, intr, seed, h):
    obj = np.ascontiguousarray(obj, np.float32)
    img = np.ascontiguousarray(img, np.float32)
    R = np.zeros(9)
    t = np.zeros(3)
    ok = lib().orc_pnp_hypothesis(_p(obj), _p(img), len(obj), _p(np.ascontiguousarray(intr, np.float64)),
                                  C.c_uint64(seed), h, _p(R), _p(t))
    return (R.reshape(3, 3), t) if ok else None


def p3p(P, f):
    P = np.ascontiguousarray(P, np.float64)
    f = np.ascontiguousarray(f, np.float64)
    R = np.zeros(72)
    t = np.zeros(24)
    ns = lib().orc_p3p(_p(P), _p(f), _p(R), _p(t))
    return [(R[9 * s:9 * s + 9].reshape(3, 3), t[3 * s:3 * s + 3].copy()) for s in range(ns)]


def poly_roots(c):
    c = np.ascontiguousarray(c, np.float64)
    out = np.zeros(4)
    n = lib().orc_poly_roots(_p(c), len(c) - 1, _p(out))
    return out[:n].copy()


def pnp_update_iters(p, ep, max_iters):
    return lib().orc_pnp_update_iters(C.c_double(p), C.c_double(ep), max_iters)


# ---------------------------------------------------------------------------- essential RANSAC
EM_OPTIONS_DTYPE = np.dtype([("max_iterations", "<i4"), ("reserved", "<i4"), ("threshold", "<f8"),
                             ("confidence", "<f8"), ("distance_thresh", "<f8"), ("seed", "<u8")])
EM_RESULT_DTYPE = np.dtype([("ok", "<i4"), ("n_inliers", "<i4"), ("n_ransac_inliers", "<i4"),
                            ("best_hypothesis", "<i4"), ("best_model", "<i4"), ("hypotheses_run", "<i4"),
                            ("pose_candidate", "<i4"), ("reserved", "<i4"), ("E", "<f8", 9), ("R", "<f8", 9),
                            ("t", "<f8", 3)])


def essential_options(max_iterations=1000, threshold=1.0, confidence=0.999, distance_thresh=50.0, seed=0x5EED):
    """findEssentialMat(.., RANSAC, 0.999, 1.0, mask) + recoverPose (tracking.cpp:521-528)."""
    o = np.zeros((), EM_OPTIONS_DTYPE)
    o["max_iterations"] = max_iterations
    o["threshold"] = threshold
    o["confidence"] = confidence
    o["distance_thresh"] = distance_thresh
    o["seed"] = seed
    return o


def essential_ransac_batch(offsets, pts1, pts2, intr, opts):
    offsets = np.ascontiguousarray(offsets, np.int32)
    pts1 = np.ascontiguousarray(pts1, np.float32)
    pts2 = np.ascontiguousarray(pts2, np.float32)
    intr = np.ascontiguousarray(intr, np.float64)
    opts = np.ascontiguousarray(opts, EM_OPTIONS_DTYPE)
    P = len(offsets) - 1
    out = np.zeros(P, EM_RESULT_DTYPE)
    mask = np.zeros(max(int(offsets[-1]), 1), np.uint8)
    assert lib().orc_essential_ransac_batch(P, _p(offsets), _p(pts1), _p(pts2), _p(intr), _p(opts), _p(mask),
                                            _p(out)) == 0
    return out, mask[:offsets[-1]].copy()


def essential_ransac(pts1, pts2, intr, opt):
    out, mask = essential_ransac_batch(np.array([0, len(pts1)]), pts1, pts2, intr, np.atleast_1d(opt))
    return out[0], mask


def five_point(x1, x2):
    x1 = np.ascontiguousarray(x1, np.float64)
    x2 = np.ascontiguousarray(x2, np.float64)
    Es = np.zeros(90)
    n = lib().orc_five_point(_p(x1), _p(x2), _p(Es))
    return Es[:9 * n].reshape(n, 3, 3)
