"""ctypes binding of libvxslam.so (include/vx_slam.h) for tests, smoke and bench.

There is no Python fallback: if the HIP library is missing or fails to load, every entry point
raises.  Names mirror the reference call surface: ``ORBExtractor.extract`` (FeatureExtractor::
Extract, core/feature/feature_extractor.h:15), ``ORBMatcher.match`` (FeatureMatcher::Match,
core/feature/feature_matcher.h:11-12) and ``LocalBA.optimize`` (LocalBA::Optimize,
core/backend/local_ba.h:23).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REPO_ROOT = os.path.dirname(PKG_ROOT)
LIB_PATH = os.environ.get("VX_LIB") or os.path.join(PKG_ROOT, "lib", "libvxslam.so")  # VX_LIB: trace build
HEADER_PATH = os.path.join(REPO_ROOT, "include", "vx_slam.h")

VX_OK, VX_ERR_INVALID, VX_ERR_HIP, VX_ERR_CAPACITY, VX_ERR_COMM, VX_ERR_STATE = 0, -1, -2, -3, -4, -5
MAX_SLOTS = 4
ORDER_STL, ORDER_RASTER = 0, 1  # vx_orb_set_order (include/vx_slam.h)
DEBUG_FAST_NO_BORDER, DEBUG_STAGES = 1, 2  # vx_orb_set_debug test hooks
CAND_DTYPE = np.dtype([("xy", "<u4"), ("score", "<i4"), ("harris", "<f4"), ("pad", "<i4")])

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("response", "<f4"), ("angle", "<f4"),
                           ("octave", "<i4")])
MATCH_DTYPE = np.dtype([("query_idx", "<i4"), ("train_idx", "<i4"), ("distance", "<f4")])


class VxError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"vx error {code}: {msg}")
        self.code = code


class OrbParams(C.Structure):
    _fields_ = [("n_features", C.c_int32), ("scale_factor", C.c_float), ("n_levels", C.c_int32),
                ("fast_threshold", C.c_int32), ("edge_threshold", C.c_int32)]


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


EXPORTS = [
    "vx_version", "vx_create", "vx_destroy", "vx_host_alloc", "vx_host_free", "vx_last_error", "vx_stream", "vx_synchronize",
    "vx_stream_wait_ctx", "vx_event_create", "vx_event_record", "vx_event_wait", "vx_event_destroy",
    "vx_orb_default_params", "vx_orb_pattern", "vx_orb_extract", "vx_orb_extract_async",
    "vx_orb_fetch", "vx_orb_slot_device", "vx_match_knn2_ratio", "vx_match_slots_async",
    "vx_match_device_async", "vx_match_fetch", "vx_ba_default_options", "vx_ba_optimize_map", "vx_ba_plan_create",
    "vx_ba_plan_run_async", "vx_ba_plan_fetch", "vx_ba_plan_destroy", "vx_ba_plan_info", "vx_ba_plan_layout", "vx_ba_plan_persistent", "vx_ba_plan_fused_tables",
    "vx_ba_plan_inspect", "vx_ba_shard_of", "vx_comm_unique_id", "vx_comm_init", "vx_comm_info", "vx_prof_enable", "vx_prof_count", "vx_prof_name",
    "vx_prof_read", "vx_sba_default_options", "vx_sba_plan_create", "vx_sba_plan_run_async",
    "vx_sba_plan_fetch", "vx_sba_plan_destroy", "vx_sba_plan_info", "vx_sba_plan_system",
    "vx_sba_optimize_map", "vx_depth_landmarks", "vx_triangulate", "vx_graph_enable", "vx_graph_counts", "vx_create_ex", "vx_device_cus", "vx_ba_plan_create_ex",
    "vx_dmap_create", "vx_dmap_add_keyframe", "vx_dmap_add_landmarks", "vx_dmap_add_observations",
    "vx_dmap_remove_observations", "vx_dmap_remove_keyframe", "vx_dmap_remove_landmarks", "vx_dmap_set_features",
    "vx_dmap_set_landmark_bad", "vx_dmap_set_poses", "vx_dmap_counts", "vx_dmap_live_counts", "vx_dmap_download",
    "vx_ba_plan_create_dmap", "vx_ba_plan_apply_dmap", "vx_ba_shard_emulate_run", "vx_ba_optimize_dmap",
    "vx_ba_dmap_results", "vx_ba_dmap_results_view", "vx_dmap_prefetch_results", "vx_sba_plan_factor_work", "vx_sba_plan_create_dmap", "vx_sba_plan_rebuild_dmap", "vx_sba_shard_emulate_run", "vx_sba_plan_apply_dmap", "vx_seq_create", "vx_seq_destroy", "vx_seq_wait", "vx_seq_record", "vx_seq_extract",
    "vx_seq_match", "vx_seq_ba_run", "vx_seq_length", "vx_seq_run", "vx_seq_set_threads",
    "vx_orb_extract_batch_async", "vx_orb_batch_fetch", "vx_orb_batch_device", "vx_match_batch_async",
    "vx_match_batch_fetch", "vx_orb_extract_batch", "vx_match_knn2_ratio_batch", "vx_orb_set_order",
    "vx_orb_get_order", "vx_orb_set_debug", "vx_orb_debug_read", "vx_test_retain_best",
]

DEPTH_TYPES = {np.dtype(np.uint16): 0, np.dtype(np.float32): 1, np.dtype(np.float64): 2}

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", PKG_ROOT, "-j8"], check=True)


def lib():
    """Load libvxslam.so (fails loudly: there is no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} missing: run __graft_entry__.build() (no CPU fallback exists)")
        L = C.CDLL(LIB_PATH)
        L.vx_last_error.restype = C.c_char_p
        L.vx_last_error.argtypes = [C.c_void_p]
        L.vx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
        L.vx_destroy.argtypes = [C.c_void_p]
        L.vx_host_alloc.restype = C.c_void_p
        L.vx_host_alloc.argtypes = [C.c_size_t]
        L.vx_host_free.argtypes = [C.c_void_p]
        L.vx_stream.restype = C.c_void_p
        L.vx_stream.argtypes = [C.c_void_p]
        L.vx_synchronize.argtypes = [C.c_void_p]
        L.vx_set_grid_share.argtypes = [C.c_void_p, C.c_float]
        L.vx_orb_set_order.argtypes = [C.c_void_p, C.c_int]
        L.vx_orb_get_order.argtypes = [C.c_void_p]
        L.vx_orb_set_debug.argtypes = [C.c_void_p, C.c_int]
        L.vx_orb_debug_read.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]
        L.vx_test_retain_best.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                          C.POINTER(C.c_int)]
        L.vx_stream_wait_ctx.argtypes = [C.c_void_p, C.c_void_p]
        L.vx_event_create.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
        L.vx_event_record.argtypes = [C.c_void_p, C.c_void_p]
        L.vx_event_wait.argtypes = [C.c_void_p, C.c_void_p]
        L.vx_event_destroy.argtypes = [C.c_void_p]
        L.vx_event_destroy.restype = None
        L.vx_orb_slot_device.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                         C.POINTER(C.c_int32)]
        L.vx_match_device_async.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                            C.c_int, C.c_float]
        L.vx_orb_extract_batch_async.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int64, C.c_int,
                                                 C.c_int, C.c_int, C.c_int64, C.c_int]
        L.vx_orb_extract_batch.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p), C.c_int, C.c_int, C.c_int,
                                           C.c_int, C.c_int64, C.c_int]
        L.vx_orb_batch_device.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_void_p),
                                          C.POINTER(C.c_void_p), C.POINTER(C.c_int32)]
        L.vx_orb_batch_fetch.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_int,
                                         C.POINTER(C.c_int)]
        L.vx_match_batch_async.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                           C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.c_int,
                                           C.c_float]
        L.vx_match_batch_fetch.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_int)]
        L.vx_prof_name.restype = C.c_char_p
        L.vx_ba_plan_destroy.argtypes = [C.c_void_p]
        L.vx_dmap_destroy.argtypes = [C.c_void_p]
        L.vx_dmap_destroy.restype = None
        L.vx_ba_plan_destroy.restype = None
        L.vx_orb_default_params.restype = None
        L.vx_ba_default_options.restype = None
        L.vx_sba_plan_destroy.argtypes = [C.c_void_p]
        L.vx_sba_plan_destroy.restype = None
        L.vx_sba_default_options.restype = None
        L.vx_pnp_default_options.restype = None
        L.vx_essential_default_options.restype = None
        L.vx_seq_destroy.argtypes = [C.c_void_p]
        L.vx_seq_destroy.restype = None
        for f in ("vx_seq_wait", "vx_seq_record"):
            getattr(L, f).argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.vx_seq_extract.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                     C.c_int64, C.c_int]
        L.vx_seq_match.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                   C.c_int, C.c_float]
        L.vx_seq_ba_run.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.vx_seq_length.argtypes = [C.c_void_p]
        L.vx_seq_run.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
        L.vx_seq_set_threads.argtypes = [C.c_void_p, C.c_int]
        L.vx_ba_shard_of.restype = C.c_uint32
        L.vx_ba_shard_of.argtypes = [C.c_uint64, C.c_int]
        _lib = L
    return _lib


def _p(a):
    return C.c_void_p(a.ctypes.data)


# vx_pnp_options / vx_pnp_result (include/vx_slam.h) as numpy records
PNP_OPTIONS_DTYPE = np.dtype([("max_iterations", "<i4"), ("refine_iterations", "<i4"), ("reproj_error", "<f8"),
                              ("confidence", "<f8"), ("seed", "<u8")])
PNP_RESULT_DTYPE = np.dtype([("ok", "<i4"), ("n_inliers", "<i4"), ("best_hypothesis", "<i4"),
                             ("hypotheses_run", "<i4"), ("refine_iterations", "<i4"), ("reserved", "<i4"),
                             ("rvec", "<f8", 3), ("tvec", "<f8", 3), ("pose", "<f8", 7), ("cost0", "<f8"),
                             ("cost", "<f8")])


EM_OPTIONS_DTYPE = np.dtype([("max_iterations", "<i4"), ("reserved", "<i4"), ("threshold", "<f8"),
                             ("confidence", "<f8"), ("distance_thresh", "<f8"), ("seed", "<u8")])
EM_RESULT_DTYPE = np.dtype([("ok", "<i4"), ("n_inliers", "<i4"), ("n_ransac_inliers", "<i4"),
                            ("best_hypothesis", "<i4"), ("best_model", "<i4"), ("hypotheses_run", "<i4"),
                            ("pose_candidate", "<i4"), ("reserved", "<i4"), ("E", "<f8", 9), ("R", "<f8", 9),
                            ("t", "<f8", 3)])


def essential_options(max_iterations=None, threshold=None, confidence=None, distance_thresh=None, seed=None):
    """findEssentialMat(.., RANSAC, 0.999, 1.0, mask) + recoverPose (tracking.cpp:521-528) defaults,
    any field overridable."""
    o = np.zeros((), EM_OPTIONS_DTYPE)
    lib().vx_essential_default_options(_p(o))
    for k, v in (("max_iterations", max_iterations), ("threshold", threshold), ("confidence", confidence),
                 ("distance_thresh", distance_thresh), ("seed", seed)):
        if v is not None:
            o[k] = v
    return o


def pnp_options(n, max_iterations=None, reproj_error=2.0, confidence=0.99, seed=0x5EED, refine_iterations=20):
    """solvePnPRansac's arguments in Tracking::TrackWithPnP (tracking.cpp:420-423) for n pairs."""
    o = np.zeros((), PNP_OPTIONS_DTYPE)
    lib().vx_pnp_default_options(int(n), _p(o))
    if max_iterations is not None:
        o["max_iterations"] = max_iterations
    o["refine_iterations"] = refine_iterations
    o["reproj_error"] = reproj_error
    o["confidence"] = confidence
    o["seed"] = seed
    return o


def default_orb_params(n_features=1000, scale_factor=1.2, n_levels=8, fast_threshold=20,
                       edge_threshold=31):
    return OrbParams(n_features, scale_factor, n_levels, fast_threshold, edge_threshold)


def default_ba_options(window=5, iters=5, min_pose=20, min_point=2, huber=5.0, max_err=5.0):
    return BAOptions(window, iters, min_pose, min_point, huber, max_err)


def default_sba_options(window=5, iters=10, min_point=2, fixed=2, huber=5.0, max_err=5.0, lam=1e-4,
                        rel_tol=1e-6):
    return SBAOptions(window, iters, min_point, fixed, huber, max_err, lam, rel_tol)


def map_view(m) -> MapView:
    """MapView over the arrays of a synth.BAMap (kf_pose / lm_pos are written in place)."""
    v = MapView()
    for name, _ in MapView._fields_:
        if name == "n_kf":
            v.n_kf = int(m["kf_id"].shape[0])
        elif name == "n_lm":
            v.n_lm = int(m["lm_id"].shape[0])
        else:
            a = m[name]
            assert a.flags["C_CONTIGUOUS"], name
            setattr(v, name, a.ctypes.data)
    return v


def pattern() -> np.ndarray:
    out = np.zeros(1024, np.int32)
    rc = lib().vx_orb_pattern(_p(out))
    assert rc == 0
    return out


def ba_plan_inspect(m, opts=None, ref_kf_id=None, shard_rank=0, shard_count=1) -> dict:
    """Host-only dry run of vx_ba_plan_create (no device needed)."""
    opts = opts or default_ba_options(window=m.get("window", 5))
    ref = m.get("ref_kf_id") if ref_kf_id is None else ref_kf_id
    v = map_view(m)
    out = np.zeros(8, np.int64)
    lm = np.zeros(max(int(m["lm_id"].shape[0]), 1), np.int32)
    kf = np.zeros(max(int(m["kf_id"].shape[0]), 1), np.int32)
    rc = lib().vx_ba_plan_inspect(C.byref(v), C.c_uint64(0 if ref is None else int(ref)), 0 if ref is None else 1,
                                  C.byref(opts), shard_rank, shard_count, _p(out), _p(lm), len(lm), _p(kf), len(kf))
    if rc != VX_OK:
        raise VxError(rc, "vx_ba_plan_inspect failed")
    keys = ["status", "n_window_kf", "n_landmarks", "n_kf", "n_opt", "n_lm", "n_pose_obs", "n_lm_obs"]
    d = {k: int(x) for k, x in zip(keys, out)}
    d["lm_map_idx"] = lm[:d["n_lm"]].copy()
    d["kf_map_idx"] = kf[:d["n_kf"]].copy()
    return d


def ba_shard_of(lm_id: int, shard_count: int) -> int:
    return int(lib().vx_ba_shard_of(C.c_uint64(int(lm_id)), int(shard_count)))


class Event:
    """A device event (vx_event) for cross-context ordering."""

    def __init__(self, ctx: "Context"):
        self._h = C.c_void_p()
        ctx._check(lib().vx_event_create(ctx.handle, C.byref(self._h)))

    def close(self):
        if self._h:
            lib().vx_event_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Context:
    """One vx_ctx = one device + one HIP stream (not thread-safe, like the reference's tracking
    thread owning the hot path, core/system/system.cpp:39-52)."""

    def __init__(self, device: int = 0, priority: int = 0, cu_mask=None):
        """cu_mask: iterable of compute-unit indices this context may use (None: all)."""
        self._h = C.c_void_p()
        self.device = int(device)
        words, nw = None, 0
        if cu_mask is not None:
            n = lib().vx_device_cus(int(device))
            nw = (n + 31) // 32
            words = (C.c_uint32 * nw)()
            for i in cu_mask:
                words[i // 32] |= 1 << (i % 32)
        rc = lib().vx_create_ex(int(device), int(priority), words, nw, C.byref(self._h))
        if rc != VX_OK:
            raise VxError(rc, f"vx_create(device={device}) failed")

    def close(self):
        if self._h:
            lib().vx_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != VX_OK:
            raise VxError(rc, lib().vx_last_error(self._h).decode())
        return rc

    @property
    def handle(self):
        return self._h

    @property
    def stream(self) -> int:
        return lib().vx_stream(self._h)

    def synchronize(self):
        self._check(lib().vx_synchronize(self._h))

    def wait_for(self, other: "Context"):
        """Order later work on this context after everything enqueued on `other` (device-side)."""
        self._check(lib().vx_stream_wait_ctx(self._h, other._h))

    # ---------------------------------------------------------------- ORB
    def orb_extract(self, img: np.ndarray, params: OrbParams | None = None, cap: int | None = None):
        img = np.ascontiguousarray(img)
        h, w = img.shape[:2]
        ch = 1 if img.ndim == 2 else img.shape[2]
        params = params or default_orb_params()
        cap = cap or (2 * params.n_features + 256)
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = C.c_int(0)
        self._check(lib().vx_orb_extract(self._h, C.byref(params), _p(img), w, h, ch,
                                         C.c_int64(img.strides[0]), _p(kps), _p(desc), cap,
                                         C.byref(n)))
        return kps[:n.value].copy(), desc[:n.value].copy()

    def orb_extract_async(self, d_img_ptr: int, w: int, h: int, channels: int, row_stride: int,
                          slot: int, params: OrbParams | None = None):
        params = params or default_orb_params()
        self._check(lib().vx_orb_extract_async(self._h, C.byref(params), C.c_void_p(d_img_ptr), w, h,
                                               channels, C.c_int64(row_stride), slot))

    def orb_fetch(self, slot: int, cap: int = 8192):
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = C.c_int(0)
        self._check(lib().vx_orb_fetch(self._h, slot, _p(kps), _p(desc), cap, C.byref(n)))
        return kps[:n.value].copy(), desc[:n.value].copy()

    def orb_extract_batch_async(self, d_imgs_ptr: int, n_frames: int, frame_stride: int, w: int, h: int,
                                channels: int, row_stride: int, bank: int = 0, params: OrbParams | None = None):
        """Extract n_frames device-resident images (frame f at d_imgs_ptr + f * frame_stride) in one
        launch per kernel; results stay in batch bank `bank`."""
        params = params or default_orb_params()
        self._check(lib().vx_orb_extract_batch_async(self._h, C.byref(params), C.c_void_p(d_imgs_ptr), n_frames,
                                                     C.c_int64(frame_stride), w, h, channels, C.c_int64(row_stride),
                                                     bank))

    def orb_batch_fetch(self, bank: int, frame: int, cap: int = 8192):
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = C.c_int(0)
        self._check(lib().vx_orb_batch_fetch(self._h, bank, frame, _p(kps), _p(desc), cap, C.byref(n)))
        return kps[:n.value].copy(), desc[:n.value].copy()

    def batch_device(self, bank: int, frame: int):
        """(device descriptor pointer, device count pointer, row capacity) of a batch frame."""
        d, n, cap = C.c_void_p(), C.c_void_p(), C.c_int32()
        self._check(lib().vx_orb_batch_device(self._h, bank, frame, C.byref(d), C.byref(n), C.byref(cap)))
        return d.value, n.value, cap.value

    def orb_extract_batch(self, imgs: np.ndarray, params: OrbParams | None = None, bank: int = 0):
        """Host convenience over vx_orb_extract_batch (host frames, uploaded by the library): a
        (B, H, W[, C]) stack extracted as one batch; returns a list of (keypoints, descriptors) per
        frame."""
        imgs = np.ascontiguousarray(imgs)
        b, h, w = imgs.shape[:3]
        ch = 1 if imgs.ndim == 3 else imgs.shape[3]
        params = params or default_orb_params()
        ptrs = (C.c_void_p * b)(*[C.c_void_p(imgs[f].ctypes.data) for f in range(b)])
        self._check(lib().vx_orb_extract_batch(self._h, C.byref(params), ptrs, b, w, h, ch, C.c_int64(imgs.strides[1]),
                                               bank))
        return [self.orb_batch_fetch(bank, f) for f in range(b)]

    # ---------------------------------------------------------------- matching
    def match(self, q: np.ndarray, t: np.ndarray, ratio: float = 0.8):
        q = np.ascontiguousarray(q, np.uint8)
        t = np.ascontiguousarray(t, np.uint8)
        cap = max(len(q), 1)
        out = np.zeros(cap, MATCH_DTYPE)
        n = C.c_int(0)
        self._check(lib().vx_match_knn2_ratio(self._h, _p(q), len(q), _p(t), len(t),
                                              C.c_float(ratio), _p(out), cap, C.byref(n)))
        return out[:n.value].copy()

    def match_slots_async(self, q_slot: int, t_slot: int, ratio: float = 0.8):
        self._check(lib().vx_match_slots_async(self._h, q_slot, t_slot, C.c_float(ratio)))

    def slot_device(self, slot: int):
        """(device descriptor pointer, device count pointer, row capacity) of an extraction slot."""
        d, n, cap = C.c_void_p(), C.c_void_p(), C.c_int32()
        self._check(lib().vx_orb_slot_device(self._h, slot, C.byref(d), C.byref(n), C.byref(cap)))
        return d.value, n.value, cap.value

    def match_device_async(self, query, train, ratio: float = 0.8):
        """Match device descriptor sets given as slot_device() triples (possibly of another context)."""
        (dq, nq, cq), (dt, nt, ct) = query, train
        self._check(lib().vx_match_device_async(self._h, C.c_void_p(dq), C.c_void_p(nq), cq, C.c_void_p(dt),
                                                C.c_void_p(nt), ct, C.c_float(ratio)))

    def event(self) -> "Event":
        return Event(self)

    def record(self, ev: "Event"):
        self._check(lib().vx_event_record(self._h, ev._h))

    def wait_event(self, ev: "Event"):
        self._check(lib().vx_event_wait(self._h, ev._h))

    def match_batch_async(self, pairs, ratio: float = 0.8):
        """pairs: list of (query, train) device triples (slot_device() / batch_device())."""
        n = len(pairs)
        arr = lambda xs: (C.c_void_p * max(n, 1))(*[C.c_void_p(x) for x in xs])
        dq, nq, dt, nt = (arr([p[0][0] for p in pairs]), arr([p[0][1] for p in pairs]),
                          arr([p[1][0] for p in pairs]), arr([p[1][1] for p in pairs]))
        cq = max([p[0][2] for p in pairs], default=0)
        ct = max([p[1][2] for p in pairs], default=0)
        self._check(lib().vx_match_batch_async(self._h, n, dq, nq, cq, dt, nt, ct, C.c_float(ratio)))

    def match_batch_fetch(self, pair: int, cap: int = 8192):
        out = np.zeros(cap, MATCH_DTYPE)
        n = C.c_int(0)
        self._check(lib().vx_match_batch_fetch(self._h, pair, _p(out), cap, C.byref(n)))
        return out[:n.value].copy()

    def match_fetch(self, cap: int = 8192):
        out = np.zeros(cap, MATCH_DTYPE)
        n = C.c_int(0)
        self._check(lib().vx_match_fetch(self._h, _p(out), cap, C.byref(n)))
        return out[:n.value].copy()

    # ---------------------------------------------------------------- bundle adjustment
    def ba_optimize(self, m, opts: BAOptions | None = None, ref_kf_id=None) -> BAStats:
        opts = opts or default_ba_options(window=m.get("window", 5))
        ref = m.get("ref_kf_id") if ref_kf_id is None else ref_kf_id
        v = map_view(m)
        st = BAStats()
        self._check(lib().vx_ba_optimize_map(self._h, C.byref(v), C.c_uint64(0 if ref is None else int(ref)),
                                             0 if ref is None else 1, C.byref(opts), C.byref(st)))
        return st

    def ba_plan(self, m, opts: BAOptions | None = None, ref_kf_id=None, shard_rank=0, shard_count=1,
                host_build=False, global_poses=False):
        return BAPlan(self, m, opts, ref_kf_id, shard_rank, shard_count, host_build, global_poses)

    def graph_enable(self, on=True):
        self._check(lib().vx_graph_enable(self._h, 1 if on else 0))

    def set_grid_share(self, share: float):
        """vx_set_grid_share: size one-round grids for this share of the CUs (concurrent contexts)."""
        self._check(lib().vx_set_grid_share(self._h, C.c_float(share)))

    def set_order(self, order: int):
        """vx_orb_set_order: ORDER_STL (default: OpenCV's libstdc++ retainBest permutation) or
        ORDER_RASTER (the same keypoint set per level in raster order)."""
        self._check(lib().vx_orb_set_order(self._h, int(order)))

    @property
    def order(self) -> int:
        return lib().vx_orb_get_order(self._h)

    def set_debug(self, flags: int):
        """vx_orb_set_debug (test hook): DEBUG_FAST_NO_BORDER | DEBUG_STAGES."""
        self._check(lib().vx_orb_set_debug(self._h, int(flags)))

    def debug_read(self, level: int, what: int):
        """vx_orb_debug_read after orb_extract: 0 level bytes, 1 blurred level, 2 candidate records
        (raster order), 3 retainBest(2q) order (indices into 2), 4 final records (CAND_DTYPE)."""
        n = C.c_int64(0)
        rc = lib().vx_orb_debug_read(self._h, level, what, None, 0, C.byref(n))
        if rc not in (VX_OK, VX_ERR_CAPACITY):
            self._check(rc)
        dt = {0: np.uint8, 1: np.uint8, 2: CAND_DTYPE, 3: np.int32, 4: CAND_DTYPE}[what]
        out = np.zeros(max(n.value, 1), dt)
        self._check(lib().vx_orb_debug_read(self._h, level, what, _p(out), out.nbytes, C.byref(n)))
        return out[:n.value]

    def test_retain_best(self, keys, npts: int, wide: bool = False, use_lds: bool = True):
        """vx_test_retain_best: the device retainBest over bare keys; kept indices in output order."""
        keys = np.ascontiguousarray(keys, np.uint32)
        out = np.zeros(max(len(keys), 1), np.int32)
        n = C.c_int(0)
        self._check(lib().vx_test_retain_best(self._h, _p(keys), len(keys), int(npts), int(wide), int(use_lds),
                                              _p(out), C.byref(n)))
        return out[:n.value].copy()

    def graph_counts(self):
        """(graphs captured, graph launches) of this context's hipGraph replay."""
        cap, lau = C.c_int(0), C.c_int(0)
        self._check(lib().vx_graph_counts(self._h, C.byref(cap), C.byref(lau)))
        return cap.value, lau.value

    # ---------------------------------------------------------------- landmark creation
    def depth_landmarks(self, uv, has, depth, intr, pose):
        """Tracking::CreateLandmarksFromDepth on the GPU: (index per feature or -1, created points)."""
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
            dptr, dt = _p(depth), DEPTH_TYPES[depth.dtype]
            rows, cols, stride = depth.shape[0], depth.shape[1], depth.strides[0]
        intr = np.ascontiguousarray(intr, np.float64)
        pose = np.ascontiguousarray(pose, np.float64)
        self._check(lib().vx_depth_landmarks(self._h, _p(uv), _p(has), n, dptr, dt, rows, cols, C.c_int64(stride),
                                             _p(intr), _p(pose), _p(idx), _p(pw), C.byref(cnt)))
        return idx[:n].copy(), pw[:cnt.value].copy()

    def triangulate(self, d, min_angle_deg=1.0, max_err=5.0, intr1=None, intr2=None):
        """Tracking::TriangulateWithLastKeyFrame on the GPU for a synth.make_keyframe_pair dict."""
        m = np.ascontiguousarray(d["matches"])
        nm = len(m)
        idx = np.full(max(nm, 1), -1, np.int32)
        pw = np.zeros((max(nm, 1), 3))
        cnt = C.c_int(0)
        i1 = np.ascontiguousarray(d["intr"] if intr1 is None else intr1, np.float64)
        i2 = np.ascontiguousarray(d["intr"] if intr2 is None else intr2, np.float64)
        self._check(lib().vx_triangulate(self._h, _p(d["uv1"]), _p(d["has1"]), len(d["has1"]), _p(i1),
                                         _p(d["pose1"]), _p(d["uv2"]), _p(d["has2"]), len(d["has2"]), _p(i2),
                                         _p(d["pose2"]), _p(m), nm, C.c_double(min_angle_deg), C.c_double(max_err),
                                         _p(idx), _p(pw), C.byref(cnt)))
        return idx[:nm].copy(), pw[:cnt.value].copy()

    def pnp_ransac_batch(self, offsets, obj, img, intr, opts):
        """cv::solvePnPRansac (Tracking::TrackWithPnP, tracking.cpp:414-423) on the GPU for independent
        problems: problem p owns rows offsets[p]:offsets[p+1] of obj (float32 x3) / img (float32 x2),
        intr[p] = fx fy cx cy, opts[p] a PNP_OPTIONS_DTYPE record.  Returns (results[P], mask[N])."""
        offsets = np.ascontiguousarray(offsets, np.int32)
        obj = np.ascontiguousarray(obj, np.float32).reshape(-1, 3)
        img = np.ascontiguousarray(img, np.float32).reshape(-1, 2)
        intr = np.ascontiguousarray(intr, np.float64).reshape(-1, 4)
        opts = np.ascontiguousarray(np.atleast_1d(opts), PNP_OPTIONS_DTYPE)
        P = len(offsets) - 1
        n = int(offsets[-1])
        assert len(obj) == n and len(img) == n and len(intr) == P and len(opts) == P
        out = np.zeros(max(P, 1), PNP_RESULT_DTYPE)
        mask = np.zeros(max(n, 1), np.uint8)
        self._check(lib().vx_pnp_ransac_batch(self._h, P, _p(offsets), _p(obj), _p(img), _p(intr), _p(opts),
                                              _p(mask), _p(out)))
        return out[:P].copy(), mask[:n].copy()

    def pnp_ransac(self, obj, img, intr, opt):
        """One solvePnPRansac call: (result record, inlier mask)."""
        obj = np.ascontiguousarray(obj, np.float32).reshape(-1, 3)
        img = np.ascontiguousarray(img, np.float32).reshape(-1, 2)
        intr = np.ascontiguousarray(intr, np.float64)
        opt = np.ascontiguousarray(opt, PNP_OPTIONS_DTYPE)
        out = np.zeros(1, PNP_RESULT_DTYPE)
        mask = np.zeros(max(len(obj), 1), np.uint8)
        self._check(lib().vx_pnp_ransac(self._h, _p(obj), _p(img), len(obj), _p(intr), _p(opt), _p(mask), _p(out)))
        return out[0], mask[:len(obj)].copy()

    def essential_ransac_batch(self, offsets, pts_last, pts_curr, intr, opts):
        """cv::findEssentialMat + cv::recoverPose (Tracking::EstimatePoseByEssential,
        tracking.cpp:503-547) on the GPU for independent problems: (results[P], mask[N])."""
        offsets = np.ascontiguousarray(offsets, np.int32)
        p1 = np.ascontiguousarray(pts_last, np.float32).reshape(-1, 2)
        p2 = np.ascontiguousarray(pts_curr, np.float32).reshape(-1, 2)
        intr = np.ascontiguousarray(intr, np.float64).reshape(-1, 4)
        opts = np.ascontiguousarray(np.atleast_1d(opts), EM_OPTIONS_DTYPE)
        P = len(offsets) - 1
        n = int(offsets[-1])
        assert len(p1) == n and len(p2) == n and len(intr) == P and len(opts) == P
        out = np.zeros(max(P, 1), EM_RESULT_DTYPE)
        mask = np.zeros(max(n, 1), np.uint8)
        self._check(lib().vx_essential_ransac_batch(self._h, P, _p(offsets), _p(p1), _p(p2), _p(intr), _p(opts),
                                                    _p(mask), _p(out)))
        return out[:P].copy(), mask[:n].copy()

    def essential_ransac(self, pts_last, pts_curr, intr, opt):
        """One findEssentialMat + recoverPose: (result record, recoverPose mask)."""
        p1 = np.ascontiguousarray(pts_last, np.float32).reshape(-1, 2)
        p2 = np.ascontiguousarray(pts_curr, np.float32).reshape(-1, 2)
        intr = np.ascontiguousarray(intr, np.float64)
        opt = np.ascontiguousarray(opt, EM_OPTIONS_DTYPE)
        out = np.zeros(1, EM_RESULT_DTYPE)
        mask = np.zeros(max(len(p1), 1), np.uint8)
        self._check(lib().vx_essential_ransac(self._h, _p(p1), _p(p2), len(p1), _p(intr), _p(opt), _p(mask),
                                              _p(out)))
        return out[0], mask[:len(p1)].copy()

    def sba_optimize(self, m, opts: SBAOptions | None = None, ref_kf_id=None) -> SBAStats:
        """Schur-complement joint BA (vx_sba_optimize_map) on a synth.BAMap, in place."""
        opts = opts or default_sba_options(window=m.get("window", 5))
        ref = m.get("ref_kf_id") if ref_kf_id is None else ref_kf_id
        v = map_view(m)
        st = SBAStats()
        self._check(lib().vx_sba_optimize_map(self._h, C.byref(v), C.c_uint64(0 if ref is None else int(ref)),
                                              0 if ref is None else 1, C.byref(opts), C.byref(st)))
        return st

    def sba_plan(self, m, opts: SBAOptions | None = None, ref_kf_id=None, shard_rank=0, shard_count=1):
        return SBAPlan(self, m, opts, ref_kf_id, shard_rank, shard_count)

    # ---------------------------------------------------------------- multi-GPU
    def sba_shard_emulate(self, plans):
        """vx_sba_shard_emulate_run: the Schur shard plans run on this one device as the ranks of a
        sharded Schur BA would, the all-reduce of the reduced system replaced by a rank-order sum."""
        arr = (C.c_void_p * len(plans))(*[pl._h.value for pl in plans])
        self._check(lib().vx_sba_shard_emulate_run(self._h, arr, len(plans)))

    def ba_shard_emulate(self, plans):
        """vx_ba_shard_emulate_run: the shard plans (rank r of len(plans)) run on this one device
        as the ranks of a sharded LocalBA would, the all-reduce replaced by a rank-order sum."""
        arr = (C.c_void_p * len(plans))(*[pl._h.value for pl in plans])
        self._check(lib().vx_ba_shard_emulate_run(self._h, arr, len(plans)))

    @staticmethod
    def comm_unique_id() -> bytes:
        buf = (C.c_uint8 * 128)()
        rc = lib().vx_comm_unique_id(buf)
        if rc != VX_OK:
            raise VxError(rc, "ncclGetUniqueId failed")
        return bytes(buf)

    def comm_init(self, uid: bytes, nranks: int, rank: int):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        self._check(lib().vx_comm_init(self._h, buf, nranks, rank))

    def comm_info(self):
        """(nranks, rank) as RCCL reports them for this context's communicator (vx_comm_info)."""
        n, r = C.c_int(0), C.c_int(0)
        self._check(lib().vx_comm_info(self._h, C.byref(n), C.byref(r)))
        return n.value, r.value

    # ---------------------------------------------------------------- profiling
    def prof_enable(self, on=True, stages=None):
        """on=False disables; stages=None brackets every stage, else an iterable of stage names."""
        if not on:
            mask = 0
        elif stages is None:
            mask = -1
        else:
            names = [lib().vx_prof_name(i).decode() for i in range(lib().vx_prof_count())]
            mask = 0
            for s in stages:
                mask |= 1 << names.index(s)
        self._check(lib().vx_prof_enable(self._h, mask))

    def prof_read(self, reset=True) -> dict:
        n = lib().vx_prof_count()
        ms = (C.c_double * n)()
        cnt = (C.c_int64 * n)()
        self._check(lib().vx_prof_read(self._h, ms, cnt, 1 if reset else 0))
        return {lib().vx_prof_name(i).decode(): (ms[i], cnt[i]) for i in range(n)}


class BAPlan:
    """vx_ba_plan: host window selection + device CSR upload, repeatable device runs."""

    def __init__(self, ctx: Context, m, opts=None, ref_kf_id=None, shard_rank=0, shard_count=1, host_build=False,
                 global_poses=False):
        """host_build: the host reference build of the plan (VX_PLAN_HOST_BUILD) instead of the
        device build; global_poses: the large-window kernels at any window size
        (VX_PLAN_GLOBAL_POSES)."""
        self.ctx = ctx
        self.m = m
        self.opts = opts or default_ba_options(window=m.get("window", 5))
        ref = m.get("ref_kf_id") if ref_kf_id is None else ref_kf_id
        self._h = C.c_void_p()
        v = map_view(m)
        ctx._check(lib().vx_ba_plan_create_ex(ctx.handle, C.byref(v), C.c_uint64(0 if ref is None else int(ref)),
                                              0 if ref is None else 1, C.byref(self.opts), shard_rank,
                                              shard_count, (1 if host_build else 0) | (2 if global_poses else 0),
                                              C.byref(self._h)))

    def info(self):
        out = np.zeros(8, np.int64)
        rc = lib().vx_ba_plan_info(self._h, _p(out))
        assert rc == 0
        keys = ["n_kf", "n_lm", "n_pose_obs", "n_lm_obs", "n_opt", "n_split", "n_lm_blocks", "max_lm_obs"]
        return {k: int(v) for k, v in zip(keys, out)}

    def layout(self):
        """vx_ba_plan_layout: whether the plan has the fused k_ba_iter layout, and its shape."""
        out = np.zeros(4, np.int64)
        self.ctx._check(lib().vx_ba_plan_layout(self._h, _p(out)))
        return {k: int(v) for k, v in zip(["fused", "threads", "workgroups", "max_slots"], out)}

    def persistent(self) -> bool:
        """vx_ba_plan_persistent: runs are one persistent k_ba_win launch per window."""
        return bool(lib().vx_ba_plan_persistent(self._h))

    def fused_tables(self) -> bytes:
        """vx_ba_plan_fused_tables: the fused layout's index tables, back to back (test hook)."""
        n = C.c_size_t(0)
        self.ctx._check(lib().vx_ba_plan_fused_tables(self.ctx.handle, self._h, None, C.c_size_t(0), C.byref(n)))
        buf = np.zeros(n.value, np.uint8)
        self.ctx._check(lib().vx_ba_plan_fused_tables(self.ctx.handle, self._h, _p(buf), n, C.byref(n)))
        return buf.tobytes()

    def run_async(self):
        self.ctx._check(lib().vx_ba_plan_run_async(self.ctx.handle, self._h))

    def fetch(self, m=None) -> BAStats:
        st = BAStats()
        v = map_view(m) if m is not None else None
        self.ctx._check(lib().vx_ba_plan_fetch(self.ctx.handle, self._h, C.byref(v) if v is not None else None,
                                               C.byref(st)))
        return st

    def apply(self, dmap: "DMap"):
        """vx_ba_plan_apply_dmap: scatter the run's poses / positions into the resident map."""
        self.ctx._check(lib().vx_ba_plan_apply_dmap(self.ctx.handle, self._h, dmap.handle))

    def close(self):
        if self._h:
            lib().vx_ba_plan_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Seq:
    """vx_seq: a recorded list of async calls replayed from C by run() (include/vx_slam.h)."""

    def __init__(self):
        self._h = C.c_void_p()
        if lib().vx_seq_create(C.byref(self._h)) != VX_OK:
            raise VxError(VX_ERR_INVALID, "vx_seq_create failed")
        self._ctxs = {}
        # every object whose raw handle or device memory a recorded call names (events, plans, the
        # tensors behind image pointers when given): the header requires them to outlive the
        # sequence, so the sequence holds them until close()
        self._keep = []

    def _add(self, rc, ctx, *keep):
        if rc != VX_OK:
            raise VxError(rc, "vx_seq: bad arguments")
        self._ctxs[len(self)] = ctx
        self._keep.extend(k for k in keep if k is not None)

    def wait(self, ctx, ev):
        self._add(lib().vx_seq_wait(self._h, ctx.handle, ev._h), ctx, ev)

    def record(self, ctx, ev):
        self._add(lib().vx_seq_record(self._h, ctx.handle, ev._h), ctx, ev)

    def extract(self, ctx, params, d_img, w, h, ch, stride, slot, owner=None):
        """d_img: a device pointer (int); owner: the object holding that memory (e.g. the torch
        tensor), kept alive with the sequence."""
        self._add(lib().vx_seq_extract(self._h, ctx.handle, C.byref(params), C.c_void_p(d_img), w, h, ch, stride, slot),
                  ctx, owner, params)

    def match(self, ctx, q, t, ratio=0.8):
        """q / t: (desc, count, cap) device triples (Context.slot_device)."""
        self._add(lib().vx_seq_match(self._h, ctx.handle, C.c_void_p(q[0]), C.c_void_p(q[1]), q[2], C.c_void_p(t[0]),
                                     C.c_void_p(t[1]), t[2], C.c_float(ratio)), ctx)

    def ba_run(self, ctx, plan):
        self._add(lib().vx_seq_ba_run(self._h, ctx.handle, plan._h), ctx, plan)

    def __len__(self):
        return lib().vx_seq_length(self._h)

    def set_threads(self, n: int):
        """vx_seq_set_threads: > 1 replays each context's calls on a host thread of its own."""
        if lib().vx_seq_set_threads(self._h, int(n)) != VX_OK:
            raise VxError(VX_ERR_INVALID, "vx_seq_set_threads")

    def run(self):
        bad = C.c_int(-1)
        rc = lib().vx_seq_run(self._h, C.byref(bad))
        if rc != VX_OK:
            ctx = self._ctxs.get(bad.value + 1)
            raise VxError(rc, f"vx_seq_run: call {bad.value}: " + (lib().vx_last_error(ctx.handle).decode() if ctx else ""))

    def close(self):
        if self._h:
            lib().vx_seq_destroy(self._h)
            self._h = C.c_void_p()
        self._keep = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DMap:
    """vx_dmap: visionx::Map resident on the device, updated incrementally (include/vx_slam.h)."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        self._h = C.c_void_p()
        ctx._check(lib().vx_dmap_create(ctx.handle, C.byref(self._h)))

    @property
    def handle(self):
        return self._h

    def add_keyframe(self, kf_id, pose7, intr4, has_cam, feat_uv, feat_lm_id, feat_flags):
        uv = np.ascontiguousarray(feat_uv, np.float64).reshape(-1, 2)
        lm = np.ascontiguousarray(feat_lm_id, np.uint64)
        fl = np.ascontiguousarray(feat_flags, np.uint8)
        pose = np.ascontiguousarray(pose7, np.float64)
        intr = np.ascontiguousarray(intr4, np.float64)
        self.ctx._check(lib().vx_dmap_add_keyframe(self._h, C.c_uint64(int(kf_id)), _p(pose), _p(intr),
                                                   1 if has_cam else 0, len(fl), _p(uv), _p(lm), _p(fl)))

    def add_landmarks(self, ids, pos, bad=None):
        ids = np.ascontiguousarray(ids, np.uint64)
        pos = np.ascontiguousarray(pos, np.float64).reshape(-1, 3)
        b = None if bad is None else np.ascontiguousarray(bad, np.uint8)
        self.ctx._check(lib().vx_dmap_add_landmarks(self._h, len(ids), _p(ids), _p(pos),
                                                    None if b is None else _p(b)))

    def add_observations(self, lm_ids, kf_ids, feat_idx):
        a = np.ascontiguousarray(lm_ids, np.uint64)
        k = np.ascontiguousarray(kf_ids, np.uint64)
        f = np.ascontiguousarray(feat_idx, np.uint64)
        self.ctx._check(lib().vx_dmap_add_observations(self._h, len(a), _p(a), _p(k), _p(f)))

    def remove_observations(self, lm_ids, kf_ids):
        """Landmark::RemoveObservation(kf_id) for each (landmark, keyframe) pair."""
        a = np.ascontiguousarray(lm_ids, np.uint64)
        k = np.ascontiguousarray(kf_ids, np.uint64)
        self.ctx._check(lib().vx_dmap_remove_observations(self._h, len(a), _p(a), _p(k)))

    def remove_keyframe(self, kf_id):
        """Map::RemoveKeyFrame(id)."""
        self.ctx._check(lib().vx_dmap_remove_keyframe(self._h, C.c_uint64(int(kf_id))))

    def remove_landmarks(self, lm_ids):
        """Map::RemoveLandmark(id) for each id."""
        a = np.ascontiguousarray(lm_ids, np.uint64)
        self.ctx._check(lib().vx_dmap_remove_landmarks(self._h, len(a), _p(a)))

    def live_counts(self):
        out = np.zeros(4, np.int64)
        self.ctx._check(lib().vx_dmap_live_counts(self._h, _p(out)))
        return dict(zip(["kf", "lm", "obs"], map(int, out[:3])))

    def set_features(self, kf_id, feat_idx, lm_ids, flags):
        i = np.ascontiguousarray(feat_idx, np.int32)
        lm = np.ascontiguousarray(lm_ids, np.uint64)
        fl = np.ascontiguousarray(flags, np.uint8)
        self.ctx._check(lib().vx_dmap_set_features(self._h, C.c_uint64(int(kf_id)), len(i), _p(i), _p(lm), _p(fl)))

    def set_landmark_bad(self, ids, bad):
        ids = np.ascontiguousarray(ids, np.uint64)
        b = np.ascontiguousarray(bad, np.uint8)
        self.ctx._check(lib().vx_dmap_set_landmark_bad(self._h, len(ids), _p(ids), _p(b)))

    def set_poses(self, kf_ids, poses):
        ids = np.ascontiguousarray(kf_ids, np.uint64)
        ps = np.ascontiguousarray(poses, np.float64).reshape(-1, 7)
        self.ctx._check(lib().vx_dmap_set_poses(self._h, len(ids), _p(ids), _p(ps)))

    def counts(self):
        out = np.zeros(4, np.int64)
        self.ctx._check(lib().vx_dmap_counts(self._h, _p(out)))
        return dict(zip(["kf", "feat", "lm", "obs"], map(int, out)))

    def download(self):
        c = self.counts()
        pose = np.zeros((max(c["kf"], 1), 7))
        pos = np.zeros((max(c["lm"], 1), 3))
        self.ctx._check(lib().vx_dmap_download(self._h, _p(pose), _p(pos)))
        return pose[:c["kf"]], pos[:c["lm"]]

    def plan(self, opts, ref_kf_id=None, shard_rank=0, shard_count=1) -> "BAPlan":
        """vx_ba_plan_create_dmap: the LocalBA plan from the resident map."""
        plan = BAPlan.__new__(BAPlan)
        plan.ctx, plan.m, plan.opts = self.ctx, None, opts
        plan._h = C.c_void_p()
        self.ctx._check(lib().vx_ba_plan_create_dmap(self.ctx.handle, self._h,
                                                     C.c_uint64(0 if ref_kf_id is None else int(ref_kf_id)),
                                                     0 if ref_kf_id is None else 1, C.byref(opts), shard_rank,
                                                     shard_count, C.byref(plan._h)))
        return plan

    def optimize(self, opts, ref_kf_id=None) -> BAStats:
        """vx_ba_optimize_dmap: LocalBA::Optimize on the resident map in one call (plan, run and the
        scatter into the map; synchronises once, at its end)."""
        st = BAStats()
        self.ctx._check(lib().vx_ba_optimize_dmap(self.ctx.handle, self._h,
                                                  C.c_uint64(0 if ref_kf_id is None else int(ref_kf_id)),
                                                  0 if ref_kf_id is None else 1, C.byref(opts), C.byref(st)))
        return st

    def sba_plan(self, opts, ref_kf_id=None) -> "SBAPlan":
        """vx_sba_plan_create_dmap: the Schur-complement BA plan from the resident map."""
        plan = SBAPlan.__new__(SBAPlan)
        plan.ctx, plan.opts = self.ctx, opts
        plan._h = C.c_void_p()
        self.ctx._check(lib().vx_sba_plan_create_dmap(self.ctx.handle, self._h,
                                                      C.c_uint64(0 if ref_kf_id is None else int(ref_kf_id)),
                                                      0 if ref_kf_id is None else 1, C.byref(opts), C.byref(plan._h)))
        return plan

    def sba_plan_rebuild(self, plan: "SBAPlan", ref_kf_id=None) -> "SBAPlan":
        """vx_sba_plan_rebuild_dmap: rebuild a plan of this map in place (its buffers reused)."""
        self.ctx._check(lib().vx_sba_plan_rebuild_dmap(self.ctx.handle, self._h,
                                                       C.c_uint64(0 if ref_kf_id is None else int(ref_kf_id)),
                                                       0 if ref_kf_id is None else 1, plan._h))
        return plan

    def prefetch_results(self, on=True):
        """vx_dmap_prefetch_results: optimize() brings its results back with its one synchronisation."""
        self.ctx._check(lib().vx_dmap_prefetch_results(self._h, 1 if on else 0))

    def results(self):
        """vx_ba_dmap_results: (keyframe rows, their poses (n, 7), landmark rows, positions (n, 3)) the
        last optimize() changed."""
        nk, nl = C.c_int(0), C.c_int(0)
        rc = lib().vx_ba_dmap_results(self.ctx.handle, self._h, 0, None, None, 0, None, None, C.byref(nk),
                                      C.byref(nl))
        if rc not in (VX_OK, VX_ERR_CAPACITY):
            self.ctx._check(rc)
        kr, kp = np.zeros(max(nk.value, 1), np.int64), np.zeros((max(nk.value, 1), 7))
        lr, lp = np.zeros(max(nl.value, 1), np.int64), np.zeros((max(nl.value, 1), 3))
        self.ctx._check(lib().vx_ba_dmap_results(self.ctx.handle, self._h, len(kr), _p(kr), _p(kp), len(lr), _p(lr),
                                                 _p(lp), C.byref(nk), C.byref(nl)))
        return kr[:nk.value], kp[:nk.value], lr[:nl.value], lp[:nl.value]

    def results_view(self):
        """vx_ba_dmap_results_view (prefetching on): the same four arrays as results(), read from the
        pinned block the last optimize() filled (copied here; the C++ adapter reads them in place)."""
        kr, lr = C.POINTER(C.c_int32)(), C.POINTER(C.c_int32)()
        kp, lp = C.POINTER(C.c_double)(), C.POINTER(C.c_double)()
        nk, nl = C.c_int(0), C.c_int(0)
        self.ctx._check(lib().vx_ba_dmap_results_view(self.ctx.handle, self._h, C.byref(kr), C.byref(kp), C.byref(lr),
                                                      C.byref(lp), C.byref(nk), C.byref(nl)))
        n, m = nk.value, nl.value
        if n == 0 and m == 0:
            return (np.zeros(0, np.int64), np.zeros((0, 7)), np.zeros(0, np.int64), np.zeros((0, 3)))
        k_rows = np.ctypeslib.as_array(kr, (n,)).astype(np.int64)
        k_pose = np.ctypeslib.as_array(kp, (n, 8))[:, :7].copy()
        l_rows = np.ctypeslib.as_array(lr, (m,)).astype(np.int64)
        l_pos = np.ctypeslib.as_array(lp, (m, 4))[:, :3].copy()
        return k_rows, k_pose, l_rows, l_pos

    def close(self):
        if self._h:
            lib().vx_dmap_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SBAPlan:
    """vx_sba_plan: Schur-complement joint BA plan (window, observation / block / pair tables)."""

    def __init__(self, ctx: Context, m, opts=None, ref_kf_id=None, shard_rank=0, shard_count=1):
        self.ctx = ctx
        self.opts = opts or default_sba_options(window=m.get("window", 5))
        ref = m.get("ref_kf_id") if ref_kf_id is None else ref_kf_id
        self._h = C.c_void_p()
        v = map_view(m)
        ctx._check(lib().vx_sba_plan_create(ctx.handle, C.byref(v), C.c_uint64(0 if ref is None else int(ref)),
                                            0 if ref is None else 1, C.byref(self.opts), shard_rank,
                                            shard_count, C.byref(self._h)))

    def info(self):
        out = np.zeros(8, np.int64)
        assert lib().vx_sba_plan_info(self._h, _p(out)) == 0
        keys = ["n_kf", "n_opt", "n_obs", "n_pairs", "n_blocks", "n", "n_tiles", "n_comp"]
        return {k: int(v) for k, v in zip(keys, out)}

    def factor_work(self):
        """vx_sba_plan_factor_work: the dense pose solve's tiles and its FP64 flops per factorisation."""
        out = np.zeros(4, np.int64)
        assert lib().vx_sba_plan_factor_work(self._h, _p(out)) == 0
        d = dict(zip(["l_tiles", "updates", "diag", "panel"], (int(x) for x in out)))
        d["flops"] = 2 * 16 ** 3 * d["updates"] + 16 ** 3 * d["panel"] + (16 ** 3 // 3) * d["diag"]
        return d

    def run_async(self):
        self.ctx._check(lib().vx_sba_plan_run_async(self.ctx.handle, self._h))

    def fetch(self, m=None) -> SBAStats:
        st = SBAStats()
        v = map_view(m) if m is not None else None
        self.ctx._check(lib().vx_sba_plan_fetch(self.ctx.handle, self._h, C.byref(v) if v is not None else None,
                                                C.byref(st)))
        return st

    def apply(self, dmap):
        """vx_sba_plan_apply_dmap: the run's best state into the resident map (plans from DMap.sba_plan)."""
        self.ctx._check(lib().vx_sba_plan_apply_dmap(self.ctx.handle, self._h, dmap.handle))

    def system(self):
        """(S, rhs) of the last assembly (lower triangle of S meaningful, damping included)."""
        n = self.info()["n"]
        S = np.zeros((n, n))
        rhs = np.zeros(n)
        self.ctx._check(lib().vx_sba_plan_system(self.ctx.handle, self._h, _p(S), _p(rhs), n))
        return S, rhs

    def close(self):
        if self._h:
            lib().vx_sba_plan_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def dmap_load(dmap: DMap, m, kf_rows=None):
    """Insert a synth.BAMap into a DMap the way a running system builds its map: keyframes in
    ascending id order (``kf_rows`` limits it to those snapshot rows, in that order), each with its
    features; the landmarks first observed by that keyframe; then that keyframe's observations
    (Landmark::AddObservation, in landmark order).  Returns (kf_order, lm_order): the snapshot
    keyframe / landmark rows in the DMap's insertion order (landmarks never observed go last)."""
    ids = m["kf_id"]
    kf_order = np.argsort(ids, kind="stable") if kf_rows is None else np.asarray(kf_rows)
    optr = m["lm_obs_ptr"]
    obs_lm = np.repeat(np.arange(len(m["lm_id"])), np.diff(optr))
    obs_kf = m["obs_kf_id"]
    seen = np.zeros(len(m["lm_id"]), bool)
    lm_order = []
    for k in kf_order:
        f0, f1 = m["kf_feat_ptr"][k], m["kf_feat_ptr"][k + 1]
        dmap.add_keyframe(ids[k], m["kf_pose"].reshape(-1, 7)[k], m["kf_intr"].reshape(-1, 4)[k], m["kf_has_cam"][k],
                          m["feat_uv"].reshape(-1, 2)[f0:f1], m["feat_lm_id"][f0:f1], m["feat_flags"][f0:f1])
        sel = np.nonzero(obs_kf == ids[k])[0]  # observation rows of this keyframe, landmark order
        new = np.unique(obs_lm[sel][~seen[obs_lm[sel]]])
        if len(new):
            dmap.add_landmarks(m["lm_id"][new], m["lm_pos"].reshape(-1, 3)[new], m["lm_bad"][new])
            seen[new] = True
            lm_order.extend(new.tolist())
        if len(sel):
            dmap.add_observations(m["lm_id"][obs_lm[sel]], obs_kf[sel], m["obs_feat_idx"][sel])
    if kf_rows is None:
        rest = np.nonzero(~seen)[0]
        if len(rest):
            dmap.add_landmarks(m["lm_id"][rest], m["lm_pos"].reshape(-1, 3)[rest], m["lm_bad"][rest])
            lm_order.extend(rest.tolist())
    return np.asarray(kf_order), np.asarray(lm_order, np.int64)


def map_reorder(m, kf_order, lm_order):
    """The snapshot with its keyframe / landmark rows permuted (per-landmark observation lists kept);
    the result has the input's type (a synth.BAMap stays one, so its deep .copy() is kept)."""
    out = type(m)(m)
    fp = m["kf_feat_ptr"]
    cnt = np.diff(fp)[kf_order]
    out["kf_id"] = m["kf_id"][kf_order].copy()
    out["kf_pose"] = m["kf_pose"].reshape(-1, 7)[kf_order].copy()
    out["kf_intr"] = m["kf_intr"].reshape(-1, 4)[kf_order].copy()
    out["kf_has_cam"] = m["kf_has_cam"][kf_order].copy()
    out["kf_feat_ptr"] = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
    fidx = np.concatenate([np.arange(fp[k], fp[k + 1]) for k in kf_order]) if len(kf_order) else np.zeros(0, int)
    out["feat_uv"] = m["feat_uv"].reshape(-1, 2)[fidx].copy()
    out["feat_lm_id"] = m["feat_lm_id"][fidx].copy()
    out["feat_flags"] = m["feat_flags"][fidx].copy()
    optr = m["lm_obs_ptr"]
    out["lm_id"] = m["lm_id"][lm_order].copy()
    out["lm_pos"] = m["lm_pos"].reshape(-1, 3)[lm_order].copy()
    out["lm_bad"] = m["lm_bad"][lm_order].copy()
    ocnt = np.diff(optr)[lm_order]
    out["lm_obs_ptr"] = np.concatenate([[0], np.cumsum(ocnt)]).astype(np.int64)
    oidx = np.concatenate([np.arange(optr[l], optr[l + 1]) for l in lm_order]) if len(lm_order) else np.zeros(0, int)
    out["obs_kf_id"] = m["obs_kf_id"][oidx].copy()
    out["obs_feat_idx"] = m["obs_feat_idx"][oidx].copy()
    return out
