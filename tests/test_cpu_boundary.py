"""The C-ABI boundary without a GPU: the library loads, exports every symbol include/vx_slam.h
declares, carries the right pattern table, plans BA windows on the host, and fails cleanly when
no device exists.  No compute call runs here."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import vxslam
from vxslam import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "vx_slam.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vx_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", vxslam.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (vx_[a-z0-9_]+)$", out, flags=re.M))
    declared = header_functions()
    assert len(declared) >= 30
    missing = [f for f in declared if f not in exported]
    assert not missing, missing
    lib = vxslam.lib()
    for f in declared:
        assert hasattr(lib, f)
    assert set(vxslam.EXPORTS) <= set(declared)


def test_library_is_gfx950_code():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", vxslam.LIB_PATH],
                         capture_output=True, text=True)
    blob = open(vxslam.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_pattern_table_matches_fixture(oracle):
    assert np.array_equal(vxslam.pattern(), oracle.load_pattern())


def test_default_params_mirror_reference():
    p = vxslam.OrbParams()
    vxslam.lib().vx_orb_default_params(C.byref(p))
    assert (p.n_features, p.n_levels, p.fast_threshold, p.edge_threshold) == (1000, 8, 20, 31)
    assert abs(p.scale_factor - 1.2) < 1e-6
    o = vxslam.BAOptions()
    vxslam.lib().vx_ba_default_options(C.byref(o))
    # LocalBA::Options defaults, core/backend/local_ba.h:12-19
    assert (o.window_size, o.max_iterations, o.min_pose_observations, o.min_point_observations) == (5, 5, 20, 2)
    assert (o.huber_delta, o.max_reproj_error) == (5.0, 5.0)


def _has_gpu():
    try:
        import torch

        return torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.mark.skipif(_has_gpu(), reason="checks the no-device error path")
def test_create_fails_cleanly_without_device():
    h = C.c_void_p()
    rc = vxslam.lib().vx_create(0, C.byref(h))
    assert rc != 0 and not h.value
    with pytest.raises(vxslam.VxError):
        vxslam.Context(0)


def test_host_plan_matches_oracle_selection(oracle):
    for seed, nk, nl, ref_off in [(1, 10, 2000, 0), (2, 6, 800, 2), (3, 12, 1500, 5)]:
        m = synth.make_ba_map(seed, nk, nl, n_old_kf=3)
        ref = int(m["kf_id"][-1 - ref_off])
        opts = oracle.ba_options(window=nk)
        d = vxslam.ba_plan_inspect(m, vxslam.default_ba_options(window=nk), ref_kf_id=ref)
        st = oracle.ba_optimize(m.copy(), opts, ref_kf_id=ref)
        assert d["status"] == st.status
        assert d["n_window_kf"] == st.n_window_kf
        assert d["n_landmarks"] == st.n_landmarks
        # window = the newest keyframes with id <= ref, ascending
        ids = m["kf_id"][d["kf_map_idx"]]
        assert (np.diff(ids.astype(np.int64)) > 0).all() and ids[-1] == ref


def test_host_plan_early_returns():
    m = synth.make_ba_map(5, 5, 300, n_old_kf=0)
    d = vxslam.ba_plan_inspect(m, vxslam.default_ba_options(window=5), ref_kf_id=int(m["kf_id"][0]))
    assert d["status"] == 1 and d["n_window_kf"] == 1
    d = vxslam.ba_plan_inspect(m, vxslam.default_ba_options(window=5, min_point=99))
    assert d["status"] == 1 and d["n_landmarks"] == 0


def test_sharded_plans_partition_the_window():
    m = synth.make_ba_map(6, 10, 3000, n_old_kf=2)
    opts = vxslam.default_ba_options(window=10)
    full = vxslam.ba_plan_inspect(m, opts)
    for n in (2, 3, 8):
        parts = [vxslam.ba_plan_inspect(m, opts, shard_rank=r, shard_count=n) for r in range(n)]
        opt_sets = [set(p["lm_map_idx"][:p["n_opt"]].tolist()) for p in parts]
        all_opt = set().union(*opt_sets)
        assert sum(len(s) for s in opt_sets) == len(all_opt) == full["n_opt"]
        assert sum(p["n_pose_obs"] for p in parts) == full["n_pose_obs"]
        assert sum(p["n_lm_obs"] for p in parts) == full["n_lm_obs"]
        for r, p in enumerate(parts):
            assert all(vxslam.ba_shard_of(int(m["lm_id"][l]), n) == r for l in p["lm_map_idx"])


def test_host_alloc_round_trip():
    """vx_host_alloc: page-locked host memory with a device, plain pageable memory without one (the
    snapshot arrays of visionx::FlatMap use it); 64-byte aligned, writable, freed by vx_host_free."""
    L = vxslam.lib()
    for n in (1, 1000, 1 << 20):
        p = L.vx_host_alloc(n)
        assert p and p % 64 == 0
        buf = (C.c_uint8 * n).from_address(p)
        buf[n - 1], buf[0] = 9, 7
        assert (buf[0], buf[n - 1]) == (7, 9 if n > 1 else 7)
        L.vx_host_free(p)
    L.vx_host_free(None)
