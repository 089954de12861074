"""Time of building a LocalBA plan (window selection + landmark set + CSRs): from a map snapshot
with the host reference build, with the device build (snapshot uploaded), and from the
device-resident map (vx_dmap: nothing uploaded but the window's keyframe tables; the observation
CSR re-sorted after the keyframe's insertion), plus the per-keyframe cost of updating the resident
map (add_keyframe + new landmarks + observations).  C2 / C3 / C4, one JSON line each."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

ctx = vxslam.Context(0)
for cfg in ("C2", "C3", "C4"):
    nk, nl, ns = synth.ba_config(cfg)
    m = synth.make_ba_map(0x5EED0003, nk, nl)
    o = vxslam.default_ba_options(window=nk)
    res = {"config": cfg, "window_kf": nk, "landmarks": nl}
    for hb in (False, True):
        for _ in range(2):
            ctx.ba_plan(m, o, host_build=hb).close()
        tc = td = 0.0
        for _ in range(10):
            t0 = time.perf_counter()
            pl = ctx.ba_plan(m, o, host_build=hb)
            t1 = time.perf_counter()
            pl.close()
            tc += t1 - t0
            td += time.perf_counter() - t1
        key = "host_build_ms" if hb else "device_build_ms"
        res[key] = round(1e3 * (tc + td) / 10, 3)
        res[key.replace("_ms", "_destroy_ms")] = round(1e3 * td / 10, 3)
    # resident map: all keyframes but the newest inserted; then time inserting the newest keyframe
    # (features, first-seen landmarks, observations) and building the plan from the resident map
    order = np.argsort(m["kf_id"], kind="stable")
    mir_lm = np.repeat(np.arange(len(m["lm_id"])), np.diff(m["lm_obs_ptr"]))
    upd, build = [], []
    for rep in range(6):
        dm = vxslam.DMap(ctx)
        vxslam.dmap_load(dm, m, kf_rows=order[:-1])
        k = order[-1]
        f0, f1 = m["kf_feat_ptr"][k], m["kf_feat_ptr"][k + 1]
        sel = np.nonzero(m["obs_kf_id"] == m["kf_id"][k])[0]
        seen = np.zeros(len(m["lm_id"]), bool)
        seen[mir_lm[np.isin(m["obs_kf_id"], m["kf_id"][order[:-1]])]] = True
        new = np.unique(mir_lm[sel][~seen[mir_lm[sel]]])
        ctx.synchronize()
        t0 = time.perf_counter()
        dm.add_keyframe(m["kf_id"][k], m["kf_pose"].reshape(-1, 7)[k], m["kf_intr"].reshape(-1, 4)[k],
                        m["kf_has_cam"][k], m["feat_uv"].reshape(-1, 2)[f0:f1], m["feat_lm_id"][f0:f1],
                        m["feat_flags"][f0:f1])
        if len(new):
            dm.add_landmarks(m["lm_id"][new], m["lm_pos"].reshape(-1, 3)[new], m["lm_bad"][new])
        dm.add_observations(m["lm_id"][mir_lm[sel]], m["obs_kf_id"][sel], m["obs_feat_idx"][sel])
        ctx.synchronize()
        t1 = time.perf_counter()
        dm.plan(o, ref_kf_id=int(m["kf_id"][k])).close()
        t2 = time.perf_counter()
        if rep >= 1:
            upd.append(t1 - t0)
            build.append(t2 - t1)
        dm.close()
    res["dmap_update_ms"] = round(1e3 * float(np.median(upd)), 3)
    res["dmap_build_ms"] = round(1e3 * float(np.median(build)), 3)
    print(json.dumps(res), flush=True)
ctx.close()
