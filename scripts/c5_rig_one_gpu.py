"""The C5 multi-camera workload on ONE MI355X: 8 camera streams of 640x480 BGR8 frames (2000 ORB
each) and one global window of 200 keyframes (8 streams x 25) / 100k landmarks.  A rig step is:
batched extraction of the 8 frames (vx_orb_extract_batch_async, bank t % 2), batched matching of
each camera's frame against its previous one (vx_match_batch_async, 8 pairs), then the global BA
of the step — LocalBA (the reference's alternating solver, <= 5 iterations) or the Schur-complement
joint BA (vx_sba_*, 8 LM iterations).  Frontend and BA run on two contexts; BA(t) waits for
Match(t) (device event), so the frontend of step t+1 overlaps BA(t).  Prints one JSON line per BA
kind with ms per rig step and per frame (everything resident in HBM, K timed steps after warm-up).

    python scripts/c5_rig_one_gpu.py [K]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import torch  # noqa: E402
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 200
CAMS, H, W, N = 8, 480, 640, 2000
nk, nl, ns = synth.ba_config("C5")
front, back = vxslam.Context(0), vxslam.Context(0)
params = vxslam.default_orb_params(n_features=N)
pool = torch.from_numpy(synth.make_frames(0xC5, 4 * CAMS, H, W)).cuda()  # 4 time steps x 8 cameras
m = synth.make_ba_map(0x5EED0000 + nk, nk, nl, n_streams=ns, n_old_kf=2 * ns)
plans = {"local_ba": back.ba_plan(m, vxslam.default_ba_options(window=nk)),
         "schur_ba": back.sba_plan(m.copy(), vxslam.default_sba_options(window=nk, iters=8))}
ev = front.event()


def step(t, plan, overlap=True):
    bank = t % 2
    base = (t % 4) * CAMS
    front.orb_extract_batch_async(pool[base].data_ptr(), CAMS, pool.stride(0), W, H, 3, pool.stride(1), bank, params)
    if t > 0:
        front.match_batch_async([(front.batch_device(1 - bank, c), front.batch_device(bank, c)) for c in range(CAMS)])
    front.record(ev)
    back.wait_event(ev)
    plan.run_async()
    if not overlap:
        back.synchronize()


for kind, plan in plans.items():
    res = {}
    for overlap in (True, False):
        for t in range(6):
            step(t, plan, overlap)
        front.synchronize()
        back.synchronize()
        kk = K if overlap else max(20, K // 4)
        t0 = time.perf_counter()
        for t in range(6, 6 + kk):
            step(t, plan, overlap)
        front.synchronize()
        back.synchronize()
        res[overlap] = 1e3 * (time.perf_counter() - t0) / kk
    # the BA alone on its context (graph replay)
    for _ in range(3):
        plan.run_async()
    back.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        plan.run_async()
    back.synchronize()
    ba_ms = 1e3 * (time.perf_counter() - t0) / 50
    print(json.dumps({"workload": "C5 on one GPU: 8 cameras x 640x480 / 2000 ORB, batched extract + match, "
                      f"{kind} over {nk} KF / {nl} landmarks ({ns} streams)", "ba": kind,
                      "ms_per_rig_step": round(res[True], 4), "ms_per_frame": round(res[True] / CAMS, 4),
                      "ms_per_rig_step_serial": round(res[False], 4), "ba_alone_ms": round(ba_ms, 4),
                      "steps": K}), flush=True)
    plan.close()
front.close()
back.close()
