"""Host cost per call of the pipeline's enqueue calls (no synchronisation inside the timed loop):
the bench's step is host-bound when these add up to its ms/frame.  `python scripts/host_cost.py`"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import torch  # noqa: E402

torch.zeros(1, device="cuda")
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

e = [vxslam.Context(0), vxslam.Context(0)]
b = vxslam.Context(0)
for c in e:
    c.set_grid_share(1.0 / 3.0)
frames = torch.from_numpy(synth.make_frames(7, 8, 480, 640)).cuda()
params = vxslam.default_orb_params(n_features=2000)
plan = b.ba_plan(synth.make_ba_map(0x5EED0003, 50, 20000), vxslam.default_ba_options(window=50))
ev = e[0].event()
for s in range(3):
    e[0].orb_extract_async(frames[s].data_ptr(), 640, 480, 3, 640 * 3, s, params)
slots = [e[0].slot_device(s) for s in range(3)]
torch.cuda.synchronize()
for c in e + [b]:
    c.synchronize()


def bench(name, fn, n=200):
    for _ in range(10):
        fn(0)
    for c in e + [b]:
        c.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        fn(i)
    t1 = time.perf_counter()
    for c in e + [b]:
        c.synchronize()
    t2 = time.perf_counter()
    print(f"{name:28s} host {1e6 * (t1 - t0) / n:7.2f} us/call   (with drain {1e6 * (t2 - t0) / n:7.2f})", flush=True)


bench("ba plan.run_async", lambda i: plan.run_async())
bench("orb_extract_async", lambda i: e[0].orb_extract_async(frames[i % 8].data_ptr(), 640, 480, 3, 640 * 3, i % 3, params))
bench("match_device_async", lambda i: e[0].match_device_async(slots[i % 3], slots[(i + 1) % 3]))
bench("record", lambda i: e[0].record(ev))
bench("wait_event", lambda i: b.wait_event(ev))
