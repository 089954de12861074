"""Is the pipelined C3 step host-enqueue-bound?  Times the host side of K steps (enqueue only)
against the elapsed time to completion, and the per-call host cost of each C-ABI entry point."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import torch  # noqa: E402
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

h, w, nf, nk, nl = 480, 640, 2000, 50, 20000
e, m, b = vxslam.Context(0), vxslam.Context(0), vxslam.Context(0)
frames = torch.from_numpy(synth.make_frames(7, 8, h, w)).cuda()
params = vxslam.default_orb_params(n_features=nf)
plan = b.ba_plan(synth.make_ba_map(0x5EED0003, nk, nl), vxslam.default_ba_options(window=nk))
ev_e = e.event()
ev_m = [m.event() for _ in range(3)]
for i in (-3, -2, -1):
    e.orb_extract_async(frames[i % 8].data_ptr(), w, h, 3, w * 3, i % 3, params)
slot = [e.slot_device(s) for s in range(3)]
T = {"wait": 0.0, "extract": 0.0, "rec": 0.0, "match": 0.0, "ba": 0.0}


def step(i, t=None):
    def tick(k, f):
        if t is None:
            f()
        else:
            a = time.perf_counter()
            f()
            t[k] += time.perf_counter() - a
    tick("wait", lambda: e.wait_event(ev_m[(i + 1) % 3]))
    tick("extract", lambda: e.orb_extract_async(frames[i % 8].data_ptr(), w, h, 3, w * 3, i % 3, params))
    tick("rec", lambda: (e.record(ev_e), m.wait_event(ev_e)))
    tick("match", lambda: m.match_device_async(slot[(i - 1) % 3], slot[i % 3]))
    tick("rec", lambda: (m.record(ev_m[i % 3]), b.wait_event(ev_m[i % 3])))
    tick("ba", lambda: plan.run_async())


for i in range(20):
    step(i)
for c in (e, m, b):
    c.synchronize()
K = 200
t0 = time.perf_counter()
for i in range(K):
    step(20 + i)
t1 = time.perf_counter()
for c in (e, m, b):
    c.synchronize()
t2 = time.perf_counter()
print(f"host enqueue {1e3 * (t1 - t0) / K:.4f} ms/step, to completion {1e3 * (t2 - t0) / K:.4f} ms/step")
for c in (e, m, b):
    c.synchronize()
for i in range(K):
    step(300 + i, T)
for c in (e, m, b):
    c.synchronize()
print("host us per call group:", {k: round(1e6 * v / K, 1) for k, v in T.items()})
