"""Extraction throughput with several frames in flight (extraction at 640x480 is
latency-bound, so report it batched too): S contexts (one HIP stream each, grid share 1/S)
extract S different frames concurrently, round after round; frames/s and us/frame against one
context extracting serially.  Usage: extract_throughput.py [C3|C4]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import torch  # noqa: E402
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

h, w, n = (960, 1280, 4000) if sys.argv[1:] == ["C4"] else (480, 640, 2000)
frames = torch.from_numpy(synth.make_frames(11, 8, h, w)).cuda()
params = vxslam.default_orb_params(n_features=n)
for S in (1, 2, 4, 8):
    ctxs = [vxslam.Context(0) for _ in range(S)]
    for c in ctxs:
        c.set_grid_share(1.0 / S)
    K = 200 // S

    def rnd(r):
        for s, c in enumerate(ctxs):
            c.orb_extract_async(frames[(r * S + s) % 8].data_ptr(), w, h, 3, w * 3, r % 3, params)

    for r in range(6):
        rnd(r)
    for c in ctxs:
        c.synchronize()
    t0 = time.perf_counter()
    for r in range(K):
        rnd(r)
    for c in ctxs:
        c.synchronize()
    dt = time.perf_counter() - t0
    print(f"{h}x{w} n={n}: {S} frames in flight: {1e6 * dt / (K * S):7.2f} us/frame  "
          f"({K * S / dt:8.0f} frames/s)", flush=True)
    for c in ctxs:
        c.close()
