"""Match alone (one context, graph replay): ms per vx_match_device_async of two C3 frames' descriptor
slots (2000 ORB each), for the kernel shape of the environment ($VX_MATCH_SHAPE, $VX_MATCH_GRID,
read once per process); checks the matches against the oracle first.

    python scripts/match_alone.py [reps]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch  # noqa: E402,F401  (its HIP runtime first, as in the tests)
import pyoracle  # noqa: E402
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
frames = synth.make_frames(0x5EED0005, 2, 480, 640)
fd = torch.from_numpy(frames).cuda()
c = vxslam.Context(0)
p = vxslam.default_orb_params(n_features=2000)
for s in range(2):
    c.orb_extract_async(fd[s].data_ptr(), 640, 480, 3, 640 * 3, s, p)
c.synchronize()
sl = [c.slot_device(s) for s in range(2)]
c.match_device_async(sl[0], sl[1])
c.synchronize()
d = [c.orb_fetch(s)[1] for s in range(2)]
assert np.array_equal(c.match_fetch(), pyoracle.match(d[0], d[1])), "match parity failed"
for _ in range(20):
    c.match_device_async(sl[0], sl[1])
c.synchronize()
best = 1e9
for rep in range(3):
    t0 = time.perf_counter()
    for _ in range(K):
        c.match_device_async(sl[0], sl[1])
    c.synchronize()
    best = min(best, 1e3 * (time.perf_counter() - t0) / K)
env = [k + "=" + v for k, v in os.environ.items() if k.startswith("VX_MATCH")]
print(f"match {len(d[0])} x {len(d[1])} env {env}: {best * 1e3:.2f} us/call (host-side replay rate)", flush=True)
c.close()
