"""ORB extraction alone, for counter passes: `rocprofv3 --pmc ... -- python3 scripts/orb_loop.py [C4]`
(C3: 640x480, 2000 features; C4: 1280x960, 4000), $VX_ORB_LOOP_N (30) synchronous extractions of one frame."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

h, w, n = (960, 1280, 4000) if sys.argv[1:] == ["C4"] else (480, 640, 2000)
f = synth.make_frames(0x5EED0003, 1, h, w)[0]
ctx = vxslam.Context(0)
p = vxslam.default_orb_params(n_features=n)
for _ in range(int(os.environ.get("VX_ORB_LOOP_N", "30"))):
    ctx.orb_extract(f, p)
ctx.close()
