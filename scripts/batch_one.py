"""One batched-extraction configuration in a loop (for rocprofv3 passes):
    python scripts/batch_one.py [B] [C3|C4] [K]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import torch  # noqa: E402
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
h, w, n = (960, 1280, 4000) if (sys.argv[2:3] == ["C4"]) else (480, 640, 2000)
K = int(sys.argv[3]) if len(sys.argv) > 3 else 20
ctx = vxslam.Context(0)
ctx.set_grid_share(1.0 / B)
p = vxslam.default_orb_params(n_features=n)
pool = torch.from_numpy(synth.make_frames(11, B, h, w)).cuda()
for r in range(K):
    ctx.orb_extract_batch_async(pool.data_ptr(), B, pool.stride(0), w, h, 3, pool.stride(1), r % 2, p)
ctx.synchronize()
print("done", B, h, w)
