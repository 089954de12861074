"""LocalBA (C3) per-run time alone and beside three kinds of concurrent load on another stream:
a streaming copy (evicts the L2s, little compute), a compute-bound FP32 matmul that fits in cache,
and the ORB extraction of bench.py (two contexts, frames alternate).  Tells whether the pipeline's
LocalBA slowdown is memory-system or compute interference."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import torch  # noqa: E402
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

b = vxslam.Context(0)
plan = b.ba_plan(synth.make_ba_map(0x5EED0003, 50, 20000), vxslam.default_ba_options(window=50))
src = torch.empty(64 << 20, dtype=torch.float32, device="cuda")  # 256 MB
dst = torch.empty_like(src)
A = torch.randn(2048, 2048, device="cuda")
side = torch.cuda.Stream()
e = [vxslam.Context(0), vxslam.Context(0)]
for c in e:
    c.set_grid_share(1.0 / 3.0)
frames = torch.from_numpy(synth.make_frames(7, 8, 480, 640)).cuda()
params = vxslam.default_orb_params(n_features=2000)
torch.cuda.synchronize()


def load(kind, i):
    if kind == "copy":
        with torch.cuda.stream(side):
            dst.copy_(src)
    elif kind == "write":  # streaming writes only: dirty lines in the L2s
        with torch.cuda.stream(side):
            dst.zero_()
    elif kind == "read":  # streaming reads only
        with torch.cuda.stream(side):
            src.sum()
    elif kind == "matmul":
        with torch.cuda.stream(side):
            for _ in range(4):
                torch.mm(A, A)
    elif kind == "extract":
        c = e[i % 2]
        c.orb_extract_async(frames[i % 8].data_ptr(), 640, 480, 3, 640 * 3, (i // 2) % 3, params)


for kind in ("none", "copy", "write", "read", "matmul", "extract"):
    for i in range(5):
        plan.run_async()
        load(kind, i)
    torch.cuda.synchronize()
    for c in e + [b]:
        c.synchronize()
    K = 100
    t_ba = 0.0
    for i in range(K):
        load(kind, i)
        b.synchronize()
        t0 = time.perf_counter()
        plan.run_async()
        b.synchronize()
        t_ba += time.perf_counter() - t0
    torch.cuda.synchronize()
    print(f"LocalBA beside {kind:8s}: {1e3 * t_ba / K:.4f} ms/run (host-timed, synchronous)", flush=True)
