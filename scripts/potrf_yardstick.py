"""Library yardstick for the Schur dense pose solve (measurement only, never shipped):
the connected C5 window's reduced pose system S (n = 6 x free keyframes, from vx_sba_plan_system)
factored by torch.linalg.cholesky (ROCm: rocSOLVER / hipSOLVER potrf) and solved by cholesky_solve
in FP64 on the same GPU, against vx_sba's own sba_solve time per LM iteration (HIP events, the plan's
profiling pass).  Prints one JSON line.

    python scripts/potrf_yardstick.py [reps]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import torch  # noqa: E402  (HIP initialised before the library)

torch.zeros(1, device="cuda")
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
ctx = vxslam.Context(0)
nk, nl, ns = synth.ba_config("C5")
m = synth.make_ba_map(0x5EED0000 + nk, nk, nl, n_streams=ns, n_old_kf=2 * ns, cross_frac=0.03)
opts = vxslam.default_sba_options(window=nk, iters=8)
plan = ctx.sba_plan(m, opts)
for _ in range(3):
    plan.run_async()
st = plan.fetch()
S, rhs = plan.system()
n = S.shape[0]
A = np.tril(S) + np.tril(S, -1).T  # (lower triangle meaningful)
ctx.prof_enable(True)
plan.run_async()
st = plan.fetch()
prof = ctx.prof_read()
ctx.prof_enable(False)
steps = [int(x) for x in list(st.step)[:st.iterations]]
n_fac = sum(1 for i in range(max(st.iterations - 1, 0)) if steps[i] != 0)
solve_ms = prof.get("sba_solve", (0.0, 0))[0]

At = torch.from_numpy(A).cuda()
bt = torch.from_numpy(rhs).cuda().reshape(-1, 1)


def lib_solve():
    L = torch.linalg.cholesky(At)
    return torch.cholesky_solve(bt, L)


for _ in range(5):
    x = lib_solve()
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for _ in range(reps):
    x = lib_solve()
ev1.record()
torch.cuda.synchronize()
lib_us = 1e3 * ev0.elapsed_time(ev1) / reps
t0 = time.perf_counter()
for _ in range(reps):
    L = torch.linalg.cholesky(At)
torch.cuda.synchronize()
potrf_us = 1e6 * (time.perf_counter() - t0) / reps
res = float(np.abs(A @ x.cpu().numpy().ravel() - rhs).max() / max(np.abs(rhs).max(), 1e-300))
print(json.dumps({"n": n, "lib": "torch.linalg.cholesky + cholesky_solve (FP64, ROCm)", "lib_potrf_potrs_us": round(lib_us, 1),
                  "lib_potrf_us_host_wall": round(potrf_us, 1), "lib_rel_residual": res,
                  "vx_sba_solve_us_per_factorisation": round(1e3 * solve_ms / max(n_fac, 1), 1),
                  "vx_factorisations": n_fac, "vx_iterations": st.iterations}), flush=True)
