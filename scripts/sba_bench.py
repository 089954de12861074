"""Schur-complement joint BA (vx_sba_*) on one MI355X: C3 window (50 KF / 20k landmarks) and the C5
global window (8 camera streams x 25 KF = 200 KF, 100k landmarks: 8 covisibility components, one
dense MFMA solve each).  Prints one JSON line per config: ms per optimisation (K replays of the
resident plan, 8 Levenberg-Marquardt iterations max), iterations, cost, per-kernel us (HIP events,
separate pass), plan-build ms (host)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
ctx = vxslam.Context(0)
CFGS = [("C3", synth.ba_config("C3"), 0.0), ("C5", synth.ba_config("C5"), 0.0),
        ("C5-connected", synth.ba_config("C5"), 0.03)]  # (round 4: the rig as one covisibility component)
only = os.environ.get("SBA_CFGS")
for cfg, (nk, nl, ns), cf in CFGS:
    if only and cfg not in only.split(","):
        continue
    m = synth.make_ba_map(0x5EED0000 + nk, nk, nl, n_streams=ns, n_old_kf=2 * ns, cross_frac=cf)
    opts = vxslam.default_sba_options(window=nk, iters=8)
    builds = []
    for rep in range(3):  # the first build also allocates the plan's device buffers
        t0 = time.perf_counter()
        plan = ctx.sba_plan(m, opts)
        builds.append(1e3 * (time.perf_counter() - t0))
        if rep < 2:
            plan.close()
    build_ms = min(builds)
    for _ in range(3):
        plan.run_async()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        plan.run_async()
    ctx.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / K
    st = plan.fetch()
    ctx.prof_enable(True)
    plan.run_async()
    plan.fetch()
    prof = ctx.prof_read()
    ctx.prof_enable(False)
    # the dense pose solve on MFMA: algorithmic FP64 flops of the symbolic tile
    # factorisation (vx_sba_plan_factor_work) per factorisation, times the factorisations of the run
    # (every iteration before the last that is not a rejection), over the run's sba_solve time
    work = plan.factor_work()
    steps = [int(x) for x in list(st.step)[:st.iterations]]
    n_fac = sum(1 for i in range(max(st.iterations - 1, 0)) if steps[i] != 0)
    solve_ms = prof.get("sba_solve", (0.0, 0))[0]
    tfs = work["flops"] * n_fac / (solve_ms * 1e-3) / 1e12 if solve_ms > 0 else None
    mfma = {"flops_per_factorisation": work["flops"], "factorisations": n_fac, "solve_ms_per_run": round(solve_ms, 4),
            "achieved_tflops": round(tfs, 4) if tfs else None, "peak_tflops": 78.6,
            "fp64_frac": round(tfs / 78.6, 6) if tfs else None, "tiles": work}
    print(json.dumps({"config": cfg, "window_kf": nk, "landmarks": nl, "streams": ns, "plan": plan.info(),
                      "ms_per_optimize": round(ms, 4), "iterations": st.iterations, "accepted": st.accepted,
                      "cost": [round(st.initial_cost, 1), round(st.final_cost, 1)],
                      "plan_build_ms_host": round(build_ms, 2), "plan_build_ms_host_first": round(builds[0], 2),
                      "factor": os.environ.get("VX_SBA_FACTOR", "auto: blocked multi-workgroup where the block LDS fits"),
                      "kernel_us_per_launch": {k: round(v[0] * 1e3 / v[1], 2) for k, v in prof.items()
                                               if k.startswith("sba") and v[1]},
                      "kernel_us_per_iteration": {k: round(v[0] * 1e3 / max(st.iterations, 1), 2)
                                                  for k, v in prof.items() if k.startswith("sba") and v[1]},
                      "mfma_fp64": mfma}),
          flush=True)
    plan.close()
ctx.close()
