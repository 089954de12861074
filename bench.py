#!/usr/bin/env python3
"""bench.py — VisionX-SLAM hot path on MI355X: ms/frame of ORB extract + match + local BA.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3]
    torchrun --nproc-per-node N ... bench.py --gpus N ...

One step = eight rounds of the pipeline: F frames (F = 8 x the extraction contexts, 24 by default;
--frames-per-step), each through the hot path, everything resident in HBM before timing starts:
  1. ORBExtractor::Extract of a 640x480 BGR8 frame (n_features 2000 at C3)   -> slot i % 3
  2. ORBMatcher::Match(previous frame, this frame): BF Hamming kNN-2 + ratio -> matches
  3. LocalBA::Optimize over the sliding window (C3: 50 KF / 20k landmarks, <= 5 iterations)
Each stage runs on its own context (HIP stream), ordered on the device by events that follow the
data dependencies (Match(t) after Extract(t), LocalBA(t) after Match(t), Extract(t) after
Match(t-2) which last read its slot), so Extract(t+1), Match(t) and LocalBA(t-1) overlap
(--streams 1 puts everything on one stream).  Every step's work completes inside the timed
region; `latency_ms_per_frame` is one frame alone through the same chain.
At N GPUs (weak scaling, "rig" workload): every rank runs steps 1-2 on its own camera stream and
the ranks jointly run ONE global window of N x 50 KF / N x 20k landmarks per step, landmarks
sharded across ranks with one RCCL all-reduce of the per-keyframe normal equations per
iteration.  value = elapsed / (frames processed by all ranks) in ms/frame (lower is better).

Rank 0 prints ONE JSON line.  Diagnostics go to stderr.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))

import numpy as np  # noqa: E402

METRIC = "ms/frame (feature-extract+match + BA solve), 640×480, 50 KF / 20k pts"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# profiling stage -> the HIP kernel it brackets (the name in the rocprofv3 summaries)
HIP_KERNEL = {"orb_pyramid": "k_pyramid", "orb_fast_harris": "k_fast", "orb_select": "k_select_stl",
              "orb_blur": "k_blur", "orb_describe": "k_describe", "match_partial": "k_knn_rows",
              "match_merge": "k_knn_compact", "ba_pose_partial": "k_pose_kf",
              "ba_landmark": "k_landmark_solve", "ba_iter": "k_ba_iter", "ba_prologue": "k_ba_iter",
              "ba_window": "k_ba_win"}

CONFIGS = {
    # name: (height, width, n_features, n_kf, n_lm)
    "C2": (480, 640, 1000, 10, 2000),
    "C3": (480, 640, 2000, 50, 20000),
    "C4": (960, 1280, 4000, 100, 50000),
    # C5: 8 camera streams of 640x480 / 2000 ORB (per camera), one global 200 KF / 100k window
    # solved by the Schur-complement BA (bench_c5 below)
    "C5": (480, 640, 2000, 200, 100000),
}
C5_CAMERAS = 8


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# LocalBA::Options as the reference runner names them (apps/main.cpp:42-47 -> tracking options)
BA_FLAGS = {"ba_window_size": int, "ba_iterations": int, "ba_min_pose_observations": int,
            "ba_min_point_observations": int, "ba_huber_delta": float, "ba_max_reproj_error": float}


def load_config_file(path):
    """apps/main.cpp LoadConfig: key=value lines, '#' comments, surrounding whitespace trimmed; the
    reference warns about keys it does not know — here everything but the ba_* keys is outside the
    measured path and ignored with a note."""
    kv = {}
    with open(path) as f:
        for line in f:
            line = line.split("#", 1)[0].strip()
            if not line or "=" not in line:
                continue
            k, v = (x.strip() for x in line.split("=", 1))
            kv[k] = v
    return kv


def resolve_ba_flags(args, window_default):
    """The LocalBA options of this run: command-line flags over the config file's ba_* keys over the
    workload's defaults (window = the configuration's keyframes; the rest the reference defaults,
    default.cfg)."""
    vals = {"ba_window_size": window_default, "ba_iterations": 5, "ba_min_pose_observations": 20,
            "ba_min_point_observations": 2, "ba_huber_delta": 5.0, "ba_max_reproj_error": 5.0}
    if getattr(args, "config_file", None):
        kv = load_config_file(args.config_file)
        for k, typ in BA_FLAGS.items():
            if k in kv:
                vals[k] = typ(kv[k])
        other = sorted(k for k in kv if k not in BA_FLAGS)
        if other:
            log(f"note: config keys outside the measured path ignored: {', '.join(other)}")
    for k in BA_FLAGS:
        v = getattr(args, k, None)
        if v is not None:
            vals[k] = v
    return vals


# ----------------------------------------------------------------------------- algorithmic bytes
def stage_bytes(stage, geo, counts):
    """Algorithmic (compulsory) HBM bytes of ONE launch of a stage.  Formulas: DESIGN.md §4."""
    W, H, C = geo["W"], geo["H"], 3
    px = geo["level_px"]            # list of level pixel counts
    N = counts["n_kp"]
    if stage == "orb_gray":
        return W * H * C + W * H
    if stage == "orb_pyramid":      # BGR in, every level out
        return W * H * C + sum(px)
    if stage == "orb_resize":       # average over the L-1 launches
        return sum(px[l - 1] + px[l] for l in range(1, len(px))) / (len(px) - 1)
    if stage == "orb_fast_harris":  # every level read, blurred levels written, candidate records
        return 2 * sum(px) + 16 * counts["n_cand"]
    if stage == "orb_select":
        return 16 * counts["n_cand"] + 16 * N
    if stage == "orb_describe":
        return N * (16 + 20 + 32)
    if stage == "match_partial":    # k_knn_rows: both descriptor sets in, one key per query out
        return (counts["n_q"] + counts["n_t"]) * 32 + counts["n_q"] * 4
    if stage == "match_merge":      # k_knn_compact: the keys in, the ordered matches out
        return counts["n_q"] * 4 + counts["n_match"] * 12
    if stage == "ba_pose_partial":
        # per observation: uv 16 + landmark slot 4 + landmark position 24 (gathered); per slice
        # partial: 32 doubles written; per keyframe: pose 64 + intrinsics 32 read
        return counts["n_pose_obs"] * 44 + counts["n_kf"] * counts["n_split"] * 256 + counts["n_kf"] * 96
    if stage == "ba_landmark":
        # per observation: uv 16 + keyframe 4 + landmark slot 4; per landmark: position read 24 +
        # written 24 + CSR pointer 4; per keyframe: slice partials 29 x 8 each, pose 64 + intrinsics
        # 32 read, pose 64 + rotation 72 + cost 16 written (by workgroup 0)
        return (counts["n_lm_obs"] * 24 + counts["n_opt"] * 52 +
                counts["n_kf"] * (counts["n_split"] * 232 + 96 + 152))
    if stage == "ba_iter":
        # one fused launch = one iteration: SURVEY §8(d)'s per-iteration bytes (pose stage: uv 16 +
        # landmark slot 4 + landmark position 24 per observation; landmark stage: uv 16 + keyframe 4
        # per observation; landmark position read + written; per keyframe pose 56, intrinsics 32,
        # the 29-double normal-equation block) — 64 O + 48 LM + 320 KF with O split by stage
        return (counts["n_pose_obs"] * 44 + counts["n_lm_obs"] * 20 + counts["n_opt"] * 48 +
                counts["n_kf"] * 320)
    if stage == "ba_prologue":  # iteration 0's pose stage
        return counts["n_pose_obs"] * 44 + counts["n_kf"] * (56 + 32 + 232)
    if stage == "ba_window":    # k_ba_win: the prologue + the iterations the window ran, one launch
        return stage_bytes("ba_prologue", geo, counts) + counts["ba_iters"] * stage_bytes("ba_iter", geo, counts)
    return None


FP64_PEAK_TFS = 78.6  # MI355X FP64 vector rate (half the 157.3 TF FP32 vector peak, MI355X_MICROARCH.md)


def stage_flops(stage, counts):
    """FP64 operations of ONE fused LocalBA launch: per pose-stage observation the
    projection, gate, Huber weight, 2x6 Jacobian and the 27 normal-equation terms (~132 flops, every
    observation issued by the branch-free form); per landmark-stage observation projection, 2x3
    Jacobian and 9 terms (~80); per landmark the 3x3 solve (~50); per keyframe entry the 6x6 block
    solve and the SE(3) update (~400)."""
    if stage in ("ba_iter", "ba_prologue"):
        lm = stage == "ba_iter"
        return (132 * counts["n_pose_obs"] + (80 * counts["n_lm_obs"] + 50 * counts["n_opt"] if lm else 0) +
                400 * counts["n_kf"])
    if stage == "ba_window":
        return stage_flops("ba_prologue", counts) + counts["ba_iters"] * stage_flops("ba_iter", counts)
    return None


# ----------------------------------------------------------------------------- drop-in LocalBA
def per_keyframe_ms(bctx, ba_map, opts, dist, N, vxslam):
    """What one drop-in LocalBA::Optimize() (local_ba.cpp:66-249) costs end to end, host clock,
    median of 7 after 2 warm-ups: plan build + solve + the results written back, (a) from the
    host map snapshot (upload, device build, run, download into the snapshot) and (b) from the
    device-resident map (vx_dmap: build from the resident map, run, scatter into it)."""
    def med(f):
        t = []
        for i in range(9):
            t0 = time.perf_counter()
            f()
            if i >= 2:
                t.append(1e3 * (time.perf_counter() - t0))
        return round(float(np.median(t)), 3)

    m = ba_map.copy()

    def snap_call():
        bctx.ba_optimize(m, opts)

    def snap():
        p = bctx.ba_plan(m, opts)
        p.run_async()
        p.fetch(m)
        p.close()

    dm = vxslam.DMap(bctx)
    vxslam.dmap_load(dm, ba_map)
    bctx.synchronize()

    def resident():
        p = dm.plan(opts)
        p.run_async()
        p.apply(dm)
        bctx.synchronize()
        p.close()

    def one_call():
        dm.optimize(opts)

    try:
        out = {"snapshot": med(snap_call), "snapshot_plan": med(snap), "resident": med(resident),
               "resident_one_call": med(one_call)}
    finally:
        dm.close()
    out["cpp_adapter"] = cpp_adapter_ms(ba_map, opts)
    out["note"] = ("host wall clock of one LocalBA::Optimize, median of 7: snapshot = vx_ba_optimize_map (the "
                   "snapshot uploaded into the context's scratch device map, the one-call build, run and results in "
                   "one synchronisation; pageable numpy arrays here); snapshot_plan = a plan from the map snapshot "
                   "(upload, device build) + run + download; resident = vx_ba_plan_create_dmap + run + "
                   "vx_ba_plan_apply_dmap; resident_one_call = vx_ba_optimize_dmap (ba_lean.hip: build, run and "
                   "scatter with no host synchronisation before the end); cpp_adapter = visionx::LocalBA::Optimize "
                   "through tests/cpp/adapter_driver (median of 20 calls, results written back into the C++ "
                   "Frame / Landmark objects) with a DeviceMap attached and on the snapshot (Flatten) path. "
                   "value excludes all of these (a resident plan is replayed per frame)")
    return out


def cpp_adapter_ms(ba_map, opts, reps=20):
    """visionx::LocalBA::Optimize through the C++ drop-in (tests/cpp/adapter_driver ba_calls) on this
    window: median ms of one call after the first, resident (DeviceMap) and snapshot (Flatten)."""
    import subprocess
    import tempfile

    drv = os.path.join(ROOT, "visionx-slam_amd", "build", "adapter_driver")
    if not os.path.exists(drv):
        return None
    keys = ["kf_id", "kf_pose", "kf_intr", "kf_has_cam", "kf_feat_ptr", "feat_uv", "feat_lm_id", "feat_flags",
            "lm_id", "lm_pos", "lm_bad", "lm_obs_ptr", "obs_kf_id", "obs_feat_idx"]
    out = {}
    with tempfile.TemporaryDirectory() as d:
        for k in keys:
            np.ascontiguousarray(ba_map[k]).tofile(os.path.join(d, k + ".bin"))
        env = dict(os.environ, VX_DEVICE=os.environ.get("LOCAL_RANK", "0"))
        for mode in ("resident", "snapshot"):
            r = subprocess.run([drv, "ba_calls", d, str(opts.window_size), str(opts.max_iterations), "-1", str(reps),
                                mode], capture_output=True, text=True, timeout=300, env=env)
            if r.returncode != 0:
                log(f"[bench] adapter_driver {mode}: {r.stderr[-500:]}")
                out[mode] = None
                continue
            st = r.stdout.split()
            out[mode] = float(st[4])
            out[mode + "_stats"] = [int(x) for x in st[:4]]
    return out


# ----------------------------------------------------------------------------- distributed
class Dist:
    def __init__(self, n_gpus):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist

            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if not dist.is_initialized():
                dist.init_process_group(backend="gloo")  # control plane only; data path is RCCL
            self.pg = dist
        if n_gpus != self.world:
            log(f"note: --gpus {n_gpus} but WORLD_SIZE {self.world}; using WORLD_SIZE")

    def barrier(self):
        if self.pg:
            self.pg.barrier()

    def max(self, x):
        if not self.pg:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.MAX)
        return float(t.item())

    def gather(self, obj):
        """rank 0: the list of every rank's obj (rank order); other ranks: None"""
        if not self.pg:
            return [obj]
        out = [None] * self.world if self.rank == 0 else None
        self.pg.gather_object(obj, out, dst=0)
        return out

    def broadcast_bytes(self, b):
        if not self.pg:
            return b
        obj = [b]
        self.pg.broadcast_object_list(obj, src=0)
        return obj[0]

    def close(self):
        if self.pg:
            self.pg.destroy_process_group()


def timed_loop(step, steps, warmup, sync, dist):
    """W untimed warm-up steps, then K steps bracketed by barrier + device sync on both sides;
    returns the max over ranks of the elapsed seconds.  Python's cyclic collector is paused over
    the timed steps (a collection there is a host stall the pipeline cannot hide)."""
    import gc

    for i in range(warmup):
        step(i)
    late = os.environ.get("VX_BENCH_GC_LATE") == "1"
    if not late:  # (the collection overlaps the warm-up's tail on the device instead of idling it)
        gc.collect()
        gc.disable()
    sync()
    dist.barrier()
    sync()
    if late:
        gc.collect()
        gc.disable()
    try:
        t0 = time.perf_counter()
        for i in range(steps):
            step(warmup + i)
        timed_loop.enqueue_s = time.perf_counter() - t0  # host enqueue alone (diagnostic)
        sync()
        dist.barrier()
        t1 = time.perf_counter()
    finally:
        gc.enable()
    return dist.max(t1 - t0)


# ----------------------------------------------------------------------------- sharded-run parity
def shard_result(ba_map, plan_inspect, stats):
    """What a rank's sharded LocalBA run produced, after plan.fetch(ba_map): the window poses (every
    rank solves all of them), its own optimised landmarks (map index, position) and the
    per-iteration statistics (the all-reduced cost / observation counts)."""
    n_opt = plan_inspect["n_opt"]
    kf = plan_inspect["kf_map_idx"]
    lm = plan_inspect["lm_map_idx"][:n_opt]
    return {"kf_idx": np.asarray(kf, np.int64), "pose": np.asarray(ba_map["kf_pose"]).reshape(-1, 7)[kf].copy(),
            "lm_idx": np.asarray(lm, np.int64), "lm_pos": np.asarray(ba_map["lm_pos"]).reshape(-1, 3)[lm].copy(),
            "iterations": int(stats.iterations), "obs": [int(x) for x in list(stats.obs)[:int(stats.iterations)]]}


def parity_vs_unsharded(shards, ref, tol=1e-4):
    """Sharded LocalBA (one shard_result per rank, rank order) against the unsharded run of the same
    global window (a shard_result of the one-rank plan): SURVEY.md §8(e) / north_star's bar, i.e.
    |a - b| <= tol * max(|b|, 1e-3) per pose component (quaternion sign canonicalised) and landmark
    coordinate, the same iteration count and per-iteration observation counts (no gate flips), the
    landmark shards a partition of the unsharded landmark set, and every rank's poses bitwise equal
    (they solve every keyframe from the same all-reduced sums)."""
    def canon(q):
        q = np.array(q, np.float64)
        q[q[:, 3] < 0, :4] *= -1
        return q

    def rel(a, b):
        return float((np.abs(a - b) / np.maximum(np.abs(b), 1e-3)).max()) if a.size else 0.0

    ranks_agree = all(np.array_equal(s["pose"], shards[0]["pose"]) and np.array_equal(s["kf_idx"], ref["kf_idx"])
                      for s in shards)
    max_rel_pose = max(rel(canon(s["pose"]), canon(ref["pose"])) for s in shards)
    idx = np.concatenate([s["lm_idx"] for s in shards])
    pos = np.concatenate([s["lm_pos"] for s in shards]).reshape(-1, 3)
    order = np.argsort(idx, kind="stable")
    ref_order = np.argsort(ref["lm_idx"], kind="stable")
    partition = np.array_equal(idx[order], ref["lm_idx"][ref_order])
    max_rel_lm = rel(pos[order], ref["lm_pos"][ref_order]) if partition else float("inf")
    it_s = [s["iterations"] for s in shards]
    flips = sum(abs(a - b) for a, b in zip(shards[0]["obs"], ref["obs"])) + \
        sum(abs(len(s["obs"]) - len(ref["obs"])) for s in shards[:1])
    out = {"max_rel_pose": max_rel_pose, "max_rel_landmark": max_rel_lm, "gate_flips": int(flips),
           "iterations": [int(min(it_s)), int(max(it_s)), int(ref["iterations"])],
           "landmarks": int(len(ref["lm_idx"])), "shards_partition": bool(partition), "ranks_agree": bool(ranks_agree)}
    out["ok"] = bool(partition and ranks_agree and flips == 0 and len(set(it_s)) == 1 and it_s[0] == ref["iterations"]
                     and max_rel_pose <= tol and max_rel_lm <= tol)
    return out


def measured_candidates(vxslam, frame, params):
    """FAST candidates kept after runByImageBorder over all levels of `frame` (what k_fast writes and
    k_select reads, 16 B each): one extraction on a scratch context with the stage hooks on."""
    ctx = vxslam.Context(int(os.environ.get("LOCAL_RANK", "0")))
    try:
        ctx.set_debug(vxslam.DEBUG_STAGES)
        ctx.orb_extract(frame, params)
        return int(sum(len(ctx.debug_read(lv, 2)) for lv in range(params.n_levels)))
    finally:
        ctx.close()


def replay_equals_eager(a, b):
    """Two runs of one sharded plan (eager and graph replay) must agree bitwise."""
    return (a["iterations"] == b["iterations"] and a["obs"] == b["obs"] and np.array_equal(a["pose"], b["pose"])
            and np.array_equal(a["lm_idx"], b["lm_idx"]) and np.array_equal(a["lm_pos"], b["lm_pos"]))


def sharded_parity_gate(parity, dist, args):
    """N > 1: a sharded LocalBA that disagrees with the unsharded run makes the whole measurement
    invalid.  Rank 0's verdict is shared with every rank; on failure rank 0 prints a JSON line whose
    metric says INVALID (value null) and every rank exits with status 3."""
    ok = bool(parity and parity.get("ok"))
    ok = dist.broadcast_bytes(b"1" if ok else b"0") == b"1"
    if ok:
        return True
    if dist.rank == 0:
        print(json.dumps({"metric": "INVALID: sharded LocalBA differs from the unsharded run", "value": None,
                          "unit": "ms/frame", "n_gpus": dist.world, "steps": args.steps, "warmup": args.warmup,
                          "higher_is_better": False, "parity_vs_unsharded": parity}), flush=True)
    dist.close()
    raise SystemExit(3)


# ----------------------------------------------------------------------------- CPU baseline
def host_cpu():
    """The host CPU model and the cores this process may use (record the host)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return f"{model}; {usable} usable of {os.cpu_count()} logical CPUs"


def cpu_baseline(cfg, frames_host, ba_map, sample_frames):
    """The CPU restatement (oracle/, single thread, -O3 -march=x86-64-v3 -ffp-contract=off: SURVEY §8(d)'s
    optimised build, portable to any AVX2 host) on a bounded sample of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O

    O.build()
    h, w, nf, nk, nl = cfg
    opts = O.ba_options(window=nk)
    n = len(frames_host)
    prev = O.orb_extract(frames_host[n - 1], nf)[1]
    t_ext = t_match = t_setup = t_iter = 0.0
    for i in range(sample_frames):
        t0 = time.perf_counter()
        _, desc = O.orb_extract(frames_host[i % n], nf)
        t1 = time.perf_counter()
        O.match(prev, desc)
        t2 = time.perf_counter()
        O.ba_optimize(ba_map.copy(), opts)
        su, it = O.ba_last_timing()
        t_ext += t1 - t0
        t_match += t2 - t1
        t_setup += su
        t_iter += it
        prev = desc
    k = 1e3 / sample_frames
    # like for like with `value`: the GPU steps replay a resident LocalBA plan, so the CPU figure is
    # extract + match + the BA iterations (local_ba.cpp:110-248); the window / landmark-set
    # selection (:66-108) is reported apart, beside the GPU's plan build (ba_plan_build_ms)
    ms = k * (t_ext + t_match + t_iter)
    return {
        "value": round(ms, 3),
        "unit": "ms/frame",
        "cores": 1,
        "kind": "port",
        "host": host_cpu(),
        "sample": f"{sample_frames} frames of the same workload (extract {k * t_ext:.2f} + match {k * t_match:.2f} + "
                  f"BA iterations {k * t_iter:.2f} ms/frame; excluded: BA window/landmark-set selection "
                  f"{k * t_setup:.2f} ms, compare ba_plan_build_ms), oracle/ C++ restatement, 1 thread",
        "ba_setup_ms": round(k * t_setup, 3),
        "ba_iterations_ms": round(k * t_iter, 3),
    }


def cpu_baseline_mt(cfg, frames_host, ba_map, n_frames):
    """Best-effort CPU: the same restatement, frames in parallel on every host core
    this process may use (threads; the oracle's C calls release the GIL).  Frame i is extract(i) +
    match(desc(i - 1), desc(i)) + LocalBA, as in the single-thread leg; the previous frame's
    descriptors are computed before the timed region so the frames are independent.  ms/frame =
    wall time x the busy share outside the BA window selection (excluded as in the 1-thread
    figure) / frames."""
    import threading

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O

    h, w, nf, nk, nl = cfg
    opts = O.ba_options(window=nk)
    n = len(frames_host)
    descs = [O.orb_extract(f, nf)[1] for f in frames_host]
    pat = O.load_pattern()
    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cores = max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", cores))))
    n_frames = max(n_frames, 2 * cores)
    busy = [[0.0, 0.0] for _ in range(cores)]  # per thread: seconds outside / inside the BA setup

    def work(tid):
        for i in range(tid, n_frames, cores):
            t0 = time.perf_counter()
            _, desc = O.orb_extract(frames_host[i % n], nf, pattern=pat)
            O.match(descs[(i - 1) % n], desc)
            O.ba_optimize(ba_map.copy(), opts)
            su, _ = O.ba_last_timing()
            busy[tid][0] += time.perf_counter() - t0 - su
            busy[tid][1] += su

    th = [threading.Thread(target=work, args=(t,)) for t in range(cores)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = time.perf_counter() - t0
    b_run, b_setup = sum(x[0] for x in busy), sum(x[1] for x in busy)
    ms = 1e3 * wall * b_run / max(b_run + b_setup, 1e-12) / n_frames
    return {"value": round(ms, 3), "unit": "ms/frame", "cores": cores, "kind": "port",
            "sample": f"{n_frames} frames on {cores} threads (frames in parallel), wall {wall:.2f} s x "
                      f"non-setup share {b_run / max(b_run + b_setup, 1e-12):.3f}; oracle/ C++ restatement"}


# ----------------------------------------------------------------------------- host placement
def idlest_cpus(n, window_s=0.3):
    """The n logical CPUs of this process's affinity set with the least busy time over window_s
    (/proc/stat deltas), or None where that is not readable."""
    def snap():
        d = {}
        with open("/proc/stat") as f:
            for line in f:
                if line.startswith("cpu") and line[3].isdigit():
                    v = [int(x) for x in line.split()[1:]]
                    d[int(line.split()[0][3:])] = (sum(v), v[3] + v[4])  # (total, idle + iowait)
        return d
    try:
        allowed = os.sched_getaffinity(0)
        a = snap()
        time.sleep(window_s)
        b = snap()
    except (OSError, AttributeError, ValueError):
        return None
    busy = {c: 1.0 - (b[c][1] - a[c][1]) / max(1, b[c][0] - a[c][0]) for c in b if c in a and c in allowed}
    if len(busy) <= n:
        return None
    return sorted(sorted(busy, key=lambda c: busy[c])[:n])


# ----------------------------------------------------------------------------- config C5
def sba_shard_result(m_after, lm_ids, rank, N, st, vxslam):
    """What a rank's sharded Schur BA run left in its copy of the map (vx_sba_plan_fetch): every window
    pose (all ranks solve all of them) and the positions of the landmarks of its shard."""
    own = np.nonzero(np.array([vxslam.ba_shard_of(int(i), N) == rank for i in lm_ids]))[0] if N > 1 else \
        np.arange(len(lm_ids))
    return {"pose": np.asarray(m_after["kf_pose"]).reshape(-1, 7).copy(), "lm_idx": own.astype(np.int64),
            "lm_pos": np.asarray(m_after["lm_pos"]).reshape(-1, 3)[own].copy(),
            "iterations": int(st.iterations), "accepted": int(st.accepted),
            "steps": [int(x) for x in list(st.step)[:int(st.iterations)]],
            "cost": [float(x) for x in list(st.cost)[:int(st.iterations)]]}


def sba_parity_vs_unsharded(shards, ref, tol=1e-4):
    """The sharded Schur BA (one sba_shard_result per rank) against the unsharded run of the same
    window: the same LM decisions (iterations, accepted, per-iteration step codes), costs to 1e-9, every
    rank's poses bitwise equal (they solve from the same all-reduced system), poses and the landmark
    shards' positions within tol relative (quaternion sign canonicalised), the shards a partition."""
    def canon(q):
        q = np.array(q, np.float64)
        q[q[:, 3] < 0, :4] *= -1
        return q

    def rel(a, b):
        return float((np.abs(a - b) / np.maximum(np.abs(b), 1e-3)).max()) if a.size else 0.0

    idx = np.concatenate([s["lm_idx"] for s in shards])
    partition = np.array_equal(np.sort(idx), ref["lm_idx"])
    pos = np.concatenate([s["lm_pos"] for s in shards])
    max_rel_lm = rel(pos[np.argsort(idx, kind="stable")], ref["lm_pos"]) if partition else float("inf")
    ranks_agree = all(np.array_equal(s["pose"], shards[0]["pose"]) for s in shards)
    max_rel_pose = max(rel(canon(s["pose"]), canon(ref["pose"])) for s in shards)
    same_lm = all((s["iterations"], s["accepted"], s["steps"]) == (ref["iterations"], ref["accepted"], ref["steps"])
                  for s in shards)
    cost_rel = max((abs(a - b) / max(abs(b), 1e-30) for s in shards for a, b in zip(s["cost"], ref["cost"])),
                   default=0.0)
    out = {"max_rel_pose": max_rel_pose, "max_rel_landmark": max_rel_lm, "max_rel_cost": cost_rel,
           "iterations": int(ref["iterations"]), "accepted": int(ref["accepted"]), "same_lm_decisions": bool(same_lm),
           "shards_partition": bool(partition), "ranks_agree": bool(ranks_agree)}
    out["ok"] = bool(partition and ranks_agree and same_lm and cost_rel <= 1e-9 and max_rel_pose <= tol
                     and max_rel_lm <= tol)
    return out


def cpu_baseline_c5(frames_host, ba_map, opts_cpu, nf, rig_steps):
    """The CPU restatement (oracle/, one thread) on a bounded sample of C5: per rig step the 8 cameras'
    extract + match against the camera's previous frame and one Schur BA of the global window."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O

    O.build()
    n = len(frames_host)
    prev = [O.orb_extract(frames_host[(n - C5_CAMERAS + c) % n], nf)[1] for c in range(C5_CAMERAS)]
    t_fe = t_ba = 0.0
    for t in range(rig_steps):
        t0 = time.perf_counter()
        for c in range(C5_CAMERAS):
            _, d = O.orb_extract(frames_host[(t * C5_CAMERAS + c) % n], nf)
            O.match(prev[c], d)
            prev[c] = d
        t1 = time.perf_counter()
        O.sba_optimize(ba_map.copy(), opts_cpu)
        t_ba += time.perf_counter() - t1
        t_fe += t1 - t0
    per_frame = 1e3 * (t_fe + t_ba) / (rig_steps * C5_CAMERAS)
    return {"value": round(per_frame, 3), "unit": "ms/frame", "cores": 1, "kind": "port", "host": host_cpu(),
            "sample": f"{rig_steps} rig steps of C5 ({rig_steps * C5_CAMERAS} camera frames: extract + match "
                      f"{1e3 * t_fe / rig_steps:.1f} ms and Schur BA {1e3 * t_ba / rig_steps:.1f} ms per rig step), "
                      "oracle/ C++ restatement (sba_oracle.cpp: the same Schur system, dense Cholesky), 1 thread"}


def bench_c5(args):
    """BASELINE configs[4]: 8 camera streams of 640x480 BGR8 (2000 ORB each) on one rig, one global
    window of 200 KF / 100k landmarks solved by the Schur-complement joint BA with the MFMA dense pose
    solve (vx_sba_*).  The cameras are split over the N ranks (8 / N each); a
    rig step is: batched extraction of the rank's cameras (one launch per kernel), batched matching
    of each against its previous frame, then the Schur BA of the step, landmark-sharded over the
    ranks with one RCCL all-reduce of the reduced pose system per LM iteration (sba.hip).  Frontend
    and BA run on two contexts; BA(t) waits for Match(t), so the frontend of step t + 1 overlaps
    BA(t).  One bench step = one rig step; value = elapsed / camera frames (ms/frame)."""
    full_affinity, host_cpus = None, None
    if args.pin_host == "auto" and args.gpus == 1 and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        host_cpus = idlest_cpus(8)
        if host_cpus:
            full_affinity = os.sched_getaffinity(0)
            os.sched_setaffinity(0, host_cpus)
    dist = Dist(args.gpus)
    import torch

    import vxslam
    from vxslam import synth

    torch.cuda.set_device(dist.local_rank)
    N, rank = dist.world, dist.rank
    if C5_CAMERAS % N:
        raise SystemExit(f"C5: {C5_CAMERAS} cameras do not split over {N} ranks")
    cams = C5_CAMERAS // N
    h, w, nf, nk, nl = CONFIGS["C5"]
    front, back = vxslam.Context(dist.local_rank), vxslam.Context(dist.local_rank)
    params = vxslam.default_orb_params(n_features=nf)
    T = 4  # time steps cycled
    # camera c of the rig at time step t: frame t * 8 + c of the rig's sequence; this rank's cameras
    # are rank * cams .. rank * cams + cams - 1
    rig_host = synth.make_frames(0xC5, T * C5_CAMERAS, h, w)
    mine = [t * C5_CAMERAS + rank * cams + c for t in range(T) for c in range(cams)]
    pool = torch.from_numpy(np.ascontiguousarray(rig_host[mine])).cuda()
    m = synth.make_ba_map(0x5EED00C5, nk, nl, n_streams=C5_CAMERAS, n_old_kf=2 * C5_CAMERAS,
                          cross_frac=args.c5_cross)
    opts = vxslam.default_sba_options(window=nk, iters=args.c5_iters)
    rccl = None
    if N > 1:
        uid = dist.broadcast_bytes(vxslam.Context.comm_unique_id() if rank == 0 else None)
        back.comm_init(uid, N, rank)
        nr, rk = back.comm_info()
        infos = dist.gather((nr, rk))
        rccl = {"nranks": nr, "world_size": N, "ranks": [list(x) for x in infos] if infos else None}
        if nr != N or rk != rank:
            raise SystemExit(f"rank {rank}: RCCL communicator reports {nr} ranks / rank {rk}")
    plan = back.sba_plan(m, opts, shard_rank=rank, shard_count=N)
    info = plan.info()
    work = plan.factor_work()
    parity = None
    if N > 1:  # the sharded run against the unsharded one, before anything is timed
        mine_r = []
        for r in range(2):
            ms = m.copy()
            plan.run_async()
            st_s = plan.fetch(ms)
            mine_r.append(sba_shard_result(ms, m["lm_id"], rank, N, st_s, vxslam))
        shards = dist.gather(mine_r)
        if rank == 0:
            mu = m.copy()
            pu = back.sba_plan(mu, opts)
            pu.run_async()
            st_u = pu.fetch(mu)
            pu.close()
            ref = sba_shard_result(mu, m["lm_id"], 0, 1, st_u, vxslam)
            parity = sba_parity_vs_unsharded([s[1] for s in shards], ref)
            parity["first_run"] = sba_parity_vs_unsharded([s[0] for s in shards], ref)["ok"]
            parity["ok"] = bool(parity["ok"] and parity["first_run"])
            log(f"[bench C5] sharded vs unsharded Schur BA: {parity}")
        sharded_parity_gate(parity, dist, args)
    ev = front.event()

    def extract(t):
        bank, base = t % 2, (t % T) * cams
        front.orb_extract_batch_async(pool[base].data_ptr(), cams, pool.stride(0), w, h, 3, pool.stride(1), bank,
                                      params)

    def step(t):
        bank = t % 2
        extract(t)
        front.match_batch_async([(front.batch_device(1 - bank, c), front.batch_device(bank, c)) for c in range(cams)])
        front.record(ev)
        back.wait_event(ev)
        plan.run_async()

    def sync():
        front.synchronize()
        back.synchronize()

    extract(-1)  # (bank 1: step 0's previous frames)
    for t in range(6):  # pre-warm: graphs captured, plan buffers touched
        step(t)
    sync()
    stages = {}
    if not args.no_profile:
        for c in (front, back):
            c.prof_enable(True)
        nw = max(args.warmup, 3)
        for t in range(nw):
            step(t)
        sync()
        prof = {}
        for c in (front, back):
            for k, v in c.prof_read(reset=True).items():
                if v[1]:
                    a, n = prof.get(k, (0.0, 0))
                    prof[k] = (a + v[0], n + v[1])
            c.prof_enable(False)
        stages = {k: (v[0] / max(v[1], 1), v[1] / nw) for k, v in prof.items() if v[1]}
    elapsed = timed_loop(step, args.steps, args.warmup, sync, dist)
    st = plan.fetch(None)
    lat = []
    for t in range(5):
        sync()
        t0 = time.perf_counter()
        step(args.steps + args.warmup + t)
        sync()
        lat.append(time.perf_counter() - t0)
    frames_total = args.steps * C5_CAMERAS
    value = 1e3 * elapsed / frames_total
    # roofline of the dominant stage: the dense pose solve on MFMA (FP64 flops of the symbolic tile
    # factorisation, vx_sba_plan_factor_work) or the Schur reduction (bytes of its W / Y gathers)
    roofline = None
    if stages:
        dominant = max(stages, key=lambda k: stages[k][0] * stages[k][1])
        ms_step = stages[dominant][0] * stages[dominant][1]
        its = int(st.iterations)
        steps_c = [int(x) for x in list(st.step)[:its]]
        # factorisations per run: every iteration before the last that is not a rejection (the LM
        # loop re-assembles without solving after a rejected step, sba_oracle.cpp)
        n_fac = sum(1 for i in range(max(its - 1, 0)) if steps_c[i] != 0)
        if dominant == "sba_solve" and n_fac:
            tfs = work["flops"] * n_fac / (ms_step * 1e-3) / 1e12
            roofline = {"kernel": "sba_solve", "hip_kernel": "k_sba_fac_blk (k_sba_fac_step, k_sba_solve) + k_sba_backsub",
                        "bound": "mfma", "achieved": round(tfs, 4), "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
                        "frac": round(tfs / FP64_PEAK_TFS, 6), "traffic": None,
                        "flops_per_factorisation": int(work["flops"]), "factorisations_per_step": n_fac,
                        "solve_ms_per_step": round(ms_step, 4), "factor_tiles": work,
                        "note": "v_mfma_f64_16x16x4 tiles; the factor is a chain of dependent tile steps "
                                "(latency-bound, DESIGN.md §18)"}
        else:
            roofline = {"kernel": dominant, "bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": None, "traffic": None, "stage_ms_per_step": round(ms_step, 4)}
    cpu = None
    if full_affinity:
        os.sched_setaffinity(0, full_affinity)
    if rank == 0 and N == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle as O

        oc = O.sba_options(window=nk, iters=args.c5_iters)
        cpu = cpu_baseline_c5(rig_host, m, oc, nf, max(2, args.cpu_sample // 10))
    if rank == 0:
        for k, (ms, n) in sorted(stages.items(), key=lambda kv: -kv[1][0] * kv[1][1]):
            log(f"[bench C5] stage {k:18s} {ms * 1e3:9.2f} us/launch x {n:6.2f} launches/step")
        out = {
            "metric": "ms/frame (feature-extract+match + BA solve), C5 rig: 8 x 640×480 cameras, 200 KF / 100k pts, "
                      "Schur + MFMA dense pose solve",
            "value": round(value, 4), "unit": "ms/frame", "n_gpus": N, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 4), "higher_is_better": False, "scaling": "strong",
            "vs_baseline": None, "dtype": "u8/i32 (FAST, pyramid, BRIEF), f32 (Harris, blur, angle), f64 (BA)",
            "data": "synthetic",
            "config": {"workload": (f"C5: per step one rig step — {C5_CAMERAS} cameras x {w}x{h} BGR8 "
                                    f"({cams} per rank: batched extract of {nf} ORB + batched kNN-2 match vs the "
                                    f"camera's previous frame), then ONE Schur-complement BA (<= {args.c5_iters} LM "
                                    f"iterations) of the global {nk} KF / {nl} landmark window "
                                    f"({info['n_comp']} covisibility component(s), cross_frac {args.c5_cross}), "
                                    f"landmark-sharded over {N} GPU(s)" +
                                    (" with one RCCL all-reduce of the reduced pose system per iteration" if N > 1
                                     else "")),
                       "frames_per_step": C5_CAMERAS, "parallelism": f"cameras x{N} ranks; Schur BA: landmark shards x{N}",
                       "ba_window_kf": nk, "ba_landmarks": nl, "orb_features": nf, "plan": info,
                       "scaling": "strong"},
            "ms_per_rig_step": round(1e3 * elapsed / args.steps, 4),
            "latency_ms_per_rig_step": round(1e3 * float(np.median(lat)), 4),
            "host_cpus": host_cpus, "parity_vs_unsharded": parity, "rccl": rccl,
            "work_per_step": {"sba_iterations": int(st.iterations), "sba_accepted": int(st.accepted),
                              "sba_initial_cost": float(st.initial_cost), "sba_final_cost": float(st.final_cost)},
            "roofline": roofline, "cpu_baseline": cpu,
            "stages_us": {k: round(v[0] * 1e3, 2) for k, v in stages.items()},
        }
        print(json.dumps(out), flush=True)
    plan.close()
    ev.close()
    back.close()
    front.close()
    dist.close()


# ----------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", default="C3",
                    help="workload C2 / C3 / C4 / C5, or a key=value file with the reference's flag names "
                         "(apps/main.cpp --config; its ba_* keys set the LocalBA options below)")
    ap.add_argument("--scaling", default="weak", choices=("weak", "strong"),
                    help="N > 1: weak = per-rank work fixed (each rank its own camera stream, one global "
                         "window of N x the config's keyframes / landmarks); strong = total work fixed (the "
                         "config's window as BASELINE states it, landmark-sharded over the N ranks, the "
                         "step's frames split over the ranks)")
    ap.add_argument("--c5-cross", type=float, default=0.03,
                    help="C5: share of landmarks seen by two neighbouring cameras of the rig (0.03: the 8 "
                         "streams form ONE covisibility component, a 1188 x 1188 dense pose system; 0: 8 "
                         "independent components)")
    ap.add_argument("--c5-iters", type=int, default=8, help="C5: Schur BA Levenberg-Marquardt iterations")
    # the reference runner's LocalBA flags (apps/main.cpp:42-47, config/default.cfg), same names;
    # unset: the workload's values (window = the config's keyframes, the reference defaults otherwise)
    for k, typ in BA_FLAGS.items():
        ap.add_argument(f"--{k}", type=typ, default=None)
    ap.add_argument("--frames", type=int, default=8, help="distinct frames cycled through")
    ap.add_argument("--cpu-sample", type=int, default=30, help="frames timed for the CPU baseline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-drop-in", action="store_true",
                    help="skip the per-keyframe drop-in timings (PMC tool runs: the C++ adapter subprocess)")
    ap.add_argument("--no-profile", action="store_true", help="skip the HIP-event roofline pass")
    ap.add_argument("--ba-cus", type=float, default=0.0,
                    help="fraction of the CUs reserved for the LocalBA context (disjoint CU masks; 0: shared)")
    ap.add_argument("--diag-skip", default="", choices=("", "ba", "match", "extract"),
                    help="diagnostics only (the JSON line is marked invalid): leave one stage out of every step")
    ap.add_argument("--diag-nodep", action="store_true",
                    help="diagnostics only (the JSON line is marked invalid): LocalBA(t) does not wait for Match(t)")
    ap.add_argument("--ba-peer", action="store_true",
                    help="N > 1: the sharded LocalBA's row sums by the one-shot peer reduction over xGMI "
                         "($VX_BA_PEER=1: IPC-mapped blocks and generation flags, DESIGN.md §6) instead of one "
                         "ncclAllReduce per iteration; verified on one GPU by emulation only")
    ap.add_argument("--ba-priority", type=int, default=0, choices=(0, 1),
                    help="stream priority of the LocalBA context (1: the device's greatest)")
    ap.add_argument("--grid-share", type=float, default=None,
                    help="share of the CUs the extraction context's one-round grids are sized for "
                         "(vx_set_grid_share; default 1/4 with more than one stream, 1 otherwise: DESIGN.md §7)")
    ap.add_argument("--streams", type=int, default=3, choices=(1, 2, 3),
                    help="1: everything on one stream; 2: Extract+Match | LocalBA; 3: Extract | Match | LocalBA")
    ap.add_argument("--extract-ctx", type=int, default=3, choices=(1, 2, 3, 4),
                    help="extraction contexts (with --streams 3): frames alternate between them, so the "
                         "extraction of frame t+1 overlaps frame t's; Match and LocalBA stay in frame order")
    ap.add_argument("--frames-per-step", type=int, default=0,
                    help="frames per timed step (default: eight times the extraction contexts with --streams 3, "
                         "i.e. eight rounds of the pipeline, else 1); every frame runs Extract, Match and LocalBA")
    ap.add_argument("--seq-threads", type=int, default=1,
                    help="> 1: each context's recorded calls replayed on a host thread of its own (vx_seq_set_threads)")
    ap.add_argument("--no-seq", action="store_true",
                    help="timed steps through per-frame binding calls instead of one recorded vx_seq per step")
    ap.add_argument("--pin-host", default="auto", choices=("auto", "off"),
                    help="auto (one process): run on the 8 least-busy host CPUs, chosen before the GPU is "
                         "initialised (the enqueueing thread and the HIP runtime's threads inherit them); the "
                         "CPU baseline legs run on the whole affinity set again (DESIGN.md §17)")
    ap.add_argument("--match-ctx", default="extract", choices=("extract", "own"),
                    help="with --streams 3: Match(t) on frame t's extraction context right after Extract(t) "
                         "(default: one hardware queue fewer; measured 0.073 vs 0.073-0.076 ms/frame, steadier) "
                         "or on a context of its own")
    args = ap.parse_args()
    if args.ba_peer:
        os.environ["VX_BA_PEER"] = "1"
    args.config_file = None
    if args.config == "C5":
        return bench_c5(args)
    if args.config not in CONFIGS:
        if not os.path.isfile(args.config):
            ap.error(f"--config: neither a workload ({', '.join(sorted(CONFIGS))}) nor a file: {args.config}")
        args.config_file, args.config = args.config, "C3"

    # host placement (on a shared GPU host, unpinned runs fell into a mode where every
    # HIP call cost 2-5x more; pinned to idle CPUs they did not)
    full_affinity, host_cpus = None, None
    if args.pin_host == "auto" and args.gpus == 1 and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        host_cpus = idlest_cpus(8)
        if host_cpus:
            full_affinity = os.sched_getaffinity(0)
            os.sched_setaffinity(0, host_cpus)
    dist = Dist(args.gpus)
    import torch

    import vxslam
    from vxslam import synth

    torch.cuda.set_device(dist.local_rank)
    # one context (HIP stream) per pipeline stage; see Pipeline.  --ba-cus > 0 gives LocalBA its own
    # compute units (a contiguous range of CU-mask bits: the same number on every XCD) and extraction /
    # matching the rest
    fe_mask = ba_mask = None
    if args.ba_cus > 0 and args.streams > 1:
        # the smaller side gets the first round(share x CUs) CU-mask bits, the other side the rest:
        # bit i lies on XCD i mod 8 (scripts/probe/xcd_probe.hip), so a contiguous range is spread
        # evenly over the XCDs — a mask that leaves an XCD without CUs (e.g. every 8th bit) is not
        # applied at all by the runtime
        ncu = vxslam.lib().vx_device_cus(dist.local_rank)
        small = min(args.ba_cus, 1.0 - args.ba_cus)
        n_few = max(8, int(round(small * ncu / 8)) * 8)
        few = list(range(n_few))
        rest = [i for i in range(ncu) if i not in set(few)]
        ba_mask, fe_mask = (few, rest) if args.ba_cus <= 0.5 else (rest, few)
    n_ex = args.extract_ctx if args.streams == 3 else 1
    ectxs = [vxslam.Context(dist.local_rank, cu_mask=fe_mask) for _ in range(n_ex)]
    ectx = ectxs[0]
    mon = args.match_ctx == "extract" and args.streams == 3  # Match(t) on frame t's extraction context
    mctx = ectx if args.streams < 3 or mon else vxslam.Context(dist.local_rank, cu_mask=fe_mask)
    bctx = ectx if args.streams < 2 else vxslam.Context(dist.local_rank, priority=args.ba_priority, cu_mask=ba_mask)
    ctxs = list({id(c): c for c in ectxs + [mctx, bctx]}.values())
    # extraction runs beside the previous frame's LocalBA: its pyramid grid leaves CUs free for it
    # (1/4: 6 alternating runs each late in round 2, median 0.0684 against 0.0696 ms/frame at 1/3)
    grid_share = args.grid_share if args.grid_share else (0.25 if args.streams > 1 else 1.0)
    for c in ectxs:
        c.set_grid_share(grid_share)
    cfg = CONFIGS[args.config]
    h, w, nf, nk, nl = cfg
    N = dist.world
    # weak: the window grows with N (every rank adds its camera stream's keyframes and landmarks);
    # strong: the config's window, its landmarks sharded over the N ranks
    NW = N if args.scaling == "weak" else 1

    # ---- inputs resident in HBM before timing
    frames_host = synth.make_frames(0x5EED0000 + 31 * dist.rank + 3, args.frames, h, w)
    frames_dev = torch.from_numpy(frames_host).cuda()
    params = vxslam.default_orb_params(n_features=nf)
    ba_map = synth.make_ba_map(0x5EED0003, nk * NW, nl * NW, n_streams=NW, n_old_kf=2 * NW)
    ba_flags = resolve_ba_flags(args, nk * NW)
    opts = vxslam.default_ba_options(window=ba_flags["ba_window_size"], iters=ba_flags["ba_iterations"],
                                     min_pose=ba_flags["ba_min_pose_observations"],
                                     min_point=ba_flags["ba_min_point_observations"],
                                     huber=ba_flags["ba_huber_delta"], max_err=ba_flags["ba_max_reproj_error"])
    rccl = None
    if N > 1:
        uid = dist.broadcast_bytes(vxslam.Context.comm_unique_id() if dist.rank == 0 else None)
        bctx.comm_init(uid, N, dist.rank)
        # what RCCL itself reports must be this launch's world (a communicator of the wrong size would
        # all-reduce a different set of shards)
        nr, rk = bctx.comm_info()
        infos = dist.gather((nr, rk))
        rccl = {"nranks": nr, "world_size": N, "ranks": [list(x) for x in infos] if infos else None}
        if nr != N or rk != dist.rank:
            raise SystemExit(f"rank {dist.rank}: RCCL communicator reports {nr} ranks / rank {rk}, "
                             f"WORLD_SIZE {N} / RANK {dist.rank}")
    plan = bctx.ba_plan(ba_map, opts, shard_rank=dist.rank, shard_count=N)
    info = plan.info()
    # N > 1: the sharded run checked against the unsharded run of the same global window (rank 0
    # runs it on its own GPU) before anything is timed
    parity = None
    if N > 1:
        # runs 1, 2, 3 of the sharded plan: eager, graph capture, graph replay (include/vx_slam.h);
        # every timed run replays the captured graph, so the replay is checked as well as the eager run
        insp = vxslam.ba_plan_inspect(ba_map, opts, shard_rank=dist.rank, shard_count=N)
        mine = []
        for r in range(3):
            m_s = ba_map.copy()
            plan.run_async()
            st_s = plan.fetch(m_s)
            if r in (0, 2):
                mine.append(shard_result(m_s, insp, st_s))
        shards = dist.gather(mine)
        if dist.rank == 0:
            m_u = ba_map.copy()
            pu = bctx.ba_plan(m_u, opts)
            pu.run_async()
            st_u = pu.fetch(m_u)
            pu.close()
            ref = shard_result(m_u, vxslam.ba_plan_inspect(ba_map, opts), st_u)
            parity = parity_vs_unsharded([s[1] for s in shards], ref)
            parity["eager"] = parity_vs_unsharded([s[0] for s in shards], ref)["ok"]
            parity["replay_equals_eager"] = all(replay_equals_eager(s[0], s[1]) for s in shards)
            parity["ok"] = bool(parity["ok"] and parity["eager"] and parity["replay_equals_eager"])
            log(f"[bench] sharded vs unsharded LocalBA: {parity}")
        sharded_parity_gate(parity, dist, args)
    # what a drop-in LocalBA::Optimize() adds per call on top of the solve: the window / CSR
    # build from the map snapshot (device build), reported beside `value`
    plan_ms = []
    for _ in range(5):
        t0 = time.perf_counter()
        bctx.ba_plan(ba_map, opts, shard_rank=dist.rank, shard_count=N).close()
        plan_ms.append(1e3 * (time.perf_counter() - t0))
    plan_build_ms = float(np.median(plan_ms))
    per_kf = None
    if N == 1 and not args.no_drop_in:
        # (the C++ drop-in's subprocess inherits this process's CPUs: the whole affinity set, not the 8
        # idlest CPUs the pipeline runs on — its host pool binds itself to one L3 slice of those)
        pinned = os.sched_getaffinity(0)
        if full_affinity:
            os.sched_setaffinity(0, full_affinity)
        try:
            per_kf = per_keyframe_ms(bctx, ba_map, opts, dist, N, vxslam)
        finally:
            if full_affinity:
                os.sched_setaffinity(0, pinned)
    torch.cuda.synchronize()

    # Pipeline.  Frame t: Extract(t) on extraction context t % E (E = --extract-ctx) into that
    # context's slot (t // E) % 3, Match(t - 1, t) on mctx, LocalBA(t) on bctx, ordered on the device
    # by events: Match(t) after Extract(t), LocalBA(t) after Match(t) (so Match and LocalBA run in
    # frame order), and Extract(t) after Match(t - 3E + 1) (the last reader of the slot it
    # overwrites).  Nothing of frame t + 1 depends on Match(t) or LocalBA(t), so consecutive frames'
    # stages overlap, and with E = 2 so do two frames' extractions (frames are independent there);
    # with --streams 1 the same calls run back to back on one stream.
    E = n_ex
    ev_e = [c.event() for c in ectxs]
    ev_m = [mctx.event() for _ in range(4 * E)]

    def loc(i):  # (extraction context, slot) of frame i
        return i % E, (i // E) % 3

    def extract(i):
        f = frames_dev[i % args.frames]
        ci, si = loc(i)
        ectxs[ci].orb_extract_async(f.data_ptr(), w, h, 3, w * 3, si, params)

    for i in range(-3 * E, 0):  # fill every slot (frame -1 is step 0's previous frame)
        extract(i)
    slot = {(ci, si): ectxs[ci].slot_device(si) for ci in range(E) for si in range(3)}

    skip = args.diag_skip
    if skip == "ba":
        plan.run_async()  # (so the statistics fetched at the end exist)
    if skip == "match":  # (so the matches fetched at the end exist)
        for mc in (ectxs if mon else [mctx]):
            mc.match_device_async(slot[loc(-2)], slot[loc(-1)])

    def step(i):
        ci, si = loc(i)
        ex = ectxs[ci]
        ex.wait_event(ev_m[(i - 3 * E + 1) % (4 * E)])  # (an event not yet recorded is an immediate no-op)
        if skip != "extract":
            extract(i)
        ex.record(ev_e[ci])
        mx = ex if mon else mctx
        if mon and E > 1:
            mx.wait_event(ev_e[(i - 1) % E])  # Match(t) also reads frame t - 1, extracted on the other context
        elif not mon:
            mx.wait_event(ev_e[ci])
        if skip != "match":
            mx.match_device_async(slot[loc(i - 1)], slot[loc(i)])
        mx.record(ev_m[i % (4 * E)])
        if not args.diag_nodep:
            bctx.wait_event(ev_m[i % (4 * E)])
        if skip != "ba":
            for _ in range(BA_PER_FRAME):
                plan.run_async()

    # Host fast path of step(): the same C-ABI calls in the same order through pre-bound ctypes
    # functions, every argument object built once.  Through the wrappers the per-frame host enqueue
    # (~60 us) was within 15 % of the GPU's frame time, and a slower host turned whole runs
    # host-bound (r03: 0.089 against 0.068 ms/frame, host enqueue 0.52 against 0.36 ms per step).
    if not skip and not args.diag_nodep:
        import ctypes as C
        L = vxslam.lib()
        f_wait, f_rec = L.vx_event_wait, L.vx_event_record
        f_ext, f_match, f_run = L.vx_orb_extract_async, L.vx_match_device_async, L.vx_ba_plan_run_async
        p_params = C.byref(params)
        fptr = [C.c_void_p(frames_dev[k].data_ptr()) for k in range(args.frames)]
        n_frames, stride = args.frames, C.c_int64(w * 3)
        eh, mh, bh, ph = [c.handle for c in ectxs], mctx.handle, bctx.handle, plan._h
        evE, evM = [e._h for e in ev_e], [e._h for e in ev_m]
        sl = {k: (C.c_void_p(d), C.c_void_p(n), cap) for k, (d, n, cap) in slot.items()}
        ratio = C.c_float(0.8)

        def step(i):  # noqa: F811 (replaces the wrapper-based step above)
            ci, si = i % E, (i // E) % 3
            x = eh[ci]
            rc = f_wait(x, evM[(i - 3 * E + 1) % (4 * E)])
            rc |= f_ext(x, p_params, fptr[i % n_frames], w, h, 3, stride, si)
            rc |= f_rec(x, evE[ci])
            m = x if mon else mh
            if mon and E > 1:
                rc |= f_wait(m, evE[(i - 1) % E])
            elif not mon:
                rc |= f_wait(m, evE[ci])
            q, t = sl[((i - 1) % E, ((i - 1) // E) % 3)], sl[(ci, si)]
            rc |= f_match(m, q[0], q[1], q[2], t[0], t[1], t[2], ratio)
            rc |= f_rec(m, evM[i % (4 * E)])
            rc |= f_wait(bh, evM[i % (4 * E)])
            for _ in range(BA_PER_FRAME):
                rc |= f_run(bh, ph)
            if rc:
                raise RuntimeError(f"frame {i}: a C-ABI call failed ({rc}): "
                                   f"{L.vx_last_error(x).decode()} {L.vx_last_error(bh).decode()}")

    def sync():
        for c in ctxs:
            c.synchronize()

    # One timed step = F frames, eight rounds of the pipeline (F = 8 E by default): each of them runs
    # Extract, Match and LocalBA.  With one frame per step the pipeline's fill (one frame's whole
    # latency, ~0.19 ms at C3) weighed ~10 % in the driver's 20-step run; measured 20-step / 2000-step:
    # 1.5-4.6 % with 12 frames, 1-6 % with 6, box noise ~2 % (scripts/jobs/gpu_r03_short_vs_long.sh); 24
    # frames against 12, alternating: 20-step runs 0.0688-0.0699 against 0.0694-0.0711 ms/frame,
    # 2000-step runs the same (scripts/gpu_fps_ab.sh, profiles/r04/host/fps_ab.txt)
    F = args.frames_per_step if args.frames_per_step > 0 else (8 * E if args.streams == 3 else 1)
    # strong scaling: the step's F frames are split over the ranks (F / N each), and every frame's
    # LocalBA is one joint run of all ranks (each over its landmark shard), so a rank runs the
    # sharded window N times per local frame: per step F extractions / matches in all and F
    # LocalBA runs, whatever N
    BA_PER_FRAME = N if args.scaling == "strong" else 1
    if args.scaling == "strong":
        if F % N:
            raise SystemExit(f"--scaling strong: {F} frames per step do not split over {N} ranks")
        F //= N

    def fstep(i):
        for f in range(F):
            step(i * F + f)

    # The timed steps through recorded sequences (vx_seq): the calls of step() above for F frames,
    # recorded once per phase of the pipeline's period (frame buffers, slots and events repeat every
    # lcm(frames, 3E, 4E) frames) and replayed from C — one binding call per step instead of ~8 per
    # frame.  --no-seq keeps the per-frame calls.
    host_path = "per-frame ctypes calls"
    seqs = []
    if not skip and not args.diag_nodep and not args.no_seq:
        period = int(np.lcm.reduce([args.frames, 3 * E, 4 * E]))
        n_seq = int(np.lcm(period, F)) // F
        for k in range(n_seq):
            sq = vxslam.Seq()
            for f in range(F):
                i = k * F + f
                ci, si = loc(i)
                x = ectxs[ci]
                sq.wait(x, ev_m[(i - 3 * E + 1) % (4 * E)])
                sq.extract(x, params, frames_dev[i % args.frames].data_ptr(), w, h, 3, w * 3, si, owner=frames_dev)
                sq.record(x, ev_e[ci])
                mx = x if mon else mctx
                if mon and E > 1:
                    sq.wait(mx, ev_e[(i - 1) % E])
                elif not mon:
                    sq.wait(mx, ev_e[ci])
                sq.match(mx, slot[loc(i - 1)], slot[loc(i)], 0.8)
                sq.record(mx, ev_m[i % (4 * E)])
                sq.wait(bctx, ev_m[i % (4 * E)])
                for _ in range(BA_PER_FRAME):
                    sq.ba_run(bctx, plan)
            if args.seq_threads > 1:
                sq.set_threads(args.seq_threads)
            seqs.append(sq)
        host_path = (f"vx_seq: one C call per step ({n_seq} recorded phases of {F} frames, {len(seqs[0])} calls each"
                     + (", one host thread per context)" if args.seq_threads > 1 else ")"))

        def fstep(i):  # noqa: F811
            seqs[i % n_seq].run()

    # ---- fixed internal pre-warm, outside the reported warm-up: every launch sequence a step can
    # take is keyed by (context, slot, frame buffer) — lcm(frames, 3 E) distinct extraction keys, 3 E
    # match keys, one LocalBA plan — and is replayed from a hipGraph only from its third sighting
    # (eager, capture, replay; include/vx_slam.h).  Two full periods + 2 make every key of every
    # later step a replay, whatever --warmup is, so a short run (the driver's --steps 20 --warmup 5)
    # times the same graph replays as a long one.
    period = int(np.lcm(args.frames, 3 * E))
    prewarm = 2 * period + 2
    for i in range(-prewarm, 0):
        step(i)
    sync()

    # ---- profiling pass (HIP events on the library stream, every stage) -> dominant kernel
    stages = {}
    # (chunks of 5 steps, at least four: a stage's duration is the median of the chunks' averages —
    # in one 5-step pass, the driver's --warmup 5, a run of persistent windows launched while the
    # extraction kernels held the CUs they wait for once doubled the average, r06final2)
    n_chunk = max(4, (args.warmup + 4) // 5)
    n_prof = 5 * n_chunk
    if not args.no_profile:
        for c in ctxs:
            c.prof_enable(True)
        chunks = []
        for ch in range(n_chunk):
            for i in range(5):
                fstep(5 * ch + i)
            prof = {}
            for c in ctxs:  # (a stage that runs on several contexts — the extraction ones — is summed)
                for k, v in c.prof_read(reset=True).items():
                    if v[1]:
                        t, n = prof.get(k, (0.0, 0))
                        prof[k] = (t + v[0], n + v[1])
            chunks.append(prof)
        for c in ctxs:
            c.prof_enable(False)
        for k in {k for p in chunks for k in p}:
            per = [p[k][0] / p[k][1] for p in chunks if k in p and p[k][1]]
            launches = sum(p[k][1] for p in chunks if k in p)
            stages[k] = (float(np.median(per)), launches / n_prof)

    # ---- the timed region: no events inside (a timing event pair per launch costs ~25 % here)
    elapsed = timed_loop(fstep, args.steps, args.warmup, sync, dist)
    enqueue_ms = 1e3 * timed_loop.enqueue_s / args.steps

    # ---- roofline pass: the same K steps again, HIP events around every launch of the dominant
    # kernel on the stream it runs on (each bracket also spans that launch's dispatch boundary)
    dominant = max(stages, key=lambda k: stages[k][0] * stages[k][1]) if stages else None
    dctx = {"ba": bctx, "ma": mctx}.get(dominant[:2] if dominant else "", ectx)
    dom_prof, elapsed_ev = (0.0, 0), None
    if dominant:
        dctx.prof_enable(True, stages=[dominant])
        elapsed_ev = timed_loop(fstep, args.steps, 0, sync, dist)
        dom_prof = dctx.prof_read(reset=True).get(dominant, (0.0, 0))
        dctx.prof_enable(False)

    # single-frame latency: one step alone through the same dependency chain, host enqueue to done
    lat = []
    for i in range(20):
        sync()
        t0 = time.perf_counter()
        step((args.warmup + args.steps) * F + i)
        sync()
        lat.append(time.perf_counter() - t0)
    latency_ms = 1e3 * float(np.median(lat))

    # counts for the byte formulas
    last = (args.warmup + args.steps) * F + 19
    kps, _ = ectxs[loc(last)[0]].orb_fetch(loc(last)[1])
    matches = (ectxs[loc(last)[0]] if mon else mctx).match_fetch()
    st = plan.fetch(None)
    lw = [int(round(w / 1.2 ** l)) for l in range(8)]
    lh = [int(round(h / 1.2 ** l)) for l in range(8)]
    geo = {"W": w, "H": h, "level_px": [a * b for a, b in zip(lw, lh)]}
    counts = {"n_kp": len(kps), "n_cand": measured_candidates(vxslam, frames_host[last % args.frames], params),
              "n_q": len(kps), "n_t": len(kps),
              "n_match": len(matches), "n_pose_obs": info["n_pose_obs"], "n_lm_obs": info["n_lm_obs"],
              "n_split": info["n_split"], "n_opt": info["n_opt"], "n_kf": info["n_kf"],
              "ba_iters": int(st.iterations)}

    frames_total = args.steps * F * N
    ms_per_step = 1e3 * elapsed / args.steps
    value = 1e3 * elapsed / frames_total

    roofline = None
    if dominant and dom_prof[1]:
        # avg_launch_us: the profiling pass's per-dispatch duration (hipExtLaunchKernelGGL's start /
        # end timestamps, the interval rocprofv3's kernel trace reports; every stage timed, so every
        # context launches eagerly) — it agrees with the committed rocprofv3 average of the same
        # command (tests/test_bench_contract.py checks profiles/r06).  The second pass (only the
        # dominant stage timed, the other contexts replaying their graphs beside its eager launches)
        # is reported as avg_launch_us_dominant_pass: under that mix its dispatches run longer.
        avg_ms = stages[dominant][0]
        nbytes = stage_bytes(dominant, geo, counts)
        if nbytes:
            achieved = nbytes / (avg_ms * 1e-3) / 1e9
            roofline = {"kernel": dominant, "hip_kernel": HIP_KERNEL.get(dominant), "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                        "bytes_per_launch": int(nbytes), "avg_launch_us": round(avg_ms * 1e3, 2),
                        "avg_launch_us_source": "profiling pass (stages_us): per-dispatch timestamps, the median of "
                                                f"{n_chunk} five-step chunks' averages",
                        "avg_launch_us_dominant_pass": round(1e3 * dom_prof[0] / dom_prof[1], 2),
                        "launches_per_step": round(dom_prof[1] / args.steps, 2),
                        "pass_ms_per_step": round(1e3 * elapsed_ev / args.steps, 4)}
            fl = stage_flops(dominant, counts)
            if fl:
                tfs = fl / (avg_ms * 1e-3) / 1e12
                roofline.update({"flops_per_launch": int(fl), "fp64_achieved_tflops": round(tfs, 4),
                                 "fp64_peak_tflops": FP64_PEAK_TFS, "fp64_frac": round(tfs / FP64_PEAK_TFS, 5),
                                 "note": "latency-bound: neither HBM nor FP64 throughput binds (DESIGN.md §7)"})
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if roofline and os.path.exists(pmc):
        try:
            d = json.load(open(pmc))
            if d.get("config") == args.config and d.get("n_gpus") == N:  # counters of this very workload
                tr = d["bytes_per_launch"].get(dominant)
                if tr:
                    roofline["traffic"] = int(tr)
                    roofline["traffic_source"] = "profiles/pmc_traffic.json (rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE)"
        except Exception:
            pass

    cpu = None
    if full_affinity:  # (the CPU legs: every core this process may use, as before)
        os.sched_setaffinity(0, full_affinity)
    if dist.rank == 0 and N == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, frames_host, ba_map, args.cpu_sample)
        cpu["multi_thread"] = cpu_baseline_mt(cfg, frames_host, ba_map, args.cpu_sample)

    if dist.rank == 0:
        log(f"[bench] rank0 keypoints {len(kps)} matches {len(matches)} BA iterations {st.iterations} "
            f"obs/iter {list(st.obs[:st.iterations])} plan {info}")
        for k, (ms, n) in sorted(stages.items(), key=lambda kv: -kv[1][0] * kv[1][1]):
            log(f"[bench] stage {k:18s} {ms * 1e3:9.2f} us/launch x {n:5.2f} launches/step")
        if skip:
            log(f"[bench] --diag-skip {skip}: diagnostic run, not the metric")
        out = {
            "metric": (METRIC if not skip and not args.diag_nodep else
                       f"DIAGNOSTIC ({f'stage {skip} skipped' if skip else 'LocalBA not ordered after Match'})"),
            "value": round(value, 4),
            "unit": "ms/frame",
            "n_gpus": N,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": False,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "u8/i32 (FAST, pyramid, BRIEF), f32 (Harris, blur, angle), f64 (BA)",
            "data": "synthetic",
            "config": {
                "workload": (f"{args.config}: per rank and step {F} {w}x{h} BGR8 frame(s), each: {nf} ORB, kNN-2 "
                             f"Hamming match vs the previous frame, then {BA_PER_FRAME} run(s) of one LocalBA window "
                             f"of {nk * NW} KF / {nl * NW} landmarks (<= 5 alternating iterations), "
                             f"landmark-sharded over {N} GPU(s)" +
                             (f" ({args.scaling} scaling: {F * N} frames and {F * N} joint LocalBA runs per step "
                              f"in all)" if N > 1 else "")),
                "scaling": args.scaling,
                "frames_per_step": F * N,
                "parallelism": f"frames: 1 per rank; BA: landmark shards x{N}" + (" + RCCL all-reduce" if N > 1 else ""),
                "streams": {1: "1: Extract, Match, LocalBA back to back",
                            2: "2: Extract+Match | LocalBA (LocalBA(t) after Match(t))",
                            3: (f"{1 + E}: Extract+Match x{E} (frames alternate; Match(t) right after "
                                f"Extract(t) on its context, after Extract(t-1) on the other) | LocalBA"
                                if mon else f"{2 + E}: Extract x{E} (frames alternate) | Match | LocalBA")
                               + ", device events (LocalBA(t) after Match(t): Match and LocalBA in frame order; "
                                 "Extract(t) after the last Match reading its slot)"}[args.streams],
                "ba_window_kf": nk * NW,
                "ba_landmarks": nl * NW,
                "orb_features": nf,
                # LocalBA::Options of this run under the reference runner's flag names
                # (apps/main.cpp:42-47; --config FILE / --ba_* flags)
                "ba_options": ba_flags,
                "config_file": args.config_file,
            },
            # one frame alone through the same dependency chain (host enqueue to completion, median
            # of 20): the per-frame latency; `value` is the pipelined throughput
            "latency_ms_per_frame": round(latency_ms, 4),
            # host time to enqueue one step (Python + C-ABI calls, graph launches), diagnostic: the
            # GPU pipeline cannot run faster than this
            "host_enqueue_ms_per_step": round(enqueue_ms, 4),
            "host_path": host_path,
            "host_cpus": host_cpus,
            # untimed steps run before the warm-up so that every step of the timed region replays
            # captured graphs (see the pre-warm above)
            "prewarm_steps": prewarm,
            # the LocalBA plan (SelectKeyFrames + landmark set + CSRs) built on the device from the
            # map snapshot, incl. upload: paid once per LocalBA::Optimize() call of a drop-in
            # (a new keyframe, tracking.cpp:76-84); the timed steps replay a resident plan
            "ba_plan_build_ms": round(plan_build_ms, 3),
            # one whole drop-in LocalBA::Optimize() (plan build + solve + results back into the
            # map), median of 7, from the host snapshot and from the device-resident map (N = 1)
            "per_keyframe_ms": per_kf,
            # N > 1: the sharded LocalBA against the unsharded run of the same window (ok = within
            # 1e-4, no gate flips, same iterations, ranks bitwise agreed); null at N = 1
            "parity_vs_unsharded": parity,
            # N > 1: the communicator's size and rank as RCCL reports them (checked against the launch)
            "rccl": rccl,
            # what one step computed (the BA iteration count actually executed is
            # reported): LocalBA iterations and their valid pose-stage observations, the last frame's
            # keypoints and matches
            "work_per_step": {"ba_iterations": int(st.iterations),
                              "ba_observations_per_iteration": [int(x) for x in list(st.obs)[:int(st.iterations)]],
                              "keypoints": int(len(kps)), "matches": int(len(matches))},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "stages_us": {k: round(v[0] * 1e3, 2) for k, v in stages.items()},
        }
        print(json.dumps(out), flush=True)
    for sq in seqs:  # (before the contexts their calls name)
        sq.close()
    plan.close()
    for e in ev_e + ev_m:
        e.close()
    for c in reversed(ctxs):
        c.close()
    dist.close()


if __name__ == "__main__":
    main()
