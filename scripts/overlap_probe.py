"""Where does the 3-stream pipeline lose time?  Per-frame time of Extract / Match / LocalBA alone,
of independent pairs on separate contexts (no events), and of the event-ordered pipeline."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visionx-slam_amd", "python"))
import torch  # noqa: E402
import vxslam  # noqa: E402
from vxslam import synth  # noqa: E402

h, w, nf, nk, nl = 480, 640, 2000, 50, 20000
# $VX_PRIO = "E M B" stream priorities (> 0: high) of the three contexts
pe, pm, pb = (int(x) for x in os.environ.get("VX_PRIO", "0 0 0").split())
e, m, b = vxslam.Context(0, priority=pe), vxslam.Context(0, priority=pm), vxslam.Context(0, priority=pb)
e.set_grid_share(float(os.environ.get("VX_GRID_SHARE", 1.0 / 3.0)))  # as bench.py
frames = torch.from_numpy(synth.make_frames(7, 8, h, w)).cuda()
params = vxslam.default_orb_params(n_features=nf)
plan = b.ba_plan(synth.make_ba_map(0x5EED0003, nk, nl), vxslam.default_ba_options(window=nk))
for i in range(3):
    e.orb_extract_async(frames[i].data_ptr(), w, h, 3, w * 3, i, params)
e.synchronize()
slot = [e.slot_device(s) for s in range(3)]
ev_e = e.event()
ev_m = [m.event() for _ in range(3)]


def E(i):
    e.orb_extract_async(frames[i % 8].data_ptr(), w, h, 3, w * 3, i % 3, params)


def M(i):
    m.match_device_async(slot[(i - 1) % 3], slot[i % 3])


def B(i):
    plan.run_async()


def piped(i):
    e.wait_event(ev_m[(i + 1) % 3])
    E(i)
    e.record(ev_e)
    m.wait_event(ev_e)
    M(i)
    m.record(ev_m[i % 3])
    b.wait_event(ev_m[i % 3])
    B(i)


def em_only(i):  # Match(t) after Extract(t); LocalBA unordered
    e.wait_event(ev_m[(i + 1) % 3])
    E(i)
    e.record(ev_e)
    m.wait_event(ev_e)
    M(i)
    m.record(ev_m[i % 3])
    B(i)


def mb_only(i):  # LocalBA(t) after Match(t); Match unordered after Extract
    E(i)
    M(i)
    m.record(ev_m[i % 3])
    b.wait_event(ev_m[i % 3])
    B(i)


def run(name, fns, K=200):
    for i in range(10):
        for f in fns:
            f(i)
    for c in (e, m, b):
        c.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        for f in fns:
            f(10 + i)
    for c in (e, m, b):
        c.synchronize()
    print(f"{name:28s} {1e3 * (time.perf_counter() - t0) / K:.4f} ms/frame", flush=True)


run("extract alone", [E])
run("match alone", [M])
run("localBA alone", [B])
run("extract | localBA (no deps)", [E, B])
run("extract | match (no deps)", [E, M])
run("extract | match | BA (no deps)", [E, M, B])
run("events E->M only", [em_only])
run("events M->B only", [mb_only])
run("pipeline (events)", [piped])

# two extraction contexts (bench.py --extract-ctx 2): frames alternate between them
e2 = vxslam.Context(0, priority=pe)
e2.set_grid_share(float(os.environ.get("VX_GRID_SHARE", 1.0 / 3.0)))
for i in range(3):
    e2.orb_extract_async(frames[i].data_ptr(), w, h, 3, w * 3, i, params)
e2.synchronize()


def E2(i):
    (e if i % 2 == 0 else e2).orb_extract_async(frames[i % 8].data_ptr(), w, h, 3, w * 3, (i // 2) % 3, params)


def run2(name, fns, K=200):
    for i in range(10):
        for f in fns:
            f(i)
    for c in (e, e2, m, b):
        c.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        for f in fns:
            f(10 + i)
    for c in (e, e2, m, b):
        c.synchronize()
    print(f"{name:28s} {1e3 * (time.perf_counter() - t0) / K:.4f} ms/frame", flush=True)


run2("extract x2 alone", [E2])
run2("extract x2 | localBA", [E2, B])
run2("match | localBA", [M, B])
run2("extract x2 | match", [E2, M])
run2("extract x2 | match | BA", [E2, M, B])
