mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sba.py tests/test_gpu_parity.py tests/test_gpu_dmap.py > gpurun_out/sba_tests.log 2>&1 || exit 1
VX_SBA_PLAN_TIMING=1 timeout -k 10 200 python -c "
import sys; sys.path.insert(0,'visionx-slam_amd/python')
import vxslam
from vxslam import synth
ctx = vxslam.Context(0)
for cfg in ('C3','C5'):
    nk, nl, ns = synth.ba_config(cfg)
    m = synth.make_ba_map(0x5EED0000 + nk, nk, nl, n_streams=ns, n_old_kf=2 * ns)
    o = vxslam.default_sba_options(window=nk, iters=8)
    for r in range(2):
        print(cfg, r, file=sys.stderr)
        ctx.sba_plan(m, o).close()
" > gpurun_out/sba_timing.log 2>&1
exit 0
