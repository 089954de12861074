for T in 1 16; do
VX_SBA_PLAN_THREADS=$T VX_SBA_PLAN_TIMING=1 timeout -k 10 200 python -c "
import sys; sys.path.insert(0,'visionx-slam_amd/python')
import vxslam
from vxslam import synth
ctx = vxslam.Context(0)
nk, nl, ns = synth.ba_config('C5')
m = synth.make_ba_map(0x5EED0000 + nk, nk, nl, n_streams=ns, n_old_kf=2 * ns)
o = vxslam.default_sba_options(window=nk, iters=8)
for r in range(3):
    print('T=$T rep', r, file=sys.stderr)
    ctx.sba_plan(m, o).close()
" > gpurun_out/sbat_$T.log 2>&1 || exit 1
tail -7 gpurun_out/sbat_$T.log
done
