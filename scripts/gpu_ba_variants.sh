cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/var
L=visionx-slam_amd/lib
for v in pb256_s8 pb256_s4 pb1024_s2; do
  VX_LIB=$L/libvxslam_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "ba or BA" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/var/t_$v.log 2>&1 || { echo "$v tests failed"; tail -20 gpurun_out/var/t_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/var/t_$v.log)"
done
for r in 1 2; do
  for v in base pb256_s8 pb256_s4 pb1024_s2; do
    if [ $v = base ]; then unset VX_LIB; else export VX_LIB=$L/libvxslam_$v.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/var/b_${v}_$r.json 2>/dev/null || { echo "$v bench failed"; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/var/b_${v}_$r.json')); s=d['stages_us']; print('$v', d['value'], d['latency_ms_per_frame'], s['ba_pose_partial'], s['ba_landmark'])"
  done
done
unset VX_LIB
