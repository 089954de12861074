# Schur plan rebuild: kernel and HIP API statistics of 10 and 60 in-place rebuilds (the difference
# / 50 is one rebuild's share, setup excluded); outputs under gpurun_out/$TAG
set -o pipefail
TAG=${TAG:-r04w}
mkdir -p gpurun_out/$TAG && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 4
for n in 10 60; do
  timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/kt$n -o kt -- python3 scripts/sba_rebuild_loop.py $n $ARGS > gpurun_out/$TAG/out$n.txt 2>&1 || exit 4
  for k in hip_api_stats kernel_stats; do
    f=$(ls gpurun_out/$TAG/kt$n/*/kt_$k.csv gpurun_out/$TAG/kt$n/kt_$k.csv 2>/dev/null | head -1)
    cp $f gpurun_out/$TAG/${k}_$n.csv
  done
  rm -rf gpurun_out/$TAG/kt$n
done
grep rebuild gpurun_out/$TAG/out*.txt
