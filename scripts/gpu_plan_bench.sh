mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/sba_bench.py 20 > gpurun_out/sba_bench.json 2> gpurun_out/sba_bench.err && \
timeout -k 10 300 python -u scripts/plan_build_time.py > gpurun_out/plan_build_time.json 2> gpurun_out/plan_build_time.err
