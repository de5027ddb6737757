set -e
mkdir -p gpurun_out/ls
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_stats_gpu.py > gpurun_out/ls/tests.log 2>&1
for W in 0 4 8; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --option rowstat_waves=$W > gpurun_out/ls/b_$W.json 2> gpurun_out/ls/b_$W.err
done
