#!/bin/bash
# per-kernel stats of one bench run: tools/kstats.sh TAG BENCH_ARGS... -> gpurun_out/ks_TAG/kernel_stats.csv
set -o pipefail
T=$1; shift
mkdir -p gpurun_out/ks_$T
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks_$T/raw -o run -- python3 bench.py "$@" > gpurun_out/ks_$T/bench.log 2>&1 || { tail -20 gpurun_out/ks_$T/bench.log; exit 1; }
find gpurun_out/ks_$T/raw -name '*kernel_stats.csv' -exec cp {} gpurun_out/ks_$T/kernel_stats.csv \;
rm -rf gpurun_out/ks_$T/raw
