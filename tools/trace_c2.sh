#!/bin/bash
# kernel trace of one clean (bench.py --steps 1 --warmup 1), summarised per dispatch
#   tools/trace_c2.sh TAG [WORKLOAD] [bench args...]
set -o pipefail
OUT=gpurun_out/trace_${1:-x}
WL=${2:-C2}
shift 2 2>/dev/null || shift $#
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/raw -o run -- \
    python3 bench.py --workload $WL --steps 1 --warmup 1 --no-cpu-baseline --no-fast-summary "$@" > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
python3 tools/trace_rounds.py $(find $OUT/raw -name '*kernel_trace.csv' | head -1) > $OUT/rounds.txt || exit 1
rm -rf $OUT/raw
echo trace done
