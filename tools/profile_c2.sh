#!/bin/bash
# rocprofv3 evidence for a bench workload (run on the GPU box from the repo root):
#   1. --kernel-trace --stats of `bench.py --steps 5` (per-kernel average durations),
#   2. two separate PMC passes (FETCH_SIZE, WRITE_SIZE) of `bench.py --steps 1 --warmup 0`,
#      summarised by tools/pmc_traffic.py into per-launch HBM traffic.
# Usage: tools/profile_c2.sh TAG [WORKLOAD] [exact|closed] [shift|fft]   -> gpurun_out/prof_TAG/{kernel_stats.csv,pmc_traffic.json,*.log}
# The raw traces are deleted (gpurun copies back at most 64 MiB).
set -o pipefail
TAG=${1:?tag}
WL=${2:-C2}
FM=${3:-exact}            # bench.py --fit-mode (closed: summaries keyed WL/closed)
DD=${4:-shift}            # bench.py --dedisp (fft: summaries keyed .../fft)
KEY=$WL; [ "$FM" = closed ] && KEY=$WL/closed; [ "$DD" != shift ] && KEY=$KEY/$DD
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
show() { echo "---- $1"; tail -20 "$1"; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
    python3 bench.py --workload $WL --fit-mode $FM --dedisp $DD --steps 5 --warmup 1 --no-cpu-baseline --no-flip-check --no-fast-summary > $OUT/bench_stats.log 2>&1 \
    || { show $OUT/bench_stats.log; exit 1; }
find $OUT/stats -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmcF -o run -- \
    python3 bench.py --workload $WL --fit-mode $FM --dedisp $DD --steps 1 --warmup 0 --no-cpu-baseline --no-flip-check --no-fast-summary > $OUT/pmcF.log 2>&1 \
    || { show $OUT/pmcF.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmcW -o run -- \
    python3 bench.py --workload $WL --fit-mode $FM --dedisp $DD --steps 1 --warmup 0 --no-cpu-baseline --no-flip-check --no-fast-summary > $OUT/pmcW.log 2>&1 \
    || { show $OUT/pmcW.log; exit 1; }
F=$(find $OUT/pmcF -name '*counter_collection.csv' | head -1)
W=$(find $OUT/pmcW -name '*counter_collection.csv' | head -1)
find $OUT -maxdepth 3 | head -40
python3 tools/pmc_traffic.py --fetch "$F" --write "$W" --workload $KEY --out $OUT/pmc_traffic.json || exit 1
rm -rf $OUT/stats $OUT/pmcF $OUT/pmcW
echo profile done
