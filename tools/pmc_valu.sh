#!/bin/bash
# f64 VALU evidence for a bench workload (run on the GPU box from the repo root): one rocprofv3
# PMC pass (8 SQ counters, nothing else) over `bench.py --steps 1 --warmup 0`, summarised per
# kernel by tools/pmc_valu.py into f64 lane-ops per launch (bench.py reads the JSON, like the
# FETCH/WRITE traffic summary).
# Usage: tools/pmc_valu.sh TAG [WORKLOAD] [exact|closed] [shift|fft] -> gpurun_out/valu_TAG/{pmc_valu.json,summary.txt}
set -o pipefail
TAG=${1:?tag}
WL=${2:-C2}
FM=${3:-exact}            # bench.py --fit-mode (closed: summaries keyed WL/closed)
DD=${4:-shift}            # bench.py --dedisp (fft: summaries keyed .../fft)
KEY=$WL; [ "$FM" = closed ] && KEY=$WL/closed; [ "$DD" != shift ] && KEY=$KEY/$DD
OUT=gpurun_out/valu_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 \
    SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVES \
    --output-format csv -d $OUT/pmc -o run -- \
    python3 bench.py --workload $WL --fit-mode $FM --dedisp $DD --steps 1 --warmup 0 --no-cpu-baseline --no-flip-check --no-fast-summary > $OUT/pmc.log 2>&1 \
    || { tail -20 $OUT/pmc.log; exit 1; }
C=$(find $OUT/pmc -name '*counter_collection.csv' | head -1)
python3 tools/pmc_summary.py "$C" > $OUT/summary.txt || exit 1
python3 tools/pmc_valu.py "$C" --workload $KEY --out $OUT/pmc_valu.json || exit 1
rm -rf $OUT/pmc
echo valu done
