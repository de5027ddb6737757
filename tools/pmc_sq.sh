#!/bin/bash
# SQ / TCC counter passes of one bench step, per kernel (separate rocprofv3 runs,
# <= 8 SQ and <= 4 TCC counters each).  Usage: tools/pmc_sq.sh TAG [WORKLOAD] [exact|closed] [shift|fft]
set -o pipefail
OUT=gpurun_out/pmcsq_${1:-x}
WL=${2:-C2}
FM=${3:-exact}
DD=${4:-shift}            # bench.py --dedisp (fft: summaries keyed .../fft)
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name counters...
    local name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- \
        python3 bench.py --workload $WL --fit-mode $FM --dedisp $DD --steps 1 --warmup 0 --no-cpu-baseline --no-flip-check --no-fast-summary > $OUT/$name.log 2>&1 \
        || { tail -20 $OUT/$name.log; return 1; }
    python3 tools/pmc_summary.py $(find $OUT/$name -name '*counter_collection.csv' | head -1) > $OUT/$name.txt \
        && rm -rf $OUT/$name
}
run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT &&
run tcc TCC_HIT_sum TCC_MISS_sum &&
echo pmc done
