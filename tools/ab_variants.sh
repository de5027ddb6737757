#!/bin/bash
# A/B of prebuilt library variants (tools/build_variant.sh) on one bench workload, alternating:
#   tools/ab_variants.sh "b16 b32 b8" [ROUNDS] [bench args...]  -> gpurun_out/ab/<variant>_<round>.json
set -o pipefail
VARS=${1:?variants}; R=${2:-2}; shift 2
mkdir -p gpurun_out/ab
for r in $(seq 1 $R); do
  for v in $VARS; do
    IC_LIBRARY=ab/libicgpu_$v.so timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline \
        --no-flip-check --no-fast-summary "$@" > gpurun_out/ab/${v}_$r.json 2> gpurun_out/ab/${v}_$r.err || exit 1
    echo "$v $r done"
  done
done
