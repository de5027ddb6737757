#!/bin/bash
# A/B of bench argument sets on one workload, alternating (session options:
# "--option NAME=VALUE ..."; the library reads no environment knobs):
#   tools/ab_args.sh TAG ROUNDS "ARGS1" "ARGS2" ... -- [common bench args...]  -> gpurun_out/abargs_TAG/<i>_<round>.json
# (each ARGS is a space-separated list of bench arguments, "-" for none)
set -o pipefail
TAG=${1:?tag}; R=${2:?rounds}; shift 2
VARS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do VARS+=("$1"); shift; done
[ "$1" = "--" ] && shift
OUT=gpurun_out/abargs_$TAG
mkdir -p $OUT
for r in $(seq 1 $R); do
  for i in "${!VARS[@]}"; do
    v=${VARS[$i]}; [ "$v" = "-" ] && v=""
    timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-fast-summary $v "$@" \
        > $OUT/${i}_$r.json 2> $OUT/${i}_$r.err || exit 1
    echo "[$i] $v round $r: $(python3 -c "import json,sys; print(json.loads(open('$OUT/${i}_$r.json').read().splitlines()[-1])['ms_per_step'])")"
  done
done
