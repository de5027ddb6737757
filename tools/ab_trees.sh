#!/bin/bash
# Same-box A/B of whole source trees (bench.py + library of each), alternating:
#   tools/ab_trees.sh "dirA dirB" ROUNDS WORKLOAD [bench args...] -> gpurun_out/abt/<name>_<wl>_<round>.json
# "." is this tree; other dirs are snapshots staged under ab/ (e.g. ab/r3).
set -o pipefail
DIRS=${1:?dirs}; R=${2:-2}; WL=${3:?workload}; shift 3
root=$(pwd)
mkdir -p gpurun_out/abt
for r in $(seq 1 $R); do
  for d in $DIRS; do
    n=$(basename $(cd $d && pwd)); [ "$d" = "." ] && n=head
    f=$root/gpurun_out/abt/${n}_${WL}_$r
    (cd $d && timeout -k 10 300 python bench.py --workload $WL --steps 5 --warmup 2 --no-cpu-baseline \
        --no-flip-check --no-fast-summary "$@" > $f.json 2> $f.err) || { tail -5 $f.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$f.json').read().splitlines()[-1])
print('$n', '$WL', $r, d['ms_per_step'])"
  done
done
