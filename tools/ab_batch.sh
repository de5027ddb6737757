#!/bin/bash
# A/B of prebuilt library variants on the batch pipeline (bench.py --batch):
#   tools/ab_batch.sh "v1 v2" WORKLOAD BATCH "LANES..." ROUNDS -> gpurun_out/abb/<wl>_<v>_<lanes>_<round>.json
set -o pipefail
VARS=${1:?variants}; WL=${2:?workload}; B=${3:?batch}; LANES=${4:?lanes}; R=${5:-2}
mkdir -p gpurun_out/abb
for r in $(seq 1 $R); do
  for l in $LANES; do
    for v in $VARS; do
      f=gpurun_out/abb/${WL}_${v}_${l}_$r
      IC_LIBRARY=ab/libicgpu_$v.so timeout -k 10 200 python bench.py --workload $WL --batch $B --lanes $l \
          --steps 3 --warmup 1 > $f.json 2> $f.err || exit 1
      python3 -c "
import json; d=json.loads(open('$f.json').read().splitlines()[-1]); c=d['config']
print('$WL $v lanes $l round $r', c['ms_per_archive'], 'ms/archive', d['value'])"
    done
  done
done
