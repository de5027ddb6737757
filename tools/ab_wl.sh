#!/bin/bash
# A/B of prebuilt library variants over several workloads, alternating, with
# the chan-partials and fit kernel times of bench.py's per-kernel breakdown:
#   tools/ab_wl.sh "v1 v2" "C1 C2" ROUNDS  -> gpurun_out/abwl/<wl>_<variant>_<round>.json
set -o pipefail
VARS=${1:?variants}; WLS=${2:?workloads}; R=${3:-2}
mkdir -p gpurun_out/abwl
for wl in $WLS; do
 for r in $(seq 1 $R); do
  for v in $VARS; do
    f=gpurun_out/abwl/${wl}_${v}_$r
    IC_LIBRARY=ab/libicgpu_$v.so timeout -k 10 200 python bench.py --workload $wl --steps 10 --warmup 2 \
        --no-cpu-baseline --no-flip-check --no-fast-summary > $f.json 2> $f.err || exit 1
    python3 -c "
import json; d=json.loads(open('$f.json').read().splitlines()[-1]); pk=d['roofline']['per_kernel']
print('$wl $v $r', d['ms_per_step'], {k: round(v['ms_per_step'], 4) for k, v in pk.items() if k in ('k_chan_partials', 'k_fit_pass', 'k_fit_tail', 'k_diag')})"
  done
 done
done
