#!/bin/bash
# A/B of prebuilt library variants on k_diag (per-kernel breakdown of bench.py, fork off):
#   tools/ab_kdiag.sh "v1 v2" ROUNDS [bench args...] -> gpurun_out/abk/<variant>_<round>.json + summary lines
set -o pipefail
VARS=${1:?variants}; R=${2:-2}; shift 2
mkdir -p gpurun_out/abk
for r in $(seq 1 $R); do
  for v in $VARS; do
    IC_LIBRARY=ab/libicgpu_$v.so timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --option diag_fork=0 \
        --no-flip-check --no-fast-summary "$@" > gpurun_out/abk/${v}_$r.json 2> gpurun_out/abk/${v}_$r.err || exit 1
    python3 -c "
import json; d=json.loads(open('gpurun_out/abk/${v}_$r.json').read().splitlines()[-1]); pk=d['roofline']['per_kernel']['k_diag']
print('$v', $r, d['ms_per_step'], 'k_diag ms/launch', round(pk['ms_per_step']/pk['launches_per_step'], 4))"
  done
done
