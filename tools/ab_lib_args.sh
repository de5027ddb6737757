#!/bin/bash
# A/B of prebuilt library variants with extra bench arguments, alternating:
#   tools/ab_lib_args.sh "v1 v2" ROUNDS [bench args...] -> gpurun_out/abl/<variant>_<round>.json
set -o pipefail
VARS=${1:?variants}; R=${2:-2}; shift 2
mkdir -p gpurun_out/abl
for r in $(seq 1 $R); do
  for v in $VARS; do
    f=gpurun_out/abl/${v}_$r
    IC_LIBRARY=ab/libicgpu_$v.so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline \
        --no-flip-check --no-fast-summary "$@" > $f.json 2> $f.err || exit 1
    python3 -c "
import json; d=json.loads(open('$f.json').read().splitlines()[-1]); pk=d['roofline']['per_kernel']
print('$v', $r, d['ms_per_step'], {k: round(x['ms_per_step'], 3) for k, x in pk.items() if k in ('k_rotate', 'k_fit_pass', 'k_diag')})"
  done
done
