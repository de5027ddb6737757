#!/bin/bash
# A/B of prebuilt library variants on the FFT-rotation mode, alternating, with
# the k_rotate / fit / diagnostics times of bench.py's per-kernel breakdown:
#   tools/ab_fft.sh "v1 v2" ROUNDS [WORKLOAD]  -> gpurun_out/abfft/<variant>_<round>.json
set -o pipefail
VARS=${1:?variants}; R=${2:-2}; WL=${3:-C2}
mkdir -p gpurun_out/abfft
for r in $(seq 1 $R); do
  for v in $VARS; do
    f=gpurun_out/abfft/${v}_$r
    IC_LIBRARY=ab/libicgpu_$v.so timeout -k 10 200 python bench.py --workload $WL --dedisp fft --steps 5 --warmup 1 \
        --no-cpu-baseline --no-flip-check --no-fast-summary > $f.json 2> $f.err || exit 1
    python3 -c "
import json; d=json.loads(open('$f.json').read().splitlines()[-1]); pk=d['roofline']['per_kernel']
print('$v $r', d['ms_per_step'], {k: round(v['ms_per_step'], 4) for k, v in pk.items() if k in ('k_rotate', 'k_fit_pass', 'k_diag')})"
  done
done
