#!/bin/bash
# One GPU session on the box (run from the repo root through gpurun):
#   tools/gpu_session.sh TAG "STEP" ["STEP" ...]
# Each STEP is a command run under its own time limit (IC_STEP_TIMEOUT, default
# 300 s), its output in gpurun_out/TAG/<n>.log.  A step that fails with an
# ordinary error (exit 1, e.g. a failing assertion) lets the session go on; a
# time limit, abort or crash (124, 134, 137, 139, ...) ends it: nothing more
# touches the GPU after a fault.
set -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
# the in-tree library must be built from the sources being shipped
for src in iterative_cleaner_amd/csrc/*.hip iterative_cleaner_amd/csrc/*.h include/*.h; do
    if [ "$src" -nt iterative_cleaner_amd/libicgpu.so ]; then
        echo "libicgpu.so is older than $src: rebuild (make -C iterative_cleaner_amd/csrc) first"
        exit 2
    fi
done
n=0
for step in "$@"; do
    n=$((n + 1))
    echo "[$n] $step" | tee -a "$OUT/steps.txt"
    timeout -k 10 "${IC_STEP_TIMEOUT:-300}" bash -c "$step" > "$OUT/$n.log" 2>&1
    rc=$?
    echo "[$n] rc=$rc" | tee -a "$OUT/steps.txt"
    tail -5 "$OUT/$n.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "step $n ended with rc=$rc: stopping the session"
        exit $rc
    fi
done
echo "session done"
