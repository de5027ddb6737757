#!/bin/bash
# Rehearsal of the driver's N-GPU bench path on one GPU: N ranks (torchrun,
# gloo process group) share the GPU, and the library's native RCCL transport
# loads the test stub librccl (tests/stub_rccl) in place of the real one, so
# ic_session_create_rccl, the unique-id broadcast, the C++-issued exchanges and
# the max-over-ranks line run exactly as on N GPUs (the time is meaningless).
#   tools/rehearse_native_rccl.sh N [bench args...] -> gpurun_out/rehearse_N.json
set -o pipefail
N=${1:?ranks}; shift
mkdir -p gpurun_out
IC_BENCH_BACKEND=gloo IC_BENCH_RCCL_LIBRARY=$PWD/tests/stub_rccl/libstubrccl.so \
    timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29500 + N)) bench.py --gpus $N "$@" > gpurun_out/rehearse_$N.json 2> gpurun_out/rehearse_$N.err \
    || { tail -20 gpurun_out/rehearse_$N.err; exit 1; }
tail -1 gpurun_out/rehearse_$N.json
