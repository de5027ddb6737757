#!/bin/bash
# Rehearsal of the driver's N-GPU bench path on one GPU: N ranks (torchrun,
# gloo process group) share the GPU, and the library's native RCCL transport
# loads the test stub librccl (tests/stub_rccl) in place of the real one, so
# ic_session_create_rccl, the unique-id broadcast, the C++-issued exchanges and
# the max-over-ranks line run exactly as on N GPUs (the time is meaningless).
# The stub stages each rank's sends in a POSIX shm outbox of IC_STUB_RCCL_OUTBOX_MB
# (default here 512: C3's diagnostics rows at world 2 exceed the stub's 32-MiB default).
#   tools/rehearse_native_rccl.sh N [bench args...] -> gpurun_out/rehearse_N.json
set -o pipefail
N=${1:?ranks}; shift
mkdir -p gpurun_out
IC_BENCH_BACKEND=gloo IC_BENCH_RCCL_LIBRARY=$PWD/tests/stub_rccl/libstubrccl.so IC_STUB_RCCL_OUTBOX_MB=${IC_STUB_RCCL_OUTBOX_MB:-512} \
    timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29500 + N)) bench.py --gpus $N "$@" > gpurun_out/rehearse_$N.json 2> gpurun_out/rehearse_$N.err \
    || { tail -20 gpurun_out/rehearse_$N.err; exit 1; }
tail -1 gpurun_out/rehearse_$N.json
