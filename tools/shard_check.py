#!/usr/bin/env python
"""Multi-process check of the channel-sharded loop (torchrun, one rank per
process; several ranks may share one GPU with --backend gloo).

    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
        tools/shard_check.py --backend gloo --shape 12 2048 256

Every rank cleans its channel shard through dist.TorchComm; rank 0 then cleans
the whole archive in one unsharded session and asserts the zap mask, test
values and loop counters are bit-identical.  Prints one JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--shape", type=int, nargs=3, default=[12, 2048, 256])
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--cli", action="store_true",
                    help="run the CLI (IC_CHANNEL_SHARDS=1) and compare its output archive and stdout")
    a = ap.parse_args()
    if a.cli:
        return cli_check(a)

    import numpy as np
    import torch
    import torch.distributed as dist

    from iterative_cleaner_amd import _native, sharded, synth
    from iterative_cleaner_amd.dist import rank_world

    rank, world, local = rank_world()
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % max(ndev, 1))
    torch.cuda.set_device(dev)
    if a.backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")
    nsub, nchan, nbin = a.shape
    data, w0, shift = synth.make_cube(nsub, nchan, nbin, a.seed, 0.2)
    raw = np.ascontiguousarray(data[:, 0])
    chans, _ = _native.shard_layout(nsub, nchan, world)
    c0, c1 = chans[rank]
    t0 = time.perf_counter()
    out = sharded.clean_cube_dist(raw[:, c0:c1], w0[:, c0:c1], shift[c0:c1], (nsub, nchan, nbin), dev)
    dt = time.perf_counter() - t0
    ok = None
    if rank == 0:
        with _native.GpuSession(nsub, nchan, nbin, device=dev.index) as s:
            s.upload(raw, w0, shift)
            one = s.run()
        ok = (out["weights"].tobytes() == one["weights"].tobytes()
              and out["test"].tobytes() == one["test"].tobytes()
              and out["loops"] == one["loops"] and list(out["changed"]) == list(one["changed"]))
        print(json.dumps({"backend": a.backend, "world": world, "shape": a.shape, "loops": out["loops"],
                          "zapped": int((out["weights"] == 0).sum()), "bit_identical": ok,
                          "seconds": round(dt, 3)}))
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0 and not ok:
        sys.exit(1)


def cli_check(a):
    """The reference CLI flow (iterative_cleaner.py:59-62, clean() + unload) with
    every archive cleaned by all ranks as channel shards; rank 0's stdout and
    output archive must equal a single-process run's."""
    import contextlib
    import io
    import tempfile

    import numpy as np
    import torch.distributed as dist

    from iterative_cleaner_amd import archive as ica
    from iterative_cleaner_amd import cleaner, synth
    from iterative_cleaner_amd.dist import rank_world

    os.environ["IC_CHANNEL_SHARDS"] = "1"
    os.environ.setdefault("IC_SHARD_BACKEND", a.backend)
    rank, world, local = rank_world()
    import torch
    os.environ["IC_DEVICE"] = str(local % max(1, torch.cuda.device_count()))
    from iterative_cleaner_amd.dist import channel_sharding
    assert channel_sharding()           # creates the process group
    tmp = os.path.join(tempfile.gettempdir(), "ic_shard_cli")
    os.makedirs(tmp, exist_ok=True)
    os.chdir(tmp)
    nsub, nchan, nbin = a.shape
    if rank == 0:
        synth.make_archive(nsub, nchan, nbin, a.seed, 0.2, npol=2, filename="cli.ar").unload("cli.ar")
    dist.barrier()
    argv = ["-l", "-u", "cli.ar"]
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        cleaner.main(cleaner.parse_arguments(argv))
    dist.barrier()
    ok = True
    if rank == 0:
        sharded_out = buf.getvalue()
        w_sh = ica.Archive_load("cli_cleaned.ar").get_weights()
        res = sorted(f for f in os.listdir(".") if "_residual_" in f)
        r_sh = ica.Archive_load(res[-1]).get_data()
        os.environ["IC_CHANNEL_SHARDS"] = "0"
        buf1 = io.StringIO()
        with contextlib.redirect_stdout(buf1):
            cleaner.main(cleaner.parse_arguments(argv))
        w_1 = ica.Archive_load("cli_cleaned.ar").get_weights()
        r_1 = ica.Archive_load(res[-1]).get_data()
        ok = (sharded_out == buf1.getvalue() and w_sh.tobytes() == w_1.tobytes()
              and np.array_equal(r_sh, r_1))
        print(json.dumps({"cli": True, "backend": a.backend, "world": world, "shape": a.shape,
                          "stdout_equal": sharded_out == buf1.getvalue(),
                          "weights_equal": w_sh.tobytes() == w_1.tobytes(),
                          "residual_equal": bool(np.array_equal(r_sh, r_1)), "stdout": sharded_out}))
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0 and not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
