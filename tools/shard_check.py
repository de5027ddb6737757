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
    ap.add_argument("--oracle", action="store_true", help="rank 0 also checks the C oracle's loop")
    ap.add_argument("--fit-mode", type=int, default=0, help="0 exact (default), 1 closed form")
    ap.add_argument("--fail-rank", type=int, default=-1,
                    help="fault injection: this rank's transport fails at collective --fail-at")
    ap.add_argument("--fail-at", type=int, default=3)
    ap.add_argument("--out", default="", help="directory for one JSON result file per rank")
    ap.add_argument("--cli-suffix", default=".ar", help="--cli: archive file suffix (.ar npz, .sf PSRFITS)")
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
    from iterative_cleaner_amd.dist import pg_timeout
    if a.backend == "nccl":
        dist.init_process_group("nccl", device_id=dev, timeout=pg_timeout())
    else:
        dist.init_process_group("gloo", timeout=pg_timeout())
    nsub, nchan, nbin = a.shape
    data, w0, shift = synth.make_cube(nsub, nchan, nbin, a.seed, 0.2)
    raw = np.ascontiguousarray(data[:, 0])
    chans, _ = _native.shard_layout(nsub, nchan, world)
    c0, c1 = chans[rank]
    t0 = time.perf_counter()
    fail_at = a.fail_at if rank == a.fail_rank else None
    try:
        out = sharded.clean_cube_dist(raw[:, c0:c1], w0[:, c0:c1], shift[c0:c1], (nsub, nchan, nbin), dev,
                                      fail_at=fail_at, fit_mode=a.fit_mode)
    except _native.NativeError as e:
        # a failed shard (injected, or a peer that failed): report and leave
        rec = {"rank": rank, "world": world, "failed": True, "error": str(e),
               "seconds": round(time.perf_counter() - t0, 3)}
        _emit(a, rank, rec)
        sys.stdout.flush()
        os._exit(3)
    dt = time.perf_counter() - t0
    ok = None
    rec = {"rank": rank, "backend": a.backend, "world": world, "shape": a.shape, "loops": out["loops"],
           "zapped": int((out["weights"] == 0).sum()), "seconds": round(dt, 3), "failed": False}
    if rank == 0:
        with _native.GpuSession(nsub, nchan, nbin, device=dev.index, fit_mode=a.fit_mode) as s:
            s.upload(raw, w0, shift)
            one = s.run()
        ok = (out["weights"].tobytes() == one["weights"].tobytes()
              and out["test"].tobytes() == one["test"].tobytes()
              and out["loops"] == one["loops"] and list(out["changed"]) == list(one["changed"]))
        rec["bit_identical"] = ok
        if a.oracle:
            from oracle import lib as oracle
            ref = oracle.clean_loop(raw, w0, shift, fit_mode=a.fit_mode)
            rec["oracle_weights_equal"] = out["weights"].tobytes() == ref["weights"].tobytes()
            rec["oracle_loops_equal"] = out["loops"] == ref["loops"]
            ok = ok and rec["oracle_weights_equal"] and rec["oracle_loops_equal"]
    _emit(a, rank, rec)
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0 and not ok:
        sys.exit(1)


def _emit(a, rank, rec):
    line = json.dumps(rec)
    if rank == 0:
        print(line)
    if a.out:
        os.makedirs(a.out, exist_ok=True)
        with open(os.path.join(a.out, "rank%d.json" % rank), "w") as f:
            f.write(line + "\n")


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
    tmp = os.path.join(a.out or tempfile.gettempdir(), "ic_shard_cli")
    os.makedirs(tmp, exist_ok=True)
    os.chdir(tmp)
    nsub, nchan, nbin = a.shape
    name = "cli" + a.cli_suffix
    if rank == 0:
        synth.make_archive(nsub, nchan, nbin, a.seed, 0.2, npol=2, filename=name).unload(name)
    dist.barrier()
    argv = ["-l", "-u", name]
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        cleaner.main(cleaner.parse_arguments(argv))
    dist.barrier()
    ok = True
    if rank == 0:
        sharded_out = buf.getvalue()
        w_sh = ica.Archive_load("cli_cleaned.ar").get_weights()
        d_sh = ica.Archive_load("cli_cleaned.ar").get_data()
        res = sorted(f for f in os.listdir(".") if "_residual_" in f)
        r_sh = ica.Archive_load(res[-1]).get_data()
        os.environ["IC_CHANNEL_SHARDS"] = "0"
        buf1 = io.StringIO()
        with contextlib.redirect_stdout(buf1):
            cleaner.main(cleaner.parse_arguments(argv))
        w_1 = ica.Archive_load("cli_cleaned.ar").get_weights()
        d_1 = ica.Archive_load("cli_cleaned.ar").get_data()
        r_1 = ica.Archive_load(res[-1]).get_data()
        ok = (sharded_out == buf1.getvalue() and w_sh.tobytes() == w_1.tobytes()
              and np.array_equal(r_sh, r_1) and np.array_equal(d_sh, d_1))
        rec = {"cli": True, "rank": 0, "backend": a.backend, "world": world, "shape": a.shape,
               "format": a.cli_suffix, "stdout_equal": sharded_out == buf1.getvalue(),
               "weights_equal": w_sh.tobytes() == w_1.tobytes(), "data_equal": bool(np.array_equal(d_sh, d_1)),
               "residual_equal": bool(np.array_equal(r_sh, r_1)), "stdout": sharded_out}
        _emit(a, 0, rec)
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0 and not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
