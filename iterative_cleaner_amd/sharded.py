"""Channel-sharded cleaning of one large archive (config C3).

The reference cleans an archive in one process (iterative_cleaner.py:83-146).
Here the same loop runs as ``world`` channel shards (shards.py), each a
libicgpu shard session; results are bit-identical to one unsharded session.

* ``clean_cube_local``: all shards in this process, one host thread each, on one
  or several devices (in-process group: device-to-device / peer copies).
* ``clean_cube_dist``: this rank's shard under torchrun, exchanging through
  torch.distributed (dist.TorchComm: RCCL over xGMI on "nccl"); the full test /
  weights arrays are all-gathered so every rank returns the same dict.
"""
from __future__ import annotations

import threading

import numpy as np

from . import _native


def _gather_cols(parts, ranges, shape, dtype):
    out = np.empty(shape, dtype)
    for (c0, c1), part in zip(ranges, parts):
        out[:, c0:c1] = part
    return out


def _loop_kwargs(args):
    return dict(max_iter=args.get("max_iter", 5), chanthresh=args.get("chanthresh", 5.0),
                subintthresh=args.get("subintthresh", 5.0),
                pulse_region=args.get("pulse_region", (0, 0, 1)),
                baseline_duty=args.get("baseline_duty", 0.15), fit_mode=args.get("fit_mode", 0),
                data_f64=args.get("data_f64", False), options=args.get("options"),
                input_dedispersed=args.get("input_dedispersed", False))


def clean_cube_local(cube, w0, shift, world, devices=None, want_details=False, fit_tail=None, **args):
    """Clean a (nsub, nchan, nbin) f32 cube as `world` in-process channel shards.
    Returns the ic_run dict with full-archive ``test`` / ``weights`` (and, with
    want_details, ``amp``, ``info``, ``std``, ``mean``, ``ptp``, ``fft``, ``T``)."""
    nsub, nchan, nbin = cube.shape
    devices = list(devices) if devices is not None else [0] * world
    if len(devices) != world:
        raise ValueError("need one device per shard")
    chans, _ = _native.shard_layout(nsub, nchan, world)
    kw = _loop_kwargs(args)
    delay = args.get("delay")
    results = [None] * world
    errors = []
    with _native.ShardGroup(world) as group:
        sessions = [_native.ShardSession(nsub, nchan, nbin, r, world, group=group, device=devices[r],
                                         delay=None if delay is None else np.asarray(delay)[..., chans[r][0]:chans[r][1]],
                                         **kw)
                    for r in range(world)]
        try:
            for r, s in enumerate(sessions):
                c0, c1 = chans[r]
                if fit_tail is not None:
                    s.set_fit_tail(fit_tail)
                s.upload(cube[:, c0:c1], w0[:, c0:c1], np.asarray(shift)[c0:c1])

            def work(r):
                try:
                    s = sessions[r]
                    out = s.run()
                    if want_details and out["n_iter"] > 0:
                        out["amp"], out["info"] = s.fit()
                        out["std"], out["mean"], out["ptp"], out["fft"] = s.diagnostics()
                        out["T"] = s.template()
                    results[r] = out
                except Exception as e:  # noqa: BLE001 - re-raised below
                    errors.append((r, e))

            threads = [threading.Thread(target=work, args=(r,)) for r in range(world)]
            for t in threads:
                t.start()
            for t in threads:
                t.join()
        finally:
            for s in sessions:
                s.close()
    if errors:
        r, e = errors[0]
        raise _native.NativeError("shard %d failed: %s" % (r, e))
    return _merge(results, chans, (nsub, nchan), want_details)


def _merge(results, chans, shape2, want_details):
    first = results[0]
    for r, out in enumerate(results[1:], 1):
        for key in ("loops", "n_iter", "converged"):
            if out[key] != first[key]:
                raise _native.NativeError("shard %d disagrees on %s" % (r, key))
        if not (np.array_equal(out["changed"], first["changed"])
                and np.array_equal(out["nzero"], first["nzero"])):
            raise _native.NativeError("shard %d disagrees on the convergence counters" % r)
    merged = dict(first)
    merged["test"] = _gather_cols([o["test"] for o in results], chans, shape2, np.float64)
    merged["weights"] = _gather_cols([o["weights"] for o in results], chans, shape2, np.float32)
    if want_details and "amp" in first:
        for key, dt in (("amp", np.float64), ("info", np.int32), ("std", np.float64),
                        ("mean", np.float64), ("ptp", np.float32), ("fft", np.float64)):
            merged[key] = _gather_cols([o[key] for o in results], chans, shape2, dt)
        for r, o in enumerate(results[1:], 1):
            if o["T"].tobytes() != first["T"].tobytes():
                raise _native.NativeError("shard %d has a different template" % r)
    return merged


def clean_cube_dist(cube_slice, w0_slice, shift_slice, global_shape, device, group=None,
                    want_residual=False, fail_at=None, **args):
    """This rank's channel shard of one archive under torch.distributed.
    `cube_slice` etc. are the rank's channel range (``_native.shard_layout``);
    returns the merged full-archive dict on every rank (with want_residual, the
    full residual cube on rank 0 only).  ``delay`` (in args): the slice's
    fractional delays (FFT-rotation dedispersion; (nchan_r,) or (nsub, nchan_r))."""
    import torch.distributed as dist

    from .dist import TorchComm
    nsub, nchan, nbin = global_shape
    comm = TorchComm(device, group, fail_at=fail_at)
    world, rank = comm.world, comm.rank
    chans, _ = _native.shard_layout(nsub, nchan, world)
    try:
        with _native.ShardSession(nsub, nchan, nbin, rank, world, comm=comm, device=_device_index(device),
                                  delay=args.get("delay"), **_loop_kwargs(args)) as s:
            if np.ndim(cube_slice) == 4:   # full-pol: pscrunched on the GPU
                s.upload_pols(cube_slice, w0_slice, shift_slice)
            else:
                s.upload(cube_slice, w0_slice, shift_slice)
            out = s.run()
            res = s.residual() if want_residual and out["n_iter"] > 0 else None
    except _native.NativeError:
        comm.abort()          # peers waiting in a collective with this rank must not block
        raise
    return _merge_dist(out, res, chans, (nsub, nchan, nbin), comm, group, want_residual)


def _merge_dist(out, res, chans, shape, comm, group, want_residual):
    """Every rank's (nsub, nchan_r) test / weights slices -> the full arrays on
    every rank, and the residual slices -> the full cube on rank 0, through
    tensor collectives (padded to the widest slice; RCCL on "nccl", host
    tensors on "gloo").  The scalar loop results are checked for agreement."""
    import torch
    import torch.distributed as dist
    nsub, nchan, nbin = shape
    world, rank = comm.world, comm.rank
    dev = comm.device if comm.backend != "gloo" else torch.device("cpu")
    wmax = max(c1 - c0 for c0, c1 in chans)
    nc = chans[rank][1] - chans[rank][0]
    scalars = {k: out[k] for k in ("loops", "n_iter", "converged")}
    scalars.update(changed=list(map(int, out["changed"])), nzero=list(map(int, out["nzero"])),
                   bad_fits=list(map(int, out.get("bad_fits", []))))
    every = [None] * world
    dist.all_gather_object(every, scalars, group=group)
    for r, sc in enumerate(every[1:], 1):
        if sc != every[0]:
            raise _native.NativeError("shard %d disagrees on the loop results: %s vs %s" % (r, sc, every[0]))
    merged = dict(out)

    def gather_cols(a, dtype, to_all=True):
        t = torch.zeros((nsub, wmax) + a.shape[2:], dtype=dtype, device=dev)
        t[:, :nc] = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        if to_all:
            parts = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(parts, t, group=group)
        else:
            parts = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
            dist.gather(t, parts, dst=0, group=group)
            if rank != 0:
                return None
        full = np.empty((nsub, nchan) + a.shape[2:], dtype=t.cpu().numpy().dtype)
        for (c0, c1), part in zip(chans, parts):
            full[:, c0:c1] = part[:, :c1 - c0].cpu().numpy()
        return full

    merged["test"] = gather_cols(out["test"], torch.float64)
    merged["weights"] = gather_cols(out["weights"], torch.float32)
    if want_residual:
        R = gather_cols(res if res is not None else np.zeros((nsub, nc, nbin), np.float32), torch.float32,
                        to_all=False)
        if rank == 0 and merged["n_iter"] > 0:
            merged["residual"] = R
    return merged


def _device_index(device):
    import torch
    d = torch.device(device)
    return d.index if d.index is not None else 0
