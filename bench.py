#!/usr/bin/env python
"""Benchmark: profiles cleaned per second on MI355X (BASELINE.json metric).

A step = one complete surgical-cleaning run (iterative_cleaner.py:83-146:
fit-cube preparation + every loop iteration until the zap mask repeats or
max_iter) over one synthetic archive already resident in HBM.  Default
workload: configs[1] of BASELINE.json, a LOFAR HBA-like archive
360 subint x 3200 chan x 1024 bin, default thresholds, max_iter 5.

Multi-GPU (``torchrun --nproc-per-node N bench.py --gpus N``): the default
workload at N > 1 is configs[2], the large archive C3 = 1024 x 8192 x 1024,
channel-sharded across the N ranks: each rank cleans its
channel slice in a libicgpu shard session that exchanges template roots,
diagnostics rows, row statistics and convergence counters over RCCL/xGMI
(torch.distributed "nccl" through dist.TorchComm); value = C3 profiles x
steps / max-over-ranks time (strong scaling: total work fixed).
``--workload C3`` at N = 1 is the unsharded 1-GPU reference point of that
curve; ``--workload C2`` at N > 1 runs independent replicas (weak scaling).

Prints ONE JSON line on rank 0 (contract in the task statement), including
``roofline`` for the dominant kernel (HIP events on the session stream) and
``cpu_baseline`` (the reference-like NumPy/SciPy loop on a bounded sample).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
F64_PEAK_TOPS = 39.3           # f64 vector ops/s (78.6 TFLOP/s FMA-counted / 2)

WORKLOADS = {
    # name: (nsub, nchan, nbin, seed, rfi_frac)
    "C1": (64, 256, 256, 0, 0.05),
    "C2": (360, 3200, 1024, 1, 0.05),
    "C3": (1024, 8192, 1024, 2, 0.05),
    "C4": (128, 1024, 512, 1000, 0.05),
    "C5": (256, 1024, 4096, 58, 0.30),   # seed 58: the loop runs to max_iter (tools/c5_seed_search.py)
}
BLOCKWISE = {"C3"}   # generated per 256-channel block: any channel shard builds its slice alone


def make_cube_device(nsub, nchan, nbin, seed, rfi, device):
    """SURVEY.md §8(d) synthetic archive generated directly in HBM (torch)."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    f32 = torch.float32
    phase = (torch.arange(nbin, device=device, dtype=torch.float64) + 0.5) / nbin
    pulse = torch.exp(-0.5 * ((phase - 0.3) / 0.02) ** 2)
    shift = (torch.arange(nchan, device=device) % 7).to(torch.int32)
    idx = (torch.arange(nbin, device=device)[None, :] - shift[:, None].long()) % nbin
    pulse_disp = pulse[idx].to(f32)                                     # (nchan, nbin)
    u = torch.rand((2, nsub, nchan), generator=g, device=device, dtype=torch.float64)
    gain = (0.5 * (-torch.log1p(-u[0]) - torch.log1p(-u[1]))).to(f32)  # Gamma(2, 0.5)
    cube = torch.randn((nsub, nchan, nbin), generator=g, device=device, dtype=f32)
    for s0 in range(0, nsub, 32):
        cube[s0:s0 + 32] += gain[s0:s0 + 32, :, None] * pulse_disp[None]
    n_nb = int(round(rfi * nchan))
    if n_nb:
        chans = torch.randperm(nchan, generator=g, device=device)[:n_nb]
        nu = 1.0 + 19.0 * torch.rand(n_nb, generator=g, device=device, dtype=torch.float64)
        amp = 5.0 * torch.randn((nsub, n_nb), generator=g, device=device, dtype=torch.float64)
        wave = torch.sin(2.0 * math.pi * nu[:, None] * phase[None, :])
        cube[:, chans, :] += (amp[:, :, None] * wave[None]).to(f32)
    n_imp = int(round(rfi * nsub))
    if n_imp:
        subs = torch.randperm(nsub, generator=g, device=device)[:n_imp]
        for s in subs.tolist():
            hits = torch.rand((nchan, nbin), generator=g, device=device) < 0.01
            cube[s] += hits.to(f32) * 20.0
    w0 = torch.ones((nsub, nchan), device=device, dtype=f32)
    n_dead = int(round(0.02 * nchan))
    if n_dead:
        w0[:, torch.randperm(nchan, generator=g, device=device)[:n_dead]] = 0.0
    return cube.contiguous(), w0.contiguous(), shift.contiguous()


def make_block_cube_device(nsub, nchan, nbin, seed, rfi, c0, c1, device):
    """Channels [c0, c1) of a SURVEY.md §8(d) synthetic archive whose every
    256-channel block has its own generator (seed, block): the cube is the same
    whichever way it is sharded.  Impulsive-RFI subints are drawn once per
    archive.  Returns (cube [nsub][c1-c0][nbin], w0, shift) on `device`."""
    import torch
    f32, f64 = torch.float32, torch.float64
    phase = (torch.arange(nbin, device=device, dtype=f64) + 0.5) / nbin
    pulse = torch.exp(-0.5 * ((phase - 0.3) / 0.02) ** 2)
    g0 = torch.Generator(device=device)
    g0.manual_seed(seed * 1000003 + 999983)
    n_imp = int(round(rfi * nsub))
    imp = torch.randperm(nsub, generator=g0, device=device)[:n_imp]
    cube = torch.empty((nsub, c1 - c0, nbin), device=device, dtype=f32)
    w0 = torch.ones((nsub, c1 - c0), device=device, dtype=f32)
    shift = (torch.arange(c0, c1, device=device) % 7).to(torch.int32)
    for b0 in range(c0 - c0 % 256, c1, 256):
        lo, hi = max(b0, c0), min(b0 + 256, nchan, c1)
        nb = min(b0 + 256, nchan) - b0
        g = torch.Generator(device=device)
        g.manual_seed(seed * 1000003 + b0 // 256)
        sh = (torch.arange(b0, b0 + nb, device=device) % 7).long()
        idx = (torch.arange(nbin, device=device)[None, :] - sh[:, None]) % nbin
        u = torch.rand((2, nsub, nb), generator=g, device=device, dtype=f64)
        gain = (0.5 * (-torch.log1p(-u[0]) - torch.log1p(-u[1]))).to(f32)
        blk = torch.randn((nsub, nb, nbin), generator=g, device=device, dtype=f32)
        blk += gain[:, :, None] * pulse[idx].to(f32)[None]
        nbm = torch.rand(nb, generator=g, device=device) < rfi
        nu = 1.0 + 19.0 * torch.rand(nb, generator=g, device=device, dtype=f64)
        amp = 5.0 * torch.randn((nsub, nb), generator=g, device=device, dtype=f64)
        wave = torch.sin(2.0 * math.pi * nu[:, None] * phase[None, :])
        blk += torch.where(nbm[None, :, None], amp[:, :, None] * wave[None], 0.0).to(f32)
        if n_imp:
            hits = torch.rand((n_imp, nb, nbin), generator=g, device=device) < 0.01
            blk[imp] += hits.to(f32) * 20.0
        dead = torch.rand(nb, generator=g, device=device) < 0.02
        cube[:, lo - c0:hi - c0] = blk[:, lo - b0:hi - b0]
        w0[:, lo - c0:hi - c0] = torch.where(dead[lo - b0:hi - b0], 0.0, 1.0)[None].to(f32)
    return cube.contiguous(), w0.contiguous(), shift.contiguous()


def s8d_bytes(name, nsub, nchan, nbin, launches, iterations, steps):
    """SURVEY.md §8(d) algorithmic bytes of a kernel over the timed region: the
    cube is read once per iteration by the template stage (k_chan_partials) and
    once by the fit + diagnostics stage (k_fit_pass + k_diag together in the
    exact mode, k_diag alone in the closed-form mode); the 4 f64 diagnostics
    are written and read once (64 B per profile).  Re-reads an implementation
    chooses (lmdif's 5.5 sweeps per profile) are NOT algorithmic.
    Fractional dedispersion (k_rotate): the residual's dededispersion
    (iterative_cleaner.py:104) reads and writes the cube once per iteration,
    8N; the template's and the fit cube's rotations (:91, :100) are carried
    between iterations here, so they are not counted."""
    P = nsub * nchan
    N = P * nbin
    per_iter = {"k_chan_partials": 4 * N, "k_fit_pass": 4 * N, "k_diag": 4 * N + 32 * P,
                "k_linestats": 16 * P, "k_combine": 16 * P, "k_rotate": 8 * N}
    if name not in per_iter:
        return None
    return per_iter[name] * iterations * steps


def algorithmic_bytes(name, nsub, nchan, nbin, launches, run, steps, exact=True, fft=False):
    """Bytes a kernel's launches actually move, summed over the timed region
    (kernel table) - the implementation's own traffic model, not
    §8(d)'s.  `run`: one clean's counts, {"n_iter", "changed" (per iteration),
    "fit_profile_sweeps", "fit_tail_sweeps", "window_moves"} (ic_run /
    ic_get_run_stats); every clean of the timed region is the same work.
      k_fit_pass       every profile-sweep reads its 4*nbin-byte profile once
                       (k_fit_tail: its own sweeps, the same);
      k_fit_state      ~2 x 188 B of lmdif state per profile of a round (read
                       and written: 18 f64 + 4 i32 fields, the sweep's 3 f64
                       outputs and the f32 first sample; the rounds' inputs are
                       the sweeps of k_fit_pass);
      k_chan_partials  (every template-stage launch, k_chan_delta included)
                       prepare's window pass reads the cube (4N); iteration 1's
                       pass reads it and writes the fit cube (8N exact, 4N
                       closed); from iteration 2 on k_chan_delta reads the rows
                       of the profiles whose weight changed in the iteration
                       before, and the flagged pass the subints whose baseline
                       window moved; plus the super-block partials written;
                       FFT dedispersion (fft): the passes read the rotated cubes
                       (rot(raw) for the window totals, the rotated rows for the
                       fscrunch sums) and write no fit cube (k_rotate does); the
                       delta reads a changed channel's row from both;
      k_base           the window samples of every profile (prepare) and of
                       the subints whose window moved (later iterations);
      k_diag           one full pass per iteration whatever the launches (the
                       fork splits it in two): the raw cube + 44 B per profile."""
    P = nsub * nchan
    N = P * nbin
    nsb = (nchan + 255) // 256
    width = max(1, int(0.15 * nbin))
    n_iter = run["n_iter"]
    if name == "k_fit_pass":
        return 4 * nbin * run["fit_profile_sweeps"] * steps
    if name == "k_fit_tail":
        return 4 * nbin * run["fit_tail_sweeps"] * steps
    if name == "k_fit_state":
        return 2 * 188 * run["fit_profile_sweeps"] * steps
    if name == "k_chan_partials":
        changed = sum(int(c) for c in run["changed"][:max(0, n_iter - 1)])
        per_run = (4 * N + (8 * N if exact and not fft else 4 * N) + (8 if fft else 4) * nbin * changed
                   + 4 * nchan * nbin * run["window_moves"] + 16 * nsub * nsb * nbin * n_iter)
        return per_run * steps
    if name == "k_base":
        return 4 * width * (P + nchan * run["window_moves"]) * steps
    if name == "k_diag":
        return (4 * N + 44 * P) * n_iter * steps
    if name == "k_rotate":
        # 8 B per sample rotated (f32 in, f32 out): preparation's rot(raw) and
        # fit cube, every iteration's residual, and the carried template rows
        # of the subints whose baseline window moved
        return (8 * N * (2 + n_iter) + 8 * nchan * nbin * run["window_moves"]) * steps
    per_launch = {"k_linestats": 2 * 4 * 8 * P, "k_combine": 4 * 8 * P + 2 * 4 * P}
    if name in per_launch:
        return per_launch[name] * launches
    return None


CACHE_RESIDENT_BYTES = 256 * 2 ** 20   # the Infinity Cache (MI355X_MICROARCH.md): a cube this small is served on-die


def check_kernel_rates(per_kernel, cube_bytes):
    """Per-kernel byte rates of the traffic model must stay under the HBM peak
    for a cube that cannot sit in the Infinity Cache: a rate above it means the
    model charges bytes the kernel does not move (round 3: k_chan_partials
    charged a full cube per launch after the incremental stage had cut most of
    them).  Returns the offending kernels; main() refuses to print such a line."""
    bad = {k: v["sweep_gbs"] for k, v in per_kernel.items() if v.get("sweep_gbs") and v["sweep_gbs"] > HBM_PEAK_GBS}
    if cube_bytes <= CACHE_RESIDENT_BYTES:
        return {}, bad   # on-die re-reads may legitimately beat HBM
    return bad, {}


def pmc_traffic(workload, kernel):
    """HBM bytes per launch of ``kernel`` from the committed rocprofv3 PMC
    summary (tools/pmc_traffic.py: separate FETCH_SIZE / WRITE_SIZE passes of
    this bench at --steps 1, FETCH_SIZE x2 for gfx950), only when it was
    measured on the HIP sources being timed (source_sha)."""
    import glob
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from pmc_traffic import source_sha
    sha = source_sha()
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*pmc_traffic*.json")), reverse=True):
        with open(path) as f:
            rec = json.load(f)
        if rec.get("workload") == workload and rec.get("source_sha") == sha and kernel in rec["kernels"]:
            return rec["kernels"][kernel]["traffic_bytes_per_launch"], os.path.basename(path)
    return None, None


VALU_PEAK_G = 614.4   # wave64 VALU instructions/s (G): 256 CUs x 4 SIMDs x 2.4 GHz / 4 cycles each


def pmc_valu(workload):
    """SQ_INSTS_VALU per launch for every kernel from the committed SQ pass
    (tools/pmc_valu.sh), only when it was measured on the HIP sources being
    timed (source_sha).  The kernels of the exact fit and the diagnostics are
    f64-VALU-bound, not HBM-bound: this is the roof they are priced against."""
    import glob
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from pmc_traffic import source_sha
    sha = source_sha()
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*pmc_valu*.json")), reverse=True):
        with open(path) as f:
            rec = json.load(f)
        if rec.get("workload") == workload and rec.get("source_sha") == sha:
            return rec["kernels"], os.path.basename(path)
    return None, None


def cpu_baseline(nchan, nbin, seed, rfi, budget_s):
    """Reference-like loop (per-profile scipy leastsq + numpy.ma), one thread,
    on the first subints of the workload shape: a 2-subint probe sizes the
    sample to 1.3 * ``budget_s`` by linear extrapolation, which lands at about
    10-20 s of CPU work in practice (the probe's subints need more loops than
    the whole sample's average)."""
    from threadpoolctl import threadpool_limits

    from iterative_cleaner_amd import archive as ica
    from iterative_cleaner_amd import synth
    from oracle import reference_like
    with threadpool_limits(1):
        data, w0, shift = synth.make_cube(2, nchan, nbin, seed, rfi)
        ar = ica.Archive(data, w0, shift)
        ar.pscrunch()
        t0 = time.perf_counter()
        reference_like.clean_loop(ar, 5, 5, 5, [0, 0, 1])
        probe = time.perf_counter() - t0
    nsub = int(max(2, min(64, 2 * 1.3 * budget_s / max(probe, 1e-3))))
    data, w0, shift = synth.make_cube(nsub, nchan, nbin, seed, rfi)
    ar = ica.Archive(data, w0, shift)
    ar.pscrunch()
    with threadpool_limits(1):
        t0 = time.perf_counter()
        _, _, loops = reference_like.clean_loop(ar, 5, 5, 5, [0, 0, 1])
        dt = time.perf_counter() - t0
    P = nsub * nchan
    return {"value": P / dt, "unit": "profiles/s", "cores": 1, "kind": "port",
            "host_cpus": os.cpu_count(), "cpu_model": cpu_model(),
            "sample": "%dx%dx%d subset of the workload shape, full loop to convergence "
                      "(%d loops) in %.1f s, single thread (oracle/reference_like.py); profiles/s of the "
                      "sample, i.e. extrapolated linearly per profile to the full archive"
                      % (nsub, nchan, nbin, loops, dt)}


def cpu_model() -> str:
    """The host CPU model (lscpu's "Model name", read from /proc/cpuinfo)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.lower().startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def fast_mode_summary(_native, cube, w0, shift, shape, device, steps, torch, delay=None):
    """fit_mode 1 (closed-form amplitude fused with the diagnostics) on the same
    archive: profiles/s, the loop's SURVEY §8(d) HBM fraction, and (filled in by
    the caller) the zap-mask flips against the exact mode.  Not the reference's
    arithmetic; the headline value stays the exact mode's."""
    nsub, nchan, nbin = shape
    with _native.GpuSession(nsub, nchan, nbin, max_iter=5, device=device, fit_mode=_native.FIT_CLOSED,
                            delay=delay) as s:
        s.upload_device(cube.data_ptr(), w0.data_ptr(), shift.data_ptr())
        s.run(fetch=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            out = s.run(fetch=False)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        weights = s.run()["weights"]
    P = nsub * nchan
    loop_gbs = (8 * P * nbin + 64 * P) * out["n_iter"] / dt / 1e9
    return {"fit_mode": "closed", "value": round(P / dt, 1), "unit": "profiles/s", "ms_per_step": round(1e3 * dt, 3),
            "loops": out["loops"], "loop_hbm_gbs": round(loop_gbs, 1),
            "loop_hbm_frac": round(loop_gbs / HBM_PEAK_GBS, 4), "weights": weights,
            "note": "closed-form amplitude sum(T*p)/sum(T*T) (IC_FIT_CLOSED): the north star's HBM-bound fast "
                    "mode, not the reference's leastsq arithmetic"}


EXCHANGE_KINDS = ("allgather", "alltoallv", "allreduce", "native")


def per_rank_report(ktimes, exch, rank, world, dev, wall_ms):
    """One clean's compute and exchange time on every rank (channel shards),
    gathered to every rank as a tensor: [{rank, world_size_seen (the process
    group's), wall_ms (the clean, host clock), compute_ms (wall_ms minus the
    exchanges), kernel_ms (the shard kernels' summed durations: above
    compute_ms when kernels overlap, e.g. the forked diagnostics beside the
    fit's late rounds), exchange_ms / calls / MB per collective type}], so that
    a multi-GPU line shows where each rank's time went."""
    import torch
    import torch.distributed as dist
    ws = dist.get_world_size() if dist.is_initialized() else 1
    kernel = sum(v["ms"] for k, v in ktimes.items() if k.startswith("k_"))
    exch_ms = sum(exch.get(kind, {"ms": 0.0})["ms"] for kind in EXCHANGE_KINDS)
    row = [float(rank), float(ws), wall_ms - exch_ms, wall_ms, kernel]
    for kind in EXCHANGE_KINDS:
        e = exch.get(kind, {"ms": 0.0, "calls": 0, "bytes": 0})
        row += [e["ms"], float(e["calls"]), e["bytes"] / 1e6]
    head = 5
    t = torch.tensor(row, dtype=torch.float64, device=dev if dist.get_backend() != "gloo" else "cpu")
    rows = [t] if world == 1 else [torch.empty_like(t) for _ in range(world)]
    if world > 1:
        dist.all_gather(rows, t)
    out = []
    for r in rows:
        v = r.cpu().tolist()
        rec = {"rank": int(v[0]), "world_size_seen": int(v[1]), "compute_ms": round(v[2], 3),
               "wall_ms": round(v[3], 3), "kernel_ms": round(v[4], 3), "exchange": {}}
        for i, kind in enumerate(EXCHANGE_KINDS):
            ms, calls, mb = v[head + 3 * i: head + 3 + 3 * i]
            rec["exchange"][kind] = {"ms": round(ms, 3), "calls": int(calls), "MB": round(mb, 3)}
        out.append(rec)
    return out


def batch_main(a, workload, rank, world, local, dev):
    """C4: every rank cleans `--batch` archives per step from page-locked host
    memory through the batch pipeline (iterative_cleaner_amd/batch.py); three
    distinct synthetic archives per rank are cycled.  value = all ranks'
    profiles / max-over-ranks time, H2D copies included."""
    import torch
    import torch.distributed as dist

    from iterative_cleaner_amd import _native, batch, synth
    from iterative_cleaner_amd.dist import max_over_ranks
    nsub, nchan, nbin, seed, rfi = WORKLOADS[workload]
    P = nsub * nchan
    pinned, items = [], []
    for k in range(3):
        data, w0, shift = synth.make_cube(nsub, nchan, nbin, seed + 3 * rank + k, rfi)
        trio = (_native.PinnedArray((nsub, nchan, nbin)), _native.PinnedArray((nsub, nchan)),
                _native.PinnedArray((nchan,), np.int32))
        trio[0].array[:] = data[:, 0]
        trio[1].array[:] = w0
        trio[2].array[:] = shift
        pinned.append(trio)
        items.append(tuple(p.array for p in trio))
    sessions = [_native.GpuSession(nsub, nchan, nbin, max_iter=5, device=local) for _ in range(a.lanes)]
    for sess in sessions:
        for opt in a.option:
            name, _, value = opt.partition("=")
            sess.set_option(name, int(value))
    stream = [items[k % 3] for k in range(a.batch)]
    for _ in range(a.warmup):
        for _out in batch.run_lanes(sessions, stream, fetch=False):
            pass

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    loops = []
    for _ in range(a.steps):
        for out in batch.run_lanes(sessions, stream, fetch=False):
            loops.append(out["loops"])
    t1 = time.perf_counter()
    barrier()
    elapsed = max_over_ranks(t1 - t0, device=dev)
    for sess in sessions:
        sess.close()
    if rank == 0:
        n_arch = a.steps * a.batch * world
        bytes_arch = 4 * P * nbin
        rec = {
            "metric": "profiles cleaned/sec (whole node)", "value": round(n_arch * P / elapsed, 1),
            "unit": "profiles/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(1000.0 * elapsed / a.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": "%s batch: %d archives of %dx%dx%d per GPU per step from page-locked "
                                   "host memory, H2D overlapped with cleaning (included), %d concurrent "
                                   "session(s) per GPU" % (workload, a.batch, nsub, nchan, nbin, a.lanes),
                       "archives_per_s": round(n_arch / elapsed, 2),
                       "ms_per_archive": round(1000.0 * elapsed / (a.steps * a.batch), 3),
                       "h2d_gbs_per_gpu": round(bytes_arch * a.steps * a.batch / elapsed / 1e9, 1),
                       "loops": sorted(set(loops)), "parallelism": "batch, one archive list per rank"},
        }
        print(json.dumps(rec))
    for trio in pinned:
        for p in trio:
            p.close()
    if dist.is_initialized():
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default=None, choices=sorted(WORKLOADS),
                    help="default: C2 on one GPU, C3 channel-sharded on several")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--untimed-kernels", action="store_true",
                    help="A/B only: no per-kernel HIP events in the timed region (the line then has no roofline)")
    ap.add_argument("--cpu-budget", type=float, default=30.0)
    ap.add_argument("--kernel-report", action="store_true", help="print per-kernel times to stderr")
    ap.add_argument("--batch", type=int, default=0,
                    help="batch mode (config C4): clean this many archives per step per GPU from "
                         "page-locked host memory, each upload overlapped with the previous cleaning "
                         "(H2D included in the time)")
    ap.add_argument("--lanes", type=int, default=1,
                    help="batch mode: concurrent sessions per GPU (each on its own HIP streams)")
    ap.add_argument("--sharded", action="store_true",
                    help="use the channel-shard session even on one GPU (one-rank RCCL group)")
    ap.add_argument("--fit-mode", choices=("exact", "closed"), default="exact",
                    help="exact: scipy leastsq emulated bit for bit (the reference's arithmetic, default); "
                         "closed: the closed-form amplitude fused with the diagnostics (fit_mode 1, fast mode; "
                         "also reports the zap-mask flips against the exact mode on the same archive)")
    ap.add_argument("--no-fast-summary", action="store_true",
                    help="exact mode at N=1: skip the closed-form (fit_mode 1) summary added to the line")
    ap.add_argument("--no-flip-check", action="store_true",
                    help="closed mode: skip the (untimed) exact run that counts zap-mask flips "
                         "(profiling passes, whose kernel tallies it would mix in)")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="a session schedule option (_native.OPTIONS; same bits under every setting), repeatable")
    ap.add_argument("--dedisp", choices=("shift", "fft", "fft_pp"), default="shift",
                    help="shift: integer dedispersion shifts (default); fft: fractional delays, dedispersed by "
                         "psrchive's FFT phase rotation (dedisp_mode IC_DEDISP_FFT); fft_pp: the same with one "
                         "delay per profile (psrchive's per-Integration folding period, ic_set_delays2)")
    a = ap.parse_args()

    import torch
    import torch.distributed as dist

    from iterative_cleaner_amd import _native
    from iterative_cleaner_amd.dist import TorchComm, max_over_ranks, rank_world

    fit_mode = _native.FIT_CLOSED if a.fit_mode == "closed" else _native.FIT_EXACT
    rank, world, local = rank_world()
    if world != a.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (a.gpus, world))
    workload = a.workload or ("C2" if world == 1 else "C3")
    sharded = (world > 1 and workload in BLOCKWISE) or a.sharded
    # IC_BENCH_BACKEND=gloo rehearses an N-rank run on fewer GPUs (ranks share
    # devices, exchanges staged through the host); the measurement is "nccl" (RCCL)
    backend = os.environ.get("IC_BENCH_BACKEND", "nccl")
    # channel shards over "nccl" use the library's native RCCL transport;
    # IC_BENCH_TRANSPORT=torch keeps the torch.distributed callbacks (A/B)
    # IC_BENCH_RCCL_LIBRARY=path (rehearsal only): the native transport loads that
    # librccl instead (ic_rccl_set_library), e.g. the test stub
    # tests/stub_rccl/libstubrccl.so, which lets N ranks share one GPU under
    # IC_BENCH_BACKEND=gloo and still run the exact code path of the N-GPU line
    rccl_lib = os.environ.get("IC_BENCH_RCCL_LIBRARY")
    if rccl_lib:
        _native.rccl_set_library(rccl_lib)
    native_rccl = (backend == "nccl" or bool(rccl_lib)) and os.environ.get("IC_BENCH_TRANSPORT", "rccl") == "rccl"
    native_error, transport_note = None, None
    gpu = local % max(1, torch.cuda.device_count()) if backend == "gloo" else local
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    elif sharded:
        dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=dev)
    local = gpu   # the device the sessions below run on

    nsub, nchan, nbin, seed, rfi = WORKLOADS[workload]
    P_total = nsub * nchan
    if a.batch:
        return batch_main(a, workload, rank, world, local, dev)
    delay = None
    if a.dedisp == "fft":
        from iterative_cleaner_amd import synth
        delay = synth.fractional_delays(np.arange(nchan) % 7, nbin)   # the generators' integer shifts + fractions
    elif a.dedisp == "fft_pp":
        from iterative_cleaner_amd import synth
        delay = synth.per_profile_delays(np.arange(nchan) % 7, nbin, nsub)
    if sharded:
        chans, _ = _native.shard_layout(nsub, nchan, world)
        c0, c1 = chans[rank]
        cube, w0, shift = make_block_cube_device(nsub, nchan, nbin, seed, rfi, c0, c1, dev)
        comm = TorchComm(dev)
        kw = dict(max_iter=5, device=local, fit_mode=fit_mode, delay=None if delay is None else delay[..., c0:c1])
        sess = None
        if native_rccl:
            # the library's own RCCL communicator: every exchange issued from C++
            # on the session stream (rank 0's unique id shared once).  Every rank
            # agrees on the transport: if any rank could not create its native
            # communicator (e.g. librccl not loadable), all fall back to the
            # torch.distributed callbacks, and the line says so.
            from iterative_cleaner_amd.dist import share_rccl_id
            try:
                sess = _native.ShardSession(nsub, nchan, nbin, rank, world, rccl_id=share_rccl_id(), **kw)
            except _native.NativeError as e:
                native_error = str(e)[:200]
            ok = torch.tensor([1 if sess is not None else 0], dtype=torch.int32,
                              device=dev if backend == "nccl" else "cpu")
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if int(ok.item()) == 0:
                if sess is not None:
                    sess.close()
                    sess = None
                native_rccl = False
                transport_note = "native RCCL unavailable on some rank (%s): torch.distributed callbacks" % (
                    native_error or "see the other ranks")
        if sess is None:
            sess = _native.ShardSession(nsub, nchan, nbin, rank, world, comm=comm, **kw)
        per_rank_P = nsub * (c1 - c0)
    else:
        if workload in BLOCKWISE:
            cube, w0, shift = make_block_cube_device(nsub, nchan, nbin, seed, rfi, 0, nchan, dev)
        else:
            cube, w0, shift = make_cube_device(nsub, nchan, nbin, seed + 7919 * rank, rfi, dev)
        sess = _native.GpuSession(nsub, nchan, nbin, max_iter=5, device=local, fit_mode=fit_mode, delay=delay)
        for opt in a.option:
            name, _, value = opt.partition("=")
            sess.set_option(name, int(value))
        per_rank_P = P_total
        if world > 1:
            P_total = P_total * world          # replicas: every rank cleans its own archive
    torch.cuda.synchronize()
    sess.upload_device(cube.data_ptr(), w0.data_ptr(), shift.data_ptr())
    fast = None
    if fit_mode == _native.FIT_EXACT and not sharded and world == 1 and not a.no_fast_summary:
        # the north star's fast mode on the same archive, beside the exact line
        fast = fast_mode_summary(_native, cube, w0, shift, (nsub, nchan, nbin), local, a.steps, torch, delay)
    flips = None
    if fit_mode == _native.FIT_CLOSED and not sharded and not a.no_flip_check:
        # zap-mask flips of the fast mode against the exact fit on this archive (untimed)
        fres = sess.run()
        with _native.GpuSession(nsub, nchan, nbin, max_iter=5, device=local, delay=delay) as ex:
            ex.upload_device(cube.data_ptr(), w0.data_ptr(), shift.data_ptr())
            exact = ex.run()
        flips = {"profiles": int(np.count_nonzero(fres["weights"] != exact["weights"])),
                 "loops_fast": fres["loops"], "loops_exact": exact["loops"]}
    del cube
    torch.cuda.empty_cache()
    for _ in range(a.warmup):
        sess.run(fetch=False)
    # Per-kernel breakdown: one run with every kernel timed, outside the timed
    # region (two HIP events per launch cost ~1 ms per C2 clean).  The timed
    # region then times only the dominant kernel, whose average launch the
    # roofline prices.
    ktimes_all = {}
    dom = None
    rank_report = None
    if not a.untimed_kernels:
        sess.set_timing(True)
        if sharded:
            comm.timing = True
        torch.cuda.synchronize()
        tb0 = time.perf_counter()
        sess.run(fetch=False)
        torch.cuda.synchronize()
        wall_ms = 1000.0 * (time.perf_counter() - tb0)
        ktimes_all = sess.kernel_times()
        if sharded:
            comm.timing = False
            exch = comm.exchange_report()
            if native_rccl:   # the session's own exchange timing (one bucket: RCCL calls from C++)
                e = ktimes_all.get("exchange", {"ms": 0.0, "launches": 0})
                exch = {"native": {"ms": e["ms"], "calls": e["launches"], "bytes": 0}}
            rank_report = per_rank_report(ktimes_all, exch, rank, world, dev, wall_ms)
        kk = {k: v for k, v in ktimes_all.items() if k.startswith("k_") and v["launches"]}
        dom = max(kk, key=lambda k: kk[k]["ms"])
        sess.set_timing(True, only=dom)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    loops = []
    for _ in range(a.steps):
        out = sess.run(fetch=False)
        loops.append(out["loops"])
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    elapsed = max_over_ranks(t1 - t0, device=dev)
    ktimes_dom = sess.kernel_times() if dom else {}
    # the breakdown run scaled to the timed steps; the dominant kernel's entry
    # is the timed region's own measurement
    ktimes = {k: dict(ms=v["ms"] * a.steps, launches=v["launches"] * a.steps) for k, v in ktimes_all.items()}
    if dom:
        ktimes[dom] = ktimes_dom[dom]
    stats = sess.run_stats()
    n_iter = out["n_iter"]
    run_counts = dict(stats, n_iter=n_iter, changed=[int(c) for c in out["changed"]])
    exact_weights = sess.run()["weights"] if fast is not None else None
    sess.close()

    if rank == 0 and a.untimed_kernels:
        print(json.dumps({"metric": "profiles cleaned/sec (whole node)", "value": round(a.steps * P_total / elapsed, 1),
                          "ms_per_step": round(1000.0 * elapsed / a.steps, 3), "untimed_kernels": True}))
        return
    if rank == 0:
        lnchan = sess.shape[1]                 # this rank's channels (kernel byte counts)
        ms_step = 1000.0 * elapsed / a.steps
        value = a.steps * P_total / elapsed
        kernels = {k: v for k, v in ktimes.items() if k.startswith("k_")}
        total_k = sum(v["ms"] for v in kernels.values())
        dk = kernels[dom]
        avg_s = dk["ms"] / 1000.0 / max(1, dk["launches"])
        # implementation bytes (every sweep the kernel makes) and SURVEY §8(d) bytes
        exact_mode = fit_mode == _native.FIT_EXACT
        total_bytes = algorithmic_bytes(dom, nsub, lnchan, nbin, dk["launches"], run_counts, a.steps, exact_mode,
                                        delay is not None)
        sweep_launch = total_bytes / max(1, dk["launches"]) if total_bytes else None
        s8d_total = s8d_bytes(dom, nsub, lnchan, nbin, dk["launches"], n_iter, a.steps)
        s8d_launch = s8d_total / max(1, dk["launches"]) if s8d_total else None
        hbm_s8d = s8d_launch / avg_s / 1e9 if s8d_launch else None
        sweep_gbs = sweep_launch / avg_s / 1e9 if sweep_launch else None
        per_kernel = {}
        for kname, kv in ktimes.items():
            if kv["launches"] == 0:
                continue
            tb = algorithmic_bytes(kname, nsub, lnchan, nbin, kv["launches"], run_counts, a.steps, exact_mode,
                                   delay is not None)
            pk = {"ms_per_step": round(kv["ms"] / a.steps, 3), "launches_per_step": kv["launches"] // a.steps,
                  "sweep_gbs": round(tb / (kv["ms"] / 1000.0) / 1e9, 1) if tb else None}
            sb = s8d_bytes(kname, nsub, lnchan, nbin, kv["launches"], n_iter, a.steps)
            if sb:
                pk["s8d_gbs"] = round(sb / (kv["ms"] / 1000.0) / 1e9, 1)
            per_kernel[kname] = pk
        wl_key = workload if not sharded else "%s/%d" % (workload, world)
        if fit_mode == _native.FIT_CLOSED:
            wl_key += "/closed"
        if delay is not None:
            wl_key += "/" + a.dedisp
        traffic, src = pmc_traffic(wl_key, dom)
        valu, vsrc = pmc_valu(wl_key)
        hbm = {"achieved": round(hbm_s8d, 1) if hbm_s8d else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "frac": round(hbm_s8d / HBM_PEAK_GBS, 4) if hbm_s8d else None,
               "algorithmic_bytes_per_launch": int(s8d_launch) if s8d_launch else None,
               "definition": "SURVEY §8(d) bytes: one 4N cube read per iteration for the fit (+ diagnostics) "
                             "and one for the template, divided over the kernel's launches"}
        roof = {"bound": "hbm", "kernel": dom, "achieved": hbm["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": hbm["frac"], "traffic": traffic,
                "traffic_source": src if traffic else "no PMC summary for these HIP sources",
                "avg_launch_ms": round(1000 * avg_s, 3), "kernel_share": round(dk["ms"] / total_k, 3),
                "hbm_frac_s8d": hbm["frac"], "hbm_s8d": hbm,
                "sweep_bytes": {"per_launch": int(sweep_launch) if sweep_launch else None,
                                "gbs": round(sweep_gbs, 1) if sweep_gbs else None,
                                "definition": "every data sweep the kernel makes (lmdif re-sweeps included)"}}
        if valu:
            for kname, pk in per_kernel.items():
                v = valu.get(kname)
                kv = ktimes[kname]
                if v and v["launches"] and kv["launches"]:
                    g = v["valu_insts_per_launch"] / (kv["ms"] / kv["launches"] / 1000.0) / 1e9
                    pk["valu_frac"] = round(g / VALU_PEAK_G, 3)
            v = valu.get(dom)
            if v:
                g = v["valu_insts_per_launch"] / avg_s / 1e9
                roof["valu"] = {"achieved": round(g, 1), "peak": VALU_PEAK_G, "unit": "G wave64 VALU inst/s",
                                "frac": round(g / VALU_PEAK_G, 4), "insts_per_launch": v["valu_insts_per_launch"],
                                "f64_share": v["f64_share_of_valu"], "source": vsrc}
        if traffic:
            # measured HBM bytes (PMC) per launch over the launch time: what the
            # kernel actually moves, re-sweeps and refetches included
            tg = traffic / avg_s / 1e9
            roof["traffic_gbs"] = round(tg, 1)
            roof["traffic_frac"] = round(tg / HBM_PEAK_GBS, 4)
        # the roof that binds is the larger measured fraction: PMC traffic
        # against HBM peak, or VALU issue against its peak
        vf = roof.get("valu", {}).get("frac")
        if vf is not None and vf > roof.get("traffic_frac", 0.0):
            vv = roof["valu"]
            roof.update({"bound": "valu", "achieved": vv["achieved"], "peak": vv["peak"], "unit": vv["unit"],
                         "frac": vv["frac"]})
            roof["bound_note"] = ("VALU issue (%.2f of peak) exceeds measured HBM traffic (%s of peak); the HBM "
                                  "fraction in SURVEY §8(d) bytes is hbm_frac_s8d" % (vf, roof.get("traffic_frac")))
        elif "traffic_frac" in roof:
            roof["bound_note"] = ("measured HBM traffic %.2f of peak (re-sweeps included); frac/achieved use "
                                  "SURVEY §8(d) algorithmic bytes" % roof["traffic_frac"])
        roof["per_kernel"] = per_kernel
        over, resident = check_kernel_rates(per_kernel, 4 * nsub * lnchan * nbin)
        if over:
            raise SystemExit("bench.py: per-kernel rates above the HBM peak (%s GB/s) on a %d-MB cube: the byte "
                             "model is wrong: %s" % (HBM_PEAK_GBS, 4 * nsub * lnchan * nbin // 2 ** 20, over))
        if resident:
            roof["cache_resident_above_hbm_peak"] = resident
        roof["timing"] = ("%s: HIP events on the session stream over the timed region (only this kernel timed "
                          "there); per_kernel: one extra run with every kernel timed, scaled to the steps" % dom)
        iter_bytes = 8 * per_rank_P * nbin + 64 * per_rank_P    # SURVEY §8(d) B_iter, one GPU's share
        loop_gbs = iter_bytes * n_iter / (elapsed / a.steps) / 1e9
        roof["loop_hbm_frac"] = round(loop_gbs / HBM_PEAK_GBS, 4)
        if sharded:
            parallelism = "channel-sharded x%d (RCCL per iteration: 3 all-to-alls to row owners, " \
                          "3 all-gathers of owner results, 1 all-reduce; %s)" % (
                              world, "native RCCL communicator, collectives issued from C++" if native_rccl
                              else (transport_note or "torch.distributed callbacks"))
            if rccl_lib:
                parallelism += " [rehearsal: librccl = %s, process group %s]" % (os.path.basename(rccl_lib), backend)
        else:
            parallelism = "replicas" if world > 1 else "single"
        rec = {
            "metric": "profiles cleaned/sec (whole node)", "value": round(value, 1),
            "unit": "profiles/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(ms_step, 3), "higher_is_better": True,
            "scaling": "strong" if sharded else "weak",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": "%s %dx%dx%d (nsub x nchan x nbin), max_iter 5, thresholds 5/5, %s"
                                   % (workload, nsub, nchan, nbin,
                                      "exact leastsq fit" if fit_mode == _native.FIT_EXACT else
                                      "closed-form fit (fit_mode 1: fast mode, not the reference's arithmetic)")
                                   + (", fractional dedispersion (FFT phase rotation%s)"
                                      % (", per-profile delays" if a.dedisp == "fft_pp" else "")
                                      if delay is not None else ""),
                       "fit_mode": a.fit_mode, "dedisp": a.dedisp,
                       "profiles_per_archive": nsub * nchan, "loops": loops[-1], "iterations": n_iter,
                       "fit_rounds": stats["fit_rounds"],
                       "fit_sweeps_per_profile": round((stats["fit_profile_sweeps"] + stats["fit_tail_sweeps"])
                                                       / per_rank_P / max(1, n_iter), 2),
                       "fit_tail_sweeps": stats["fit_tail_sweeps"] // max(1, n_iter),
                       "options": dict(opt.partition("=")[::2] for opt in a.option) or None,
                       "near_threshold_profiles": stats["near_threshold"],
                       "parallelism": parallelism,
                       "loop_hbm_gbs_per_gpu": round(loop_gbs, 1),
                       "loop_hbm_frac": round(loop_gbs / HBM_PEAK_GBS, 4)},
            "roofline": roof,
        }
        if flips is not None:
            rec["config"]["mask_flips_vs_exact"] = flips
        if fast is not None:
            fast["mask_flips_vs_exact"] = int(np.count_nonzero(fast.pop("weights") != exact_weights))
            rec["fast_mode"] = fast
        if "exchange" in ktimes and ktimes["exchange"]["launches"]:
            rec["config"]["exchange_ms_per_step"] = round(ktimes["exchange"]["ms"] / a.steps, 3)
        if rank_report is not None:
            rec["config"]["per_rank"] = rank_report
        if world == 1 and not a.no_cpu_baseline:
            try:
                rec["cpu_baseline"] = cpu_baseline(nchan, nbin, seed, rfi, a.cpu_budget)
            except Exception as e:  # pragma: no cover
                rec["cpu_baseline"] = {"value": None, "error": repr(e)}
        if a.kernel_report:
            for k, v in sorted(ktimes.items(), key=lambda kv: -kv[1]["ms"]):
                print("%-16s %9.3f ms  %4d launches  %.3f ms/launch" %
                      (k, v["ms"], v["launches"], v["ms"] / max(1, v["launches"])), file=sys.stderr)
        print(json.dumps(rec))
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
