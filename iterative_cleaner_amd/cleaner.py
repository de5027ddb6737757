"""Drop-in host for the surgical RFI cleaner: same CLI, same ``clean(ar, args,
arch)``, same prints, log and files as the reference
(/root/reference/iterative_cleaner.py), with the cleaning loop
(iterative_cleaner.py:83-146) executed by libicgpu.so on an MI355X.

Reference map
  parse_arguments  iterative_cleaner.py:16-42   (flags and defaults kept,
                   including the int default 5 of -c/-s and the -r order
                   (factor, start, end) used at :281-283)
  main             :45-62
  clean            :65-178
  set_weights_archive :300-305, find_bad_parts :308-335
"""
from __future__ import annotations

import argparse
import datetime
import os

import numpy as np

from . import _native

__all__ = ["parse_arguments", "main", "clean", "set_weights_archive", "find_bad_parts",
           "archive_backend", "run_loop"]


def archive_backend():
    """The archive module: real psrchive when importable, else the NumPy stand-in."""
    try:
        import psrchive  # noqa: F401
        return psrchive
    except ImportError:
        from . import archive
        return archive


def parse_arguments(argv=None):
    p = argparse.ArgumentParser(description="Commands for the cleaner")
    p.add_argument("archive", nargs="+", help="The chosen archives")
    p.add_argument("-c", "--chanthresh", type=float, default=5, metavar=("channel_threshold"),
                   help="The threshold (in number of sigmas) a profile needs to stand out compared "
                        "to others in the same channel for it to be removed.")
    p.add_argument("-s", "--subintthresh", type=float, default=5, metavar=("subint_threshold"),
                   help="The threshold (in number of sigmas) a profile needs to stand out compared "
                        "to others in the same subint for it to be removed.")
    p.add_argument("-m", "--max_iter", type=int, default=5, metavar=("maximum_iterations"),
                   help="Maximum number of iterations.")
    p.add_argument("-z", "--print_zap", action="store_true",
                   help="Creates a plot that shows which profiles get zapped.")
    p.add_argument("-u", "--unload_res", action="store_true",
                   help="Creates an archive that contains the pulse free residual.")
    p.add_argument("-p", "--pscrunch", action="store_true", help="Pscrunches the output archive.")
    p.add_argument("-q", "--quiet", action="store_true", help="Do not print cleaning information.")
    p.add_argument("-l", "--no_log", action="store_true", help="Do not create cleaning log.")
    p.add_argument("-r", "--pulse_region", nargs=3, type=float, default=[0, 0, 1],
                   metavar=("pulse_start", "pulse_end", "scaling_factor"),
                   help="Defines the range of the pulse and a suppression factor.")
    p.add_argument("-o", "--output", type=str, default="", metavar=("output_filename"),
                   help="Name of the output file. If set to 'std' the pattern NAME.FREQ.MJD.ar "
                        "will be used.")
    p.add_argument("--memory", action="store_true",
                   help="Do not pscrunch the archive while it is in memory. Costs RAM but prevents "
                        "having to reload the archive.")
    p.add_argument("--bad_chan", type=float, default=1,
                   help="Fraction of subints that needs to be removed in order to remove the whole "
                        "channel.")
    p.add_argument("--bad_subint", type=float, default=1,
                   help="Fraction of channels that needs to be removed in order to remove the whole "
                        "subint.")
    return p.parse_args(argv)


def _output_name(ar, args):
    if args.output == "":
        return str(ar).split(":", 1)[1].strip() + "_cleaned.ar"
    if args.output == "std":
        mjd = (float(ar.start_time().strtempo()) + float(ar.end_time().strtempo())) / 2.0
        return "%s.%.3f.%f.ar" % (ar.get_source(), ar.get_centre_frequency(), mjd)
    return args.output


def main(args):
    """CLI driver (iterative_cleaner.py:59-62).  Under torchrun each rank cleans
    its round-robin share of the archive list on its own GPU (batch mode,
    SURVEY.md §8(e): no collective).  With IC_CHANNEL_SHARDS=1 the ranks instead
    clean every archive together, each on its channel shard (config C3): a rank
    reads only its channel slice of the file, and rank 0 writes the outputs."""
    from .dist import channel_sharding, rank_world, shard
    rank, world, _ = rank_world()
    backend = archive_backend()
    together = channel_sharding()
    for arch in (args.archive if together else shard(args.archive, rank, world)):
        ar = _load_shard(backend, arch, rank, world) if together else backend.Archive_load(arch)
        o_name = _output_name(ar, args)
        ar = clean(ar, args, arch)
        if together and rank != 0:
            continue
        ar.unload(o_name)
        if not args.quiet:
            print("Cleaned archive: %s" % o_name)


def _load_shard(backend, arch, rank, world):
    """This rank's channel slice of the archive (channel-sharded CLI).  The
    stand-in formats (npz, PSRFITS) are read slice-only from their headers and a
    memory map; an archive backend that cannot do that (real psrchive) is loaded
    whole and sliced in memory (run_loop)."""
    if backend.__name__.endswith("archive") and hasattr(backend, "load_channels"):
        from . import archive_io
        nsub, _, nchan, _ = archive_io.probe_shape(arch)
        chans, _ = _native.shard_layout(nsub, nchan, world)
        return backend.load_channels(arch, *chans[rank])
    return backend.Archive_load(arch)


def _dedispersion(ar):
    """(shift, delay) of the archive's dedisperse / dededisperse
    (iterative_cleaner.py:91, :100, :104): integer shifts in bins
    (ded[i] = raw[(i+shift)%nbin]) with delay None, or zero shifts and the
    fractional delays in bins of psrchive's FFT phase rotation, (nchan,) or
    (nsub, nchan).  The archive stand-in states its own (get_dm_shift /
    get_dm_delay); any other archive (real psrchive) gets psrchive's delays from
    its DM, channel frequencies and per-Integration folding periods
    (dedispersion.py), integer only when every delay is integral, and an error
    where the fractional rotation cannot serve its nbin."""
    if hasattr(ar, "get_dm_shift"):
        shift = np.asarray(ar.get_dm_shift(), dtype=np.int64)
        get = getattr(ar, "get_dm_delay", None)
        d = get() if get is not None else None
        return shift, (None if d is None else np.asarray(d, dtype=np.float64))
    from . import dedispersion
    return dedispersion.plan(dedispersion.archive_delays(ar), ar.get_nbin(), ar.get_filename())


def _stored_dedispersed(ar) -> bool:
    """The archive holds its samples dedispersed (psrchive get_dedispersed()):
    the reference's dedisperse (:91, :100) is then a no-op."""
    get = getattr(ar, "get_dedispersed", None)
    return bool(get()) if get is not None else False


def _to_dispersed(cube, shift):
    """Integer dedispersion of an archive stored dedispersed: its samples moved
    back to the dispersed frame (raw[j] = ded[(j - shift) % nbin]), exactly, so
    that the loop's own integer dedispersion reproduces the stored samples."""
    nbin = cube.shape[-1]
    out = np.empty_like(cube)
    for c, sh in enumerate(np.asarray(shift, np.int64)):
        idx = (np.arange(nbin) - int(sh)) % nbin
        out[..., c, :] = cube[..., c, idx]
    return out


def _state(ar) -> str:
    """psrchive polarisation state name ("Intensity", "PPQQ", "Coherence",
    "Stokes"); archives without get_state are taken by their npol."""
    if hasattr(ar, "get_state"):
        return str(ar.get_state())
    return {1: "Intensity", 2: "PPQQ", 4: "Coherence"}.get(ar.get_npol(), "PPQQ")


def _loop_input(ar) -> np.ndarray:
    """What the loop cleans (the pscrunched data of iterative_cleaner.py:70,
    :89, :98): (nsub, nchan, nbin) f32 when the archive holds one polarisation
    or is in the Stokes state (total intensity = I = pol 0, psrchive pscrunch),
    else the full-pol (nsub, npol, nchan, nbin) f32 AA, BB(, CR, CI) data, which
    the GPU pscrunches (ic_upload_pols: total intensity f32(pol0 + pol1))."""
    data = ar.get_data()
    if data.shape[1] == 1 or _state(ar) == "Stokes":
        data = data[:, 0]
    cube = np.ascontiguousarray(data, dtype=np.float32)
    if data.dtype != np.float32 and not np.array_equal(cube, data, equal_nan=True):
        raise ValueError("get_data() returned %s values that are not f32 amplitudes" % data.dtype)
    return cube


def _data_f64(ar) -> bool:
    """True when the archive binding's get_data returns f64 (a psrchive build;
    the masked statistics then run in f64: ic_params.data_f64)."""
    dt = getattr(ar, "get_data_dtype", None)
    if dt is not None:
        return np.dtype(dt) == np.float64
    return ar.get_data().dtype == np.float64


def _device() -> int:
    for key in ("IC_DEVICE", "LOCAL_RANK"):
        if os.environ.get(key, "") != "":
            return int(os.environ[key])
    return 0


def run_loop(cube, w0, shift, args, device=None, want_residual=False, baseline_duty=0.15, nchan_total=None,
             data_f64=False, delay=None, input_dedispersed=False):
    """Run the GPU loop on a (nsub, nchan, nbin) f32 cube, or on full-polarisation
    data (nsub, npol, nchan, nbin) that the GPU pscrunches; returns the ic_run dict
    (+ ``residual`` when requested).  Under channel sharding (dist.channel_sharding)
    every rank runs its channel shard and gets the merged result: `cube` is then
    either the whole archive (sliced here) or, with ``nchan_total`` set, already
    this rank's channel slice (read slice-only from the file).  ``delay``:
    fractional delays, (nchan,) or (nsub, nchan) (dedispersion by FFT phase
    rotation); ``input_dedispersed``: the cube is stored dedispersed (FFT
    dedispersion only)."""
    pols = cube.ndim == 4
    nsub, nchan, nbin = (cube.shape[0], cube.shape[2], cube.shape[3]) if pols else cube.shape
    from .dist import channel_sharding
    if channel_sharding():
        import torch

        from . import sharded
        from .dist import rank_world
        rank, world, local = rank_world()
        dev = torch.device("cuda", _device() if device is None else device)
        if nchan_total is None:
            chans, _ = _native.shard_layout(nsub, nchan, world)
            c0, c1 = chans[rank]
            cube = cube[:, :, c0:c1] if pols else cube[:, c0:c1]
            w0, shift = np.asarray(w0)[:, c0:c1], np.asarray(shift)[c0:c1]
            delay = None if delay is None else np.asarray(delay)[..., c0:c1]
            nchan_total = nchan
        return sharded.clean_cube_dist(
            np.ascontiguousarray(cube), np.ascontiguousarray(w0), np.asarray(shift), (nsub, nchan_total, nbin),
            dev, want_residual=want_residual,
            max_iter=args.max_iter, chanthresh=args.chanthresh, subintthresh=args.subintthresh,
            pulse_region=args.pulse_region, baseline_duty=baseline_duty, data_f64=data_f64, delay=delay,
            input_dedispersed=input_dedispersed)
    if nchan_total is not None and nchan_total != nchan:
        raise ValueError("a channel slice of an archive needs channel sharding")
    with _native.GpuSession(nsub, nchan, nbin, args.max_iter, args.chanthresh, args.subintthresh,
                            args.pulse_region, baseline_duty,
                            device=_device() if device is None else device, data_f64=data_f64, delay=delay,
                            input_dedispersed=input_dedispersed) as s:
        if pols:
            s.upload_pols(cube, w0, shift)
        else:
            s.upload(cube, w0, shift)
        out = s.run()
        if want_residual and out["n_iter"] > 0:
            out["residual"] = s.residual()
    return out


def set_weights_archive(archive, test_results):
    """Zero the weight of every profile whose test value is >= 1 (ic.py:300-305)."""
    for isub, ichan in np.argwhere(test_results >= 1):
        archive.get_Integration(int(isub)).set_weight(int(ichan), 0.0)


def find_bad_parts(archive, args):
    """Zap whole subints / channels whose zero-weight fraction exceeds the limit
    (ic.py:308-335); both passes read the weights as they were on entry."""
    weights = archive.get_weights()
    n_subints = archive.get_nsubint()
    n_channels = archive.get_nchan()
    n_bad_channels = 0
    n_bad_subints = 0
    for i in range(n_subints):
        bad_frac = 1 - np.count_nonzero(weights[i, :]) / float(n_channels)
        if bad_frac > args.bad_subint:
            for j in range(n_channels):
                archive.get_Integration(int(i)).set_weight(int(j), 0.0)
            n_bad_subints += 1
    for j in range(n_channels):
        bad_frac = 1 - np.count_nonzero(weights[:, j]) / float(n_subints)
        if bad_frac > args.bad_chan:
            for i in range(n_subints):
                archive.get_Integration(int(i)).set_weight(int(j), 0.0)
            n_bad_channels += 1
    if not args.quiet and n_bad_channels + n_bad_subints != 0:
        print("Removed %s bad subintegrations and %s bad channels." % (n_bad_subints, n_bad_channels))
    return archive


def _plot_zap(test, ar_name, args):
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.cm as cm
    import matplotlib.pyplot as plt
    plt.imshow(test.T, vmin=0.999, vmax=1.001, aspect="auto", interpolation="nearest",
               cmap=cm.coolwarm)
    plt.gca().invert_yaxis()
    plt.title("%s cthresh=%s sthresh=%s" % (ar_name, args.chanthresh, args.subintthresh))
    plt.savefig("%s_%s_%s.png" % (ar_name, args.chanthresh, args.subintthresh), bbox_inches="tight")


BAD_STATUS = "Bad status for least squares fit when removing profile."


def clean(ar, args, arch):
    """Surgical cleaning of one archive (iterative_cleaner.py:65-178).  Under
    channel sharding only rank 0 prints and writes files; `ar` may then be this
    rank's channel slice (main() reads slice-only) and rank 0 loads the whole
    archive for the output."""
    from .dist import channel_sharding, rank_world
    sharding = channel_sharding()
    if sharding and rank_world()[0] != 0:
        args = argparse.Namespace(**dict(vars(args), quiet=True, no_log=True, print_zap=False))
        _side_effects = False
    else:
        _side_effects = True
    backend = archive_backend()
    chan_slice = getattr(ar, "_chan_range", None) is not None
    nchan_total = ar._nchan_total if chan_slice else None
    orig_weights = ar.get_weights()
    # The reference pscrunches the archive in memory unless --memory without -p
    # (iterative_cleaner.py:67-70).  Only -p keeps that pscrunched copy as the
    # output; otherwise the archive is reloaded (or kept full-pol with --memory),
    # so its data go to the GPU full-pol and are pscrunched there.
    if args.pscrunch and not chan_slice:
        ar.pscrunch()
    ar_name = ar.get_filename().split()[-1]
    max_iterations = args.max_iter
    size = orig_weights.shape[0] * nchan_total if chan_slice else orig_weights.size
    if not args.quiet:
        print("Total number of profiles: %s" % size)

    cube = _loop_input(ar)
    shift, delay = _dedispersion(ar)
    stored_ded = _stored_dedispersed(ar)
    if stored_ded and delay is None:
        cube = _to_dispersed(cube, shift)
    duty = ar.get_baseline_duty() if hasattr(ar, "get_baseline_duty") else 0.15
    out = run_loop(cube, orig_weights, shift, args, want_residual=args.unload_res, baseline_duty=duty,
                   nchan_total=nchan_total, data_f64=_data_f64(ar), delay=delay,
                   input_dedispersed=stored_ded and delay is not None)
    del cube

    x = 0
    loops = None
    bad = out.get("bad_fits", [0] * out["n_iter"])
    for k in range(out["n_iter"]):
        x = k + 1
        if not args.quiet:
            print("Loop: %s" % x)
        if _side_effects:
            # printed by remove_profile1d for every failed fit, -q or not (:284-285)
            for _ in range(int(bad[k])):
                print(BAD_STATUS)
        if not args.quiet:
            rfi_frac = out["nzero"][k] / float(size)
            print("Differences to previous weights: %s  RFI fraction: %s"
                  % (int(out["changed"][k]), rfi_frac))
        if k == out["n_iter"] - 1 and out["converged"]:
            if not args.quiet:
                print("RFI removal stops after %s loops." % x)
            loops = x
            x = 1000000
    if x == max_iterations:
        if not args.quiet:
            print("Cleaning was interrupted after the maximum amount of loops (%s)" % max_iterations)
        loops = max_iterations
    if out["n_iter"] == 0:
        raise NameError("name 'avg_test_results' is not defined")
    avg_test_results = out["test"]

    if chan_slice:
        if not _side_effects:
            return ar              # outputs are rank 0's
        # the whole archive for the output: what the reference holds at :150-153
        # (reloaded; or the in-memory archive, pscrunched with -p)
        ar = backend.Archive_load(arch)
        orig_weights = ar.get_weights()      # the residual archive's weights (pscrunch keeps them)
        if args.pscrunch:
            ar.pscrunch()
        shift, delay = _dedispersion(ar)
    elif not args.pscrunch and not args.memory:
        ar = backend.Archive_load(arch)
    set_weights_archive(ar, avg_test_results)
    if args.bad_chan != 1 or args.bad_subint != 1:
        ar = find_bad_parts(ar, args)
    if args.unload_res and _side_effects:
        _residual_archive(ar, out["residual"], orig_weights, shift, backend, delay).unload(
            "%s_residual_%s.ar" % (ar_name, loops))
    if args.print_zap:
        _plot_zap(avg_test_results, ar_name, args)
    if not args.no_log:
        with open("clean.log", "a") as fh:
            fh.write("\n %s: Cleaned %s with %s, required loops=%s"
                     % (datetime.datetime.now(), ar_name, args, loops))
    return ar


def _residual_archive(ar, residual, weights, shift, backend, delay=None):
    """The pulse-free residual archive of the last loop (ic.py:106-108, :161-162)."""
    from .archive import Archive
    return Archive(residual[:, None], weights, shift, dedispersed=False, dm_delay=delay,
                   filename="residual.ar",
                   source=ar.get_source() if hasattr(ar, "get_source") else "J0000+0000")


if __name__ == "__main__":  # pragma: no cover
    main(parse_arguments())
