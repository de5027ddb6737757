"""GPU parity of the channel-sharded loop (config C3): an
archive cleaned as 2/4/8 in-process channel shards (libicgpu shard sessions,
exchanging through device copies) must be bit-identical to one unsharded
session and to the C oracle — masks, weights, loops, counters, template, fit
amplitudes/status and std/mean/ptp; fftmax within 1e-9 relative of the oracle
and bit-identical to the unsharded GPU run (same kernels)."""
import numpy as np
import pytest

from helpers import bits_equal, bits_equal_nan

pytestmark = pytest.mark.gpu

CASES = [
    # (nsub, nchan, nbin, seed, rfi, worlds)
    (7, 520, 64, 31, 0.2, (1, 2)),            # 3 super-blocks: shards of 1 and 2 blocks; 1-rank group
    (9, 1100, 128, 32, 0.3, (2, 4)),          # 5 super-blocks, ragged last shard
    (3, 1024, 32, 33, 0.2, (4,)),             # fewer subints than shards: a rank owns no rows
    (12, 2048, 256, 34, 0.2, (2, 4, 8)),      # 8 super-blocks, one per shard at world 8
    (5, 777, 100, 35, 0.3, (2,)),             # non power-of-two nbin (generic k_diag)
]


def _single(raw, w0, shift, **kw):
    from iterative_cleaner_amd import _native
    nsub, nchan, nbin = raw.shape
    with _native.GpuSession(nsub, nchan, nbin, device=0, **kw) as s:
        s.upload(raw, w0, shift)
        out = s.run()
        out["amp"], out["info"] = s.fit()
        out["std"], out["mean"], out["ptp"], out["fft"] = s.diagnostics()
        out["T"] = s.template()
    return out


@pytest.mark.parametrize("case", CASES, ids=lambda c: "%dx%dx%d" % c[:3])
def test_local_shards_match_single_session(case, oracle_lib):
    from iterative_cleaner_amd import sharded, synth
    nsub, nchan, nbin, seed, rfi, worlds = case
    data, w0, shift = synth.make_cube(nsub, nchan, nbin, seed, rfi)
    raw = np.ascontiguousarray(data[:, 0])
    one = _single(raw, w0, shift)
    ref = oracle_lib.clean_loop(raw, w0, shift, want_details=True)
    assert one["loops"] == ref["loops"] and bits_equal(one["weights"], ref["weights"])
    for world in worlds:
        out = sharded.clean_cube_local(raw, w0, shift, world, want_details=True)
        assert out["loops"] == one["loops"] and out["n_iter"] == one["n_iter"]
        assert np.array_equal(out["changed"], one["changed"])
        assert np.array_equal(out["nzero"], one["nzero"])
        for key in ("weights", "test", "amp", "info", "std", "mean", "ptp", "fft", "T"):
            assert bits_equal(out[key], one[key]), "world %d: %s differs" % (world, key)


def test_local_shards_moving_window_and_pulse_region():
    """Baseline windows that move between iterations (flagged recompute on
    every shard) and an active pulse region, at world 4."""
    from iterative_cleaner_amd import sharded, synth
    data, w0, shift = synth.make_cube(6, 1030, 128, 36, 0.2)
    raw = np.ascontiguousarray(data[:, 0])
    raw[2, 5, 70:80] -= 400.0
    raw[4, 700, 90:95] -= 300.0
    kw = dict(chanthresh=4.0, subintthresh=3.5, pulse_region=[0.5, 20, 50])
    one = _single(raw, w0, shift, **kw)
    for tail in (0, 1 << 40):
        out = sharded.clean_cube_local(raw, w0, shift, 4, want_details=True, fit_tail=tail, **kw)
        for key in ("weights", "test", "amp", "std", "fft", "T"):
            assert bits_equal(out[key], one[key]), key
        assert out["loops"] == one["loops"]


@pytest.mark.parametrize("opts", [{"tail_split": 1, "diag_fork": 2}, {"diag_fork": 0},
                                  {"fork_delay": 0, "template_incr": 0}])
def test_local_shards_under_schedule_options(opts):
    """Schedule options on every shard (the second fork at the tail, no fork,
    the forked pass at once with the full template passes): the same bits as
    one default session."""
    from iterative_cleaner_amd import sharded, synth
    data, w0, shift = synth.make_cube(12, 2048, 256, 34, 0.2)
    raw = np.ascontiguousarray(data[:, 0])
    one = _single(raw, w0, shift)
    out = sharded.clean_cube_local(raw, w0, shift, 4, want_details=True, fit_tail=1024, options=opts)
    assert out["loops"] == one["loops"] and np.array_equal(out["changed"], one["changed"])
    for key in ("weights", "test", "amp", "info", "std", "mean", "ptp", "fft", "T"):
        assert bits_equal(out[key], one[key]), key


def test_local_shards_with_non_finite_samples(oracle_lib):
    """NaN / +-Inf samples (they poison the template: nothing is zapped, std is
    0 where numpy.ma masks the non-finite mean; clean_s8x24x128_nonfinite_edge)
    and a zero-weight channel, at world 2 and 4: the single session's values,
    NaN for NaN (a NaN's sign is the hardware's), and the oracle's weights."""
    from iterative_cleaner_amd import sharded, synth
    data, w0, shift = synth.make_cube(6, 1100, 128, 38, 0.2)
    raw = np.ascontiguousarray(data[:, 0])
    raw[1, 700, 10] = np.nan
    raw[4, 300, 100] = np.inf
    raw[5, 1050, 0] = -np.inf
    w0 = w0.copy()
    w0[:, 17] = 0.0
    one = _single(raw, w0, shift)
    ref = oracle_lib.clean_loop(raw, w0, shift, want_details=True)
    assert one["loops"] == ref["loops"] and bits_equal(one["weights"], ref["weights"])
    assert bits_equal_nan(one["std"], ref["std"]) and not one["std"][w0 != 0].any()
    for world in (2, 4):
        out = sharded.clean_cube_local(raw, w0, shift, world, want_details=True)
        assert out["loops"] == one["loops"] and np.array_equal(out["changed"], one["changed"])
        for key in ("weights", "test", "amp", "info", "std", "mean", "ptp", "fft", "T"):
            assert bits_equal_nan(out[key], one[key]), "world %d: %s differs" % (world, key)


def test_shard_layout_rejects_bad_worlds():
    from iterative_cleaner_amd import _native
    with pytest.raises(_native.NativeError):
        _native.ShardSession(4, 600, 64, 0, 3, group=_native.ShardGroup(3))   # not a power of two
    with pytest.raises(_native.NativeError):
        _native.ShardSession(4, 300, 64, 0, 4, group=_native.ShardGroup(4))   # 2 super-blocks < 4


@pytest.mark.parametrize("backend", ["nccl", "gloo"])
def test_torch_comm_one_rank_shard_session(backend):
    """A one-rank shard session whose exchanges run through dist.TorchComm on a
    real process group: on "nccl" that is RCCL on the session's HIP stream
    (ExternalStream), the path the multi-GPU bench uses; on "gloo" the
    host-staged path.  Must equal the unsharded session bit for bit."""
    import torch
    import torch.distributed as dist

    from iterative_cleaner_amd import _native, synth
    from iterative_cleaner_amd.dist import TorchComm
    data, w0, shift = synth.make_cube(8, 600, 256, 37, 0.2)
    raw = np.ascontiguousarray(data[:, 0])
    one = _single(raw, w0, shift)
    dev = torch.device("cuda", 0)
    kw = dict(store=dist.HashStore(), rank=0, world_size=1)
    if backend == "nccl":
        kw["device_id"] = dev
    dist.init_process_group(backend, **kw)
    try:
        comm = TorchComm(dev)
        with _native.ShardSession(8, 600, 256, 0, 1, comm=comm, device=0) as s:
            s.upload(raw, w0, shift)
            out = s.run()
            amp, _ = s.fit()
            T = s.template()
        assert comm.error is None
        assert out["loops"] == one["loops"] and np.array_equal(out["changed"], one["changed"])
        assert bits_equal(out["weights"], one["weights"]) and bits_equal(out["test"], one["test"])
        assert bits_equal(amp, one["amp"]) and bits_equal(T, one["T"])
        assert len(comm.bufs) == 0          # every exchange buffer released on close
    finally:
        dist.destroy_process_group()


def test_native_rccl_one_rank_shard_session():
    """The library's own RCCL transport (ic_session_create_rccl, the path
    bench.py --gpus N takes on "nccl"): a one-rank communicator whose every
    exchange is issued from C++ on the session stream, the unique id shared
    through a one-rank process group as the multi-rank runs share it.  Must
    equal the unsharded session bit for bit, on both fit schedules."""
    import torch
    import torch.distributed as dist

    from iterative_cleaner_amd import _native, synth
    from iterative_cleaner_amd.dist import share_rccl_id
    data, w0, shift = synth.make_cube(8, 600, 256, 37, 0.2)
    raw = np.ascontiguousarray(data[:, 0])
    one = _single(raw, w0, shift)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=dev)
    try:
        for _ in range(1):
            rid = share_rccl_id()          # one unique id per communicator
            assert len(rid) == 128
            with _native.ShardSession(8, 600, 256, 0, 1, rccl_id=rid, device=0,
                                      options={"diag_fork": 3}) as s:
                s.upload(raw, w0, shift)
                out = s.run()
                amp, _ = s.fit()
                T = s.template()
            assert out["loops"] == one["loops"] and np.array_equal(out["changed"], one["changed"])
            assert bits_equal(out["weights"], one["weights"]) and bits_equal(out["test"], one["test"])
            assert bits_equal(amp, one["amp"]) and bits_equal(T, one["T"])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("nbin,per_profile", [(256, False), (1024, False), (1024, True)])
def test_local_shards_fft_dedispersion(nbin, per_profile, oracle_lib):
    """psrchive's fractional dedispersion on channel shards: each rank rotates
    its channels' rows with their delays (one per channel, or one per profile
    as psrchive's per-Integration periods give), and at nbin 1024 its residual
    rotation measures the rows in the same kernel.  World 2 and 4 equal one
    session bit for bit, and the session equals the C oracle."""
    from iterative_cleaner_amd import sharded, synth
    nsub, nchan = 6, 1100
    data, w0, shift = synth.make_cube(nsub, nchan, nbin, 39, 0.2)
    raw = np.ascontiguousarray(data[:, 0])
    delay = (synth.per_profile_delays(shift, nbin, nsub) if per_profile
             else synth.fractional_delays(shift, nbin))
    zero = np.zeros(nchan, np.int32)
    one = _single(raw, w0, zero, delay=delay)
    ref = oracle_lib.clean_loop(raw, w0, shift, want_details=True, delay=delay)
    assert one["loops"] == ref["loops"] and bits_equal(one["weights"], ref["weights"])
    assert bits_equal(one["amp"], ref["amp"]) and bits_equal(one["std"], ref["std"])
    for world in (2, 4):
        out = sharded.clean_cube_local(raw, w0, zero, world, want_details=True, delay=delay)
        assert out["loops"] == one["loops"] and np.array_equal(out["changed"], one["changed"])
        for key in ("weights", "test", "amp", "info", "std", "mean", "ptp", "fft", "T"):
            assert bits_equal(out[key], one[key]), "world %d: %s differs" % (world, key)
