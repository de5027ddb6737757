"""Fractional dedispersion on the GPU (dedisp_mode IC_DEDISP_FFT, psrchive's FFT
phase rotation at iterative_cleaner.py:91, :100, :104) against the C oracle's
restatement of the same written-order rotation (orc_rotate, orc_clean_loop
with delays).  Bit-exact: rotated cubes, templates, amplitudes, status,
weights, residual, std/mean/ptp; fftmax and test values within 1e-9 relative.
NaN samples compare as NaN (payloads are not part of the definition).  The
reference's own clean() on FFT-mode stand-in archives is covered by the
clean_*_fft fixtures in tests/test_gpu_parity.py.  Parity against real
psrchive: unpinned."""
import ctypes

import numpy as np
import pytest

from helpers import bits_equal

pytestmark = pytest.mark.gpu


def _same(a, b):
    """Bit-equal, except that NaNs only need to be NaN."""
    a = np.asarray(a)
    b = np.asarray(b)
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    nan = np.isnan(a) & np.isnan(b)
    eq = a.view(np.uint32 if a.dtype == np.float32 else np.uint64) == b.view(np.uint32 if b.dtype == np.float32
                                                                             else np.uint64)
    return bool(np.all(eq | nan))


def _close(a, b, tol=1e-9):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    same = (a == b) | (np.isnan(a) & np.isnan(b))
    fin = np.isfinite(a) & np.isfinite(b)
    return bool(np.all(same | (fin & (np.abs(a - b) <= tol * np.maximum(1.0, np.abs(b))))))


@pytest.mark.parametrize("nbin", [64, 128, 256, 512, 1024, 2048, 4096])
def test_rotate_profiles_matches_oracle(nbin, oracle_lib):
    from iterative_cleaner_amd import _native
    rng = np.random.default_rng(nbin)
    nsub, nchan = 3, 11
    d = rng.uniform(-5 * nbin, 5 * nbin, nchan)
    d[0], d[1], d[2] = 0.0, 7.0, 0.25
    x = (rng.standard_normal((nsub, nchan, nbin)) * 50).astype(np.float32)
    x[0, 3, nbin - 1] = np.nan
    x[1, 4, :] = 0.0
    x[2, 5, 2] = np.inf
    for sign in (1, -1):
        got = _native.rotate_profiles(x, d, sign)
        assert _same(got, oracle_lib.rotate(x, d, sign)), "sign %d" % sign


@pytest.mark.parametrize("nbin", [64, 1024, 4096])
def test_rotate_profiles_f32_edge_values(nbin, oracle_lib):
    """The f32 rotation (packed v_pk_* arithmetic, f32 denormals kept) on
    subnormal, overflowing, signed-zero and spike profiles, per channel and per
    profile: bit-equal to the C oracle's scalar f32 code (NaNs as NaNs)."""
    from iterative_cleaner_amd import _native
    from test_phase_rotation import _edge_cube
    x = _edge_cube(nbin)
    rng = np.random.default_rng(nbin + 1)
    d = rng.uniform(-2 * nbin, 2 * nbin, 6)
    d[1], d[2] = 0.0, 0.5
    d2 = rng.uniform(-2 * nbin, 2 * nbin, (4, 6))
    for delay in (d, d2):
        for sign in (1, -1):
            got = _native.rotate_profiles(x, delay, sign)
            assert _same(got, oracle_lib.rotate(x, delay, sign)), "sign %d, per-profile %s" % (sign, delay.ndim == 2)


CASES = [
    # (nsub, nchan, nbin, seed, rfi, extra)
    (7, 300, 64, 11, 0.2, {}),                 # two channel super-blocks
    (9, 70, 128, 15, 0.3, {"chanthresh": 3.0, "subintthresh": 2.5}),
    (8, 64, 256, 16, 0.2, {"pulse_region": [0.25, 40, 90]}),
    (6, 50, 512, 17, 0.2, {}),
    (5, 70, 1024, 18, 0.2, {}),
    (4, 30, 2048, 19, 0.3, {}),
    (6, 40, 4096, 13, 0.1, {}),
    (4, 3200, 1024, 1, 0.05, {}),             # the C2 channel count: 13 super-blocks
]


def _pr(args, nbin):
    if list(args["pulse_region"]) == [0, 0, 1]:
        return None
    from iterative_cleaner_amd import _native
    _, fac, a, b = _native.normalise_pulse_region(args["pulse_region"], nbin)
    return (fac, a, b)


@pytest.mark.parametrize("fit_tail", [0, None])
@pytest.mark.parametrize("case", CASES, ids=lambda c: "%dx%dx%d" % c[:3])
def test_fft_loop_matches_c_oracle(case, fit_tail, oracle_lib):
    from iterative_cleaner_amd import _native, synth
    nsub, nchan, nbin, seed, rfi, extra = case
    data, w0, shift = synth.make_cube(nsub, nchan, nbin, seed, rfi)
    delay = synth.fractional_delays(shift, nbin)
    raw = np.ascontiguousarray(data[:, 0])
    args = dict(max_iter=5, chanthresh=5.0, subintthresh=5.0, pulse_region=[0, 0, 1])
    args.update(extra)
    ref = oracle_lib.clean_loop(raw, w0, shift, args["chanthresh"], args["subintthresh"], args["max_iter"],
                                _pr(args, nbin), want_residual=True, want_details=True, delay=delay)
    with _native.GpuSession(nsub, nchan, nbin, args["max_iter"], args["chanthresh"], args["subintthresh"],
                            args["pulse_region"], device=0, delay=delay) as s:
        if fit_tail is not None:
            s.set_fit_tail(fit_tail)
        s.upload(raw, w0, np.zeros(nchan, np.int32))
        out = s.run()
        T = s.template()
        amp, info = s.fit()
        sd, mn, pt, ff = s.diagnostics()
        R = s.residual()
    assert out["loops"] == ref["loops"]
    assert np.array_equal(out["changed"], ref["changed"][:out["n_iter"]])
    assert bits_equal(T, ref["T"][out["n_iter"] - 1])
    assert bits_equal(amp, ref["amp"]) and bits_equal(info, ref["info"])
    assert bits_equal(out["weights"], ref["weights"])
    assert bits_equal(sd, ref["std"]) and bits_equal(mn, ref["mean"]) and bits_equal(pt, ref["ptp"])
    assert _close(ff, ref["fft"]) and _close(out["test"], ref["test"])
    assert _same(R, ref["residual"])


SCHEDULES = [
    # (diag_fork, template_incr, fit_tiled, fit_tail, rot_stats): the round-3
    # schedule on the FFT mode against its plain form, and (nbin 1024) the
    # residual rotation that measures its rows against the rotation + STATS pass
    (0, 0, 0, None, 1),
    (1, 1, 1, 0, 1),
    (3, 1, 0, 512, 0),
    (5, 0, 1, None, 1),
    (0, 1, 1, None, 0),
    (3, 1, 1, None, 1),
]


@pytest.mark.parametrize("case", [CASES[0], CASES[2], CASES[4], CASES[5], CASES[7]],
                         ids=lambda c: "%dx%dx%d" % c[:3])
def test_fft_schedules_are_bit_identical(case, oracle_lib):
    """The diagnostics fork (the residual rotation of the fitted profiles on the
    second stream), the incremental template stage (k_chan_delta on rot(raw)
    and the rotated rows) and the tiled fit cube in the FFT mode: every output
    the same bits under every setting, and the default setting equal to the
    C oracle."""
    from iterative_cleaner_amd import _native, synth
    nsub, nchan, nbin, seed, rfi, extra = case
    data, w0, shift = synth.make_cube(nsub, nchan, nbin, seed, rfi)
    delay = synth.fractional_delays(shift, nbin)
    raw = np.ascontiguousarray(data[:, 0])
    args = dict(max_iter=5, chanthresh=5.0, subintthresh=5.0, pulse_region=[0, 0, 1])
    args.update(extra)

    def run(opts, tail):
        with _native.GpuSession(nsub, nchan, nbin, args["max_iter"], args["chanthresh"], args["subintthresh"],
                                args["pulse_region"], device=0, delay=delay, options=opts) as s:
            if tail is not None:
                s.set_fit_tail(tail)
            s.upload(raw, w0, np.zeros(nchan, np.int32))
            out = s.run()
            out["T"] = s.template()
            out["amp"], out["info"] = s.fit()
            out["diag"] = s.diagnostics()
            out["R"] = s.residual()
        return out

    base = run({}, None)
    ref = oracle_lib.clean_loop(raw, w0, shift, args["chanthresh"], args["subintthresh"], args["max_iter"],
                                _pr(args, nbin), want_residual=True, want_details=True, delay=delay)
    assert base["loops"] == ref["loops"] and bits_equal(base["weights"], ref["weights"])
    assert bits_equal(base["amp"], ref["amp"]) and _same(base["R"], ref["residual"])
    for fork, incr, tiled, tail, rst in SCHEDULES:
        got = run({"diag_fork": fork, "template_incr": incr, "fit_tiled": tiled, "rot_stats": rst}, tail)
        assert got["loops"] == base["loops"] and np.array_equal(got["changed"], base["changed"])
        for key in ("weights", "test", "T", "amp", "info"):
            assert bits_equal(got[key], base[key]), (fork, incr, tiled, key)
        for x0, x1 in zip(base["diag"], got["diag"]):
            assert bits_equal(x1, x0), (fork, incr, tiled)
        assert _same(got["R"], base["R"])


@pytest.mark.parametrize("case", [CASES[0], CASES[2], CASES[4], CASES[6]], ids=lambda c: "%dx%dx%d" % c[:3])
def test_fft_closed_form_loop_matches_c_oracle(case, oracle_lib):
    """fit_mode 1 (closed-form amplitude) with fractional dedispersion: the
    amplitudes of the rotated fit cube (k_diag DIAG_FIT), then the same rotated
    residual and statistics as the exact fit."""
    from iterative_cleaner_amd import _native, synth
    nsub, nchan, nbin, seed, rfi, extra = case
    data, w0, shift = synth.make_cube(nsub, nchan, nbin, seed, rfi)
    delay = synth.fractional_delays(shift, nbin)
    raw = np.ascontiguousarray(data[:, 0])
    args = dict(max_iter=5, chanthresh=5.0, subintthresh=5.0, pulse_region=[0, 0, 1])
    args.update(extra)
    ref = oracle_lib.clean_loop(raw, w0, shift, args["chanthresh"], args["subintthresh"], args["max_iter"],
                                _pr(args, nbin), want_residual=True, want_details=True, fit_mode=1, delay=delay)
    with _native.GpuSession(nsub, nchan, nbin, args["max_iter"], args["chanthresh"], args["subintthresh"],
                            args["pulse_region"], device=0, delay=delay, fit_mode=_native.FIT_CLOSED) as s:
        s.upload(raw, w0, np.zeros(nchan, np.int32))
        out = s.run()
        T = s.template()
        amp, info = s.fit()
        sd, mn, pt, ff = s.diagnostics()
        R = s.residual()
        st = s.run_stats()
    assert st["fit_rounds"] == 0
    assert out["loops"] == ref["loops"]
    assert bits_equal(T, ref["T"][out["n_iter"] - 1])
    assert bits_equal(amp, ref["amp"]) and bits_equal(info, ref["info"])
    assert bits_equal(out["weights"], ref["weights"])
    assert bits_equal(sd, ref["std"]) and bits_equal(mn, ref["mean"]) and bits_equal(pt, ref["ptp"])
    assert _close(ff, ref["fft"]) and _close(out["test"], ref["test"])
    assert _same(R, ref["residual"])


@pytest.mark.parametrize("opts", [{"diag_fork": 3}, {"diag_fork": 1, "template_incr": 0, "fit_tiled": 0}])
def test_fft_local_shards_under_schedule_options(opts):
    """FFT-mode channel shards with the fork (each shard's forked residual
    rotation) and the plain schedule: the same bits as one default session."""
    from iterative_cleaner_amd import sharded, synth
    nsub, nchan, nbin = 8, 1100, 256
    data, w0, shift = synth.make_cube(nsub, nchan, nbin, 91, 0.2)
    delay = synth.fractional_delays(shift, nbin)
    raw = np.ascontiguousarray(data[:, 0])
    zero = np.zeros(nchan, np.int32)
    with _native_session(nsub, nchan, nbin, delay) as s:
        s.upload(raw, w0, zero)
        one = s.run()
        one["amp"], one["info"] = s.fit()
        one["std"], one["mean"], one["ptp"], one["fft"] = s.diagnostics()
    out = sharded.clean_cube_local(raw, w0, zero, 4, want_details=True, fit_tail=512, delay=delay,
                                   options=opts)
    assert out["loops"] == one["loops"] and np.array_equal(out["changed"], one["changed"])
    for key in ("weights", "test", "amp", "info", "std", "mean", "ptp", "fft"):
        assert bits_equal(out[key], one[key]), key


def _native_session(nsub, nchan, nbin, delay):
    from iterative_cleaner_amd import _native
    return _native.GpuSession(nsub, nchan, nbin, device=0, delay=delay)


def test_fft_pols_f64_and_local_shards(oracle_lib):
    """Device pscrunch, f64 data and in-process channel shards in FFT mode."""
    import threading

    from iterative_cleaner_amd import _native, synth
    nsub, nchan, nbin = 6, 600, 256
    data, w0, shift = synth.make_cube(nsub, nchan, nbin, 77, 0.2, npol=2)
    w0 = synth.fractional_weights(w0)
    delay = synth.fractional_delays(shift, nbin)
    raw = (data[:, 0] + data[:, 1]).astype(np.float32)
    zero = np.zeros(nchan, np.int32)
    ref = oracle_lib.clean_loop(raw, w0, shift, want_residual=True, delay=delay)
    with _native.GpuSession(nsub, nchan, nbin, device=0, delay=delay) as s:
        s.upload_pols(data, w0, zero)
        out = s.run()
        R = s.residual()
    assert out["loops"] == ref["loops"] and bits_equal(out["weights"], ref["weights"])
    assert _same(R, ref["residual"])
    ref64 = oracle_lib.clean_loop(raw, w0, shift, data_f64=True, want_details=True, delay=delay)
    with _native.GpuSession(nsub, nchan, nbin, device=0, delay=delay, data_f64=True) as s:
        s.upload(raw, w0, zero)
        out64 = s.run()
        sd, mn, pt, ff = s.diagnostics()
    assert out64["loops"] == ref64["loops"] and bits_equal(out64["weights"], ref64["weights"])
    assert bits_equal(pt, ref64["ptp"]) and bits_equal(mn, ref64["mean"]) and bits_equal(sd, ref64["std"])
    world = 2
    chans, _ = _native.shard_layout(nsub, nchan, world)
    results = [None] * world
    with _native.ShardGroup(world) as g:
        sess = [_native.ShardSession(nsub, nchan, nbin, r, world, group=g, device=0,
                                     delay=delay[chans[r][0]:chans[r][1]]) for r in range(world)]
        for r, (c0, c1) in enumerate(chans):
            sess[r].upload(np.ascontiguousarray(raw[:, c0:c1]), np.ascontiguousarray(w0[:, c0:c1]), zero[c0:c1])

        def go(r):
            results[r] = sess[r].run()
        th = [threading.Thread(target=go, args=(r,)) for r in range(world)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for x in sess:
            x.close()
    merged = np.concatenate([results[r]["weights"] for r in range(world)], axis=1)
    assert bits_equal(merged, ref["weights"])


def test_fft_mode_argument_errors():
    from iterative_cleaner_amd import _native
    with pytest.raises(_native.NativeError, match="power-of-two"):
        _native.GpuSession(4, 8, 100, device=0, delay=np.zeros(8))
    with pytest.raises(_native.NativeError, match="not finite"):
        _native.GpuSession(4, 8, 64, device=0, delay=np.full(8, np.nan))
    with pytest.raises(_native.NativeError, match="power-of-two"):
        _native.rotate_profiles(np.zeros((2, 3, 48), np.float32), np.zeros(3))
    # ic_run before ic_set_delays
    lib = _native.load_library()
    prm = _native.Params(4, 8, 64, 5, 5.0, 5.0, 0, 1.0, 0, 0, 0.15, 0, 0, _native.DEDISP_FFT)
    h = ctypes.c_void_p()
    assert lib.ic_session_create(ctypes.byref(prm), 0, ctypes.byref(h)) == 0
    try:
        cube = np.zeros((4, 8, 64), np.float32)
        w = np.ones((4, 8), np.float32)
        sh = np.zeros(8, np.int32)
        assert lib.ic_upload(h, cube.ctypes.data, w.ctypes.data, sh.ctypes.data) == 0
        rc = lib.ic_run(h, None, None, None, None, None, None, None)
        assert rc == -4 and b"ic_set_delays" in lib.ic_last_error()
    finally:
        lib.ic_session_destroy(h)


@pytest.mark.parametrize("per_profile", [False, True])
def test_fused_residual_statistics_edge_cases(per_profile, oracle_lib):
    """The residual rotation that measures its rows (nbin 1024, IC_OPT_ROT_STATS)
    on the inputs its epilogue branches on: fractional weights (X = f32(R w)),
    zero weights (invalid profiles: fftmax 0), a pulse region in the residual,
    an all-zero profile and a spike, per-channel and per-profile delays (the
    non-finite samples are the fft_nonfinite_edge fixture's).  Fused and
    two-pass runs are bit-identical, and both equal the C oracle."""
    from iterative_cleaner_amd import _native, synth
    nsub, nchan, nbin = 6, 96, 1024
    data, w0, shift = synth.make_cube(nsub, nchan, nbin, 41, 0.2)
    raw = np.ascontiguousarray(data[:, 0])
    raw[2, 60, :] = 0.0
    raw[1, 7, 100:104] += 5e3                  # an impulsive spike
    w0 = w0.copy()
    w0[:, 3] = 0.0
    w0[0, 10:20] = 0.25
    w0[5, 50] = 0.6
    delay = (synth.per_profile_delays(shift, nbin, nsub) if per_profile
             else synth.fractional_delays(shift, nbin))
    args = dict(max_iter=5, chanthresh=4.0, subintthresh=4.0, pulse_region=[0.5, 200, 340])

    def run(rst):
        with _native.GpuSession(nsub, nchan, nbin, args["max_iter"], args["chanthresh"], args["subintthresh"],
                                args["pulse_region"], device=0, delay=delay, options={"rot_stats": rst}) as s:
            s.upload(raw, w0, np.zeros(nchan, np.int32))
            out = s.run()
            out["amp"], out["info"] = s.fit()
            out["diag"] = s.diagnostics()
        return out

    fused, split = run(1), run(0)
    ref = oracle_lib.clean_loop(raw, w0, shift, args["chanthresh"], args["subintthresh"], args["max_iter"],
                                _pr(args, nbin), want_details=True, delay=delay)
    for key in ("weights", "test", "amp", "info"):
        assert bits_equal(fused[key], split[key]), key
    for x0, x1 in zip(split["diag"], fused["diag"]):
        assert _same(x1, x0)
    assert fused["loops"] == ref["loops"] and bits_equal(fused["weights"], ref["weights"])
    sd, mn, pt, ff = fused["diag"]
    assert _same(sd, ref["std"]) and _same(mn, ref["mean"]) and _same(pt, ref["ptp"])
    assert _close(ff, ref["fft"]) and _close(fused["test"], ref["test"])
