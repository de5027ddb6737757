"""GPU parity: the HIP loop (through the C-ABI) against the reference's golden
fixtures and the C oracle.  Bit-exact for masks, weights, loops, template,
fit amplitudes/status and the std/mean/ptp diagnostics; fftmax within 1e-9
relative (our FFT vs pocketfft) and test values within 1e-9 absolute (the
fftmax tolerance propagated through median/MAD scaling)."""
import os

import numpy as np
import pytest

from helpers import (bits_equal, bits_equal_nan, case_delay, case_kwargs, clean_fixtures, load_clean_case, nan_equal,
                     poke_cube)

pytestmark = pytest.mark.gpu

FFT_RTOL = 1e-9
TEST_ATOL = 1e-9


# exact-fit schedules: sweep/state rounds only, k_fit_tail only, the default mix
FIT_MODES = {"rounds": 0, "tail": 1 << 40, "default": None}


def _session(shape, args, duty=0.15, fit_mode="default", data_f64=False, delay=None, input_dedispersed=False):
    from iterative_cleaner_amd import _native
    nsub, nchan, nbin = shape
    s = _native.GpuSession(nsub, nchan, nbin, args["max_iter"], args["chanthresh"],
                           args["subintthresh"], args["pulse_region"], duty, device=0, data_f64=data_f64,
                           delay=delay, input_dedispersed=input_dedispersed)
    if FIT_MODES[fit_mode] is not None:
        s.set_fit_tail(FIT_MODES[fit_mode])
    return s


def _close_fft(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    both_nan = np.isnan(a) & np.isnan(b)
    ok = both_nan | (np.abs(a - b) <= FFT_RTOL * np.maximum(np.abs(b), 1e-300)) | (a == b)
    return bool(ok.all())


def _close_test(a, b):
    both_nan = np.isnan(a) & np.isnan(b)
    same_inf = np.isinf(a) & np.isinf(b) & (np.sign(a) == np.sign(b))
    fin = np.isfinite(a) & np.isfinite(b)
    ok = both_nan | same_inf | (fin & (np.abs(a - b) <= TEST_ATOL * np.maximum(1.0, np.abs(b))))
    return bool(ok.all())


@pytest.mark.parametrize("fit_mode", sorted(FIT_MODES))
@pytest.mark.parametrize("path", clean_fixtures(), ids=lambda p: os.path.basename(p)[6:-4])
def test_loop_matches_reference(path, fit_mode):
    z, meta, raw, w0, shift, args = load_clean_case(path)
    nit = int(z["n_iter"])
    with _session(raw.shape, args, fit_mode=fit_mode, data_f64=meta.get("data_f64", False),
                  **case_kwargs(z, meta)) as s:
        s.upload(raw, w0, shift)
        out = s.run()
        T = s.template()
        amp, info = s.fit()
        sd, mn, pt, ff = s.diagnostics()
    assert out["n_iter"] == nit
    assert out["loops"] == int(z["loops"])
    assert bits_equal(out["weights"], z["weights_%d" % nit]), "zap mask differs"
    assert bits_equal_nan(T, z["T_%d" % nit])
    assert bits_equal(amp.ravel(), z["amp_%d" % nit]), "leastsq amplitudes differ"
    assert bits_equal(info.ravel(), z["info_%d" % nit])
    assert bits_equal_nan(sd, z["diag_std_%d" % nit])
    assert bits_equal_nan(mn, z["diag_mean_%d" % nit])
    assert bits_equal_nan(pt, z["diag_ptp_%d" % nit])
    assert _close_fft(ff, z["diag_fft_%d" % nit])
    assert _close_test(out["test"], z["test_%d" % nit])
    # per-iteration counters reproduce the reference's prints (ic.py:129-130)
    prev = w0
    for k in range(1, nit + 1):
        wk = z["weights_%d" % k]
        assert out["changed"][k - 1] == int(np.sum(wk != prev))
        assert out["nzero"][k - 1] == int(wk.size - np.count_nonzero(wk))
        prev = wk


@pytest.mark.parametrize("path", clean_fixtures(), ids=lambda p: os.path.basename(p)[6:-4])
def test_every_iteration_matches_reference(path):
    """Iterations 1 .. n_iter-1 of the reference's loop, stage by stage: a
    session stopped at max_iter = k holds iteration k's template (ic.py:94),
    leastsq amplitudes and status (:278), diagnostics (:206-217), test values
    (:225) and weights (:125), which must equal the fixture's *_k records
    (test_loop_matches_reference checks the last iteration)."""
    z, meta, raw, w0, shift, args = load_clean_case(path)
    nit = int(z["n_iter"])
    for k in range(1, nit):
        a = dict(args, max_iter=k)
        with _session(raw.shape, a, data_f64=meta.get("data_f64", False), **case_kwargs(z, meta)) as s:
            s.upload(raw, w0, shift)
            out = s.run()
            T = s.template()
            amp, info = s.fit()
            sd, mn, pt, ff = s.diagnostics()
        assert out["n_iter"] == k
        assert bits_equal_nan(T, z["T_%d" % k]), "template, iteration %d" % k
        assert bits_equal(amp.ravel(), z["amp_%d" % k]), "leastsq amplitudes, iteration %d" % k
        assert bits_equal(info.ravel(), z["info_%d" % k]), "leastsq status, iteration %d" % k
        assert bits_equal_nan(sd, z["diag_std_%d" % k]), "std, iteration %d" % k
        assert bits_equal_nan(mn, z["diag_mean_%d" % k]), "mean, iteration %d" % k
        assert bits_equal_nan(pt, z["diag_ptp_%d" % k]), "ptp, iteration %d" % k
        assert _close_fft(ff, z["diag_fft_%d" % k]), "fftmax, iteration %d" % k
        assert _close_test(out["test"], z["test_%d" % k]), "test, iteration %d" % k
        assert bits_equal(out["weights"], z["weights_%d" % k]), "weights, iteration %d" % k


@pytest.mark.parametrize("path", clean_fixtures(), ids=lambda p: os.path.basename(p)[6:-4])
def test_clean_stdout_matches_reference(path, tmp_path, monkeypatch, capsys):
    """clean() prints exactly what the reference printed (ic.py:82-145)."""
    from iterative_cleaner_amd import archive as ica
    from iterative_cleaner_amd import cleaner
    z, meta, raw, w0, shift, args = load_clean_case(path)
    from iterative_cleaner_amd import synth
    data, w0_, shift_ = synth.make_cube(meta["nsub"], meta["nchan"], meta["nbin"], meta["seed"],
                                        meta["rfi"], npol=meta["npol"])
    if meta.get("frac_weights"):
        w0_ = synth.fractional_weights(w0_)
    if meta.get("weights_zero"):
        w0_ = np.zeros_like(w0_)
    poke_cube(data, meta)
    monkeypatch.chdir(tmp_path)
    arpath = str(tmp_path / ("%s.ar" % meta["name"]))
    src = ica.Archive(data, w0_, shift_, filename=arpath, dm_delay=case_delay(z, meta))
    if meta.get("stored_dedispersed"):
        src.dedisperse()
    src.unload(arpath)
    ar = ica.Archive_load(arpath)
    plain_load = ica.Archive_load       # the fixture read the residual archive through this one
    if meta.get("data_f64"):
        # a binding whose get_data returns f64 (the reference's reload at :150 saw the same)
        ar.get_data_dtype = np.float64
        orig_load = ica.Archive_load

        def load64(path):
            a = orig_load(path)
            a.get_data_dtype = np.float64
            return a
        monkeypatch.setattr(ica, "Archive_load", load64)
    ns = cleaner.parse_arguments(["-l", *meta["extra_args"], arpath])
    out_ar = cleaner.clean(ar, ns, arpath)
    printed = capsys.readouterr().out
    assert printed == str(z["stdout"])
    assert bits_equal(out_ar.get_weights(), z["final_weights"])
    if "-u" in meta["extra_args"]:
        # the residual archive (iterative_cleaner.py:106-108, :161-162) equals the reference's
        import hashlib
        res = plain_load("%s_residual_%s.ar" % (arpath, int(z["loops"])))
        rdata = res.get_data()
        assert rdata.shape == tuple(z["residual_shape"])
        assert bits_equal(res.get_weights(), z["residual_weights"])
        if "residual_data" in z.files:
            assert bits_equal_nan(rdata, z["residual_data"])
        else:
            assert bits_equal_nan(rdata[0], z["residual_subint0"])
        if not np.isnan(rdata).any():   # a NaN's sign is the hardware's (helpers.bits_equal_nan)
            assert hashlib.sha256(rdata.tobytes()).hexdigest() == str(z["residual_sha256"])


CASES = [
    # (nsub, nchan, nbin, seed, rfi, extra)
    (7, 300, 64, 11, 0.2, {}),                 # two channel super-blocks
    (5, 33, 100, 12, 0.3, {}),                 # non power-of-two nbin (direct DFT)
    (6, 40, 4096, 13, 0.1, {}),                # long profiles
    (3, 20, 8, 14, 0.3, {}),                   # tiny profiles
    (9, 70, 128, 15, 0.3, {"chanthresh": 3.0, "subintthresh": 2.5}),
    (8, 64, 256, 16, 0.2, {"pulse_region": [0.25, 40, 90]}),
    (6, 50, 512, 17, 0.2, {}),
    (5, 70, 1024, 18, 0.2, {}),                # the C2 profile length
    (4, 30, 2048, 19, 0.3, {}),
    (4, 520, 32, 20, 0.2, {}),                 # three super-blocks, short profiles
]


@pytest.mark.parametrize("fit_mode", ["rounds", "tail"])
@pytest.mark.parametrize("case", CASES, ids=lambda c: "%dx%dx%d" % c[:3])
def test_loop_matches_c_oracle(case, fit_mode, oracle_lib):
    from iterative_cleaner_amd import synth
    nsub, nchan, nbin, seed, rfi, extra = case
    data, w0, shift = synth.make_cube(nsub, nchan, nbin, seed, rfi)
    raw = np.ascontiguousarray(data[:, 0])
    args = dict(max_iter=5, chanthresh=5, subintthresh=5, pulse_region=[0, 0, 1])
    args.update(extra)
    pr = None if args["pulse_region"] == [0, 0, 1] else args["pulse_region"]
    ref = oracle_lib.clean_loop(raw, w0, shift, args["chanthresh"], args["subintthresh"],
                                args["max_iter"], pr, want_residual=True, want_details=True)
    with _session(raw.shape, args, fit_mode=fit_mode) as s:
        s.upload(raw, w0, shift)
        out = s.run()
        amp, info = s.fit()
        sd, mn, pt, ff = s.diagnostics()
        R = s.residual()
        st = s.run_stats()
    if fit_mode == "rounds":
        assert st["fit_tail_sweeps"] == 0 and st["fit_profile_sweeps"] > 0
    else:
        assert st["fit_profile_sweeps"] == 0 and st["fit_tail_sweeps"] > 0
    assert out["loops"] == ref["loops"]
    assert bits_equal(out["weights"], ref["weights"])
    assert np.array_equal(out["changed"], ref["changed"][:out["n_iter"]])
    assert bits_equal(amp, ref["amp"]) and bits_equal(info, ref["info"])
    assert bits_equal(sd, ref["std"]) and bits_equal(mn, ref["mean"]) and bits_equal(pt, ref["ptp"])
    assert _close_fft(ff, ref["fft"])
    assert _close_test(out["test"], ref["test"])
    assert bits_equal(R, ref["residual"])


@pytest.mark.parametrize("fit_mode", ["rounds", "tail"])
def test_edge_profiles_match_c_oracle(fit_mode, oracle_lib):
    """Dead (all-zero) channels with weight 1, zero profiles, a NaN-free
    constant channel, fractional weights (K2, K7, K10)."""
    from iterative_cleaner_amd import synth
    data, w0, shift = synth.make_cube(10, 48, 128, 99, 0.2)
    raw = np.ascontiguousarray(data[:, 0])
    raw[:, 3, :] = 0.0                       # dead channel, weight 1
    raw[:, 5, :] = 2.5                       # constant channel
    raw[4, :, :] = 0.0                       # zero subint
    w0 = w0.copy()
    w0[:, 7] = 0.5                           # fractional weights
    w0[2, 9] = 0.0
    ref = oracle_lib.clean_loop(raw, w0, shift, want_details=True)
    args = dict(max_iter=5, chanthresh=5, subintthresh=5, pulse_region=[0, 0, 1])
    with _session(raw.shape, args, fit_mode=fit_mode) as s:
        s.upload(raw, w0, shift)
        out = s.run()
        amp, info = s.fit()
    assert out["loops"] == ref["loops"]
    assert bits_equal(out["weights"], ref["weights"])
    assert bits_equal(amp, ref["amp"]) and bits_equal(info, ref["info"])
    assert _close_test(out["test"], ref["test"])


def test_moving_baseline_window_matches_c_oracle(oracle_lib):
    """A deep narrow dip in one profile drags its subint's baseline window onto
    it until the profile is zapped; the window then moves, and the carried
    baseline levels / fscrunch partials of that subint must be recomputed."""
    from iterative_cleaner_amd import synth
    data, w0, shift = synth.make_cube(6, 40, 128, 123, 0.1)
    raw = np.ascontiguousarray(data[:, 0])
    raw[2, 5, 70:80] -= 400.0           # dispersed frame; lands off-pulse after dedispersion
    raw[4, 11, 90:95] -= 300.0
    ref = oracle_lib.clean_loop(raw, w0, shift, want_details=True)
    args = dict(max_iter=5, chanthresh=5, subintthresh=5, pulse_region=[0, 0, 1])
    with _session(raw.shape, args) as s:
        s.upload(raw, w0, shift)
        out = s.run()
        T = s.template()
        amp, info = s.fit()
        st = s.run_stats()
    assert st["window_moves"] > 0
    assert out["loops"] == ref["loops"]
    assert bits_equal(out["weights"], ref["weights"])
    assert bits_equal(amp, ref["amp"]) and bits_equal(info, ref["info"])
    assert _close_test(out["test"], ref["test"])


@pytest.mark.parametrize("fit_mode", ["rounds", "default"])
def test_extreme_amplitudes_match_c_oracle(fit_mode, oracle_lib):
    """Profiles whose fitted amplitudes fall outside the fast sweep's ranges
    (|x| < 2^-100 or > 2^100 for the A sweep, 2^+-500 for B) or whose samples
    are tiny / huge: the exact re-sweeps must reproduce MINPACK bit for bit."""
    from iterative_cleaner_amd import synth
    data, w0, shift = synth.make_cube(6, 40, 128, 321, 0.1)
    raw = np.ascontiguousarray(data[:, 0])
    raw[1, 3] *= np.float32(1e-33)           # amplitude ~1e-33: exact A sweeps
    raw[2, 4] *= np.float32(3e33)            # huge samples, amplitude ~1e33
    raw[3, 5] *= np.float32(1e-25)
    raw[4, 6] = np.float32(1e-38) * (np.arange(128) % 3)   # near-denormal samples
    raw[5, 7, 10] = np.float32(3e38)         # one huge spike
    ref = oracle_lib.clean_loop(raw, w0, shift, want_details=True)
    args = dict(max_iter=5, chanthresh=5, subintthresh=5, pulse_region=[0, 0, 1])
    with _session(raw.shape, args, fit_mode=fit_mode) as s:
        s.upload(raw, w0, shift)
        out = s.run()
        amp, info = s.fit()
        sd, mn, pt, ff = s.diagnostics()
    assert out["loops"] == ref["loops"]
    assert bits_equal(out["weights"], ref["weights"])
    assert bits_equal(amp, ref["amp"]) and bits_equal(info, ref["info"])
    assert bits_equal(sd, ref["std"]) and bits_equal(mn, ref["mean"])


@pytest.mark.parametrize("path", [p for p in clean_fixtures() if "fft" not in os.path.basename(p)][:4],
                         ids=lambda p: os.path.basename(p)[6:-4])
def test_row_major_fit_cube_matches_tiled(path, monkeypatch):
    """The fit cube's two layouts (session option fit_tiled: tiled by
    default, row-major as the A/B baseline) give the same bits, and
    both the reference's: layout moves bytes, never arithmetic."""
    z, meta, raw, w0, shift, args = load_clean_case(path)
    nit = int(z["n_iter"])
    outs = []
    for tiled in (1, 0):
        with _session(raw.shape, args, data_f64=meta.get("data_f64", False)) as s:
            s.set_option("fit_tiled", tiled)
            assert s.get_option("fit_tiled") == tiled
            s.upload(raw, w0, shift)
            out = s.run()
            amp, info = s.fit()
            resid = s.residual()
        outs.append((out, amp, info, resid))
    (o1, a1, i1, r1), (o0, a0, i0, r0) = outs
    assert bits_equal(o1["weights"], z["weights_%d" % nit]) and bits_equal(o0["weights"], o1["weights"])
    assert o1["loops"] == o0["loops"] == int(z["loops"])
    assert bits_equal(a1, a0) and bits_equal(i1, i0)
    assert nan_equal(r1, r0)
