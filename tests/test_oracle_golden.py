"""Pin the CPU oracle to the reference: every golden fixture was produced by
running /root/reference/iterative_cleaner.py itself (tests/golden/make_golden.py).
These run on CPU; they make the oracle a trustworthy checker for the GPU."""
import os

import numpy as np
import pytest

from helpers import (GOLDEN, bits_equal, bits_equal_nan, case_delay, case_kwargs, clean_fixtures, load_clean_case, long_stats_cases, nan_equal,
                     thresholds)


def test_leastsq_cases_bit_exact(oracle_lib):
    """orc_lmdif1 == scipy 1.15.3 leastsq (x and info) on edge-case profiles."""
    z = np.load(os.path.join(GOLDEN, "leastsq_cases.npz"))
    off = 0
    for k, n in enumerate(z["nbin"]):
        T = z["T"][off:off + n]
        p = z["p"][off:off + n]
        x, info, _ = oracle_lib.lmdif1(T, p)
        assert np.float64(x).tobytes() == np.float64(z["x"][k]).tobytes(), (k, n, x, z["x"][k])
        assert info == z["info"][k]
        amp, inf, R = oracle_lib.fit_residual(p[None], T)
        want = z["resid"][off:off + n].astype(np.float32)
        assert bits_equal(R[0], want)
        off += n


def test_leastsq_nonfinite_cases_bit_exact(oracle_lib):
    """NaN / Inf profiles and templates (scipy keeps x = 1, status 4) and exact
    large multiples of the template (status 8: the reference prints "Bad
    status" and zeroes the residual), against the reference's outputs."""
    z = np.load(os.path.join(GOLDEN, "leastsq_nonfinite.npz"))
    assert 8 in set(z["info"].tolist())
    off = 0
    for k, n in enumerate(z["nbin"]):
        T, p = z["T"][off:off + n], z["p"][off:off + n]
        x, info, _ = oracle_lib.lmdif1(T, p)
        assert np.float64(x).tobytes() == np.float64(z["x"][k]).tobytes(), (k, x, z["x"][k])
        assert info == z["info"][k], (k, info, z["info"][k])
        assert (str(z["stdout"][k]) != "") == (info not in (1, 2, 3, 4))
        _, _, R = oracle_lib.fit_residual(p[None], T)
        assert bits_equal(R[0], z["resid"][off:off + n].astype(np.float32)), k
        off += n


def test_pulse_region_cases(oracle_lib):
    z = np.load(os.path.join(GOLDEN, "pulse_region_cases.npz"))
    from iterative_cleaner_amd._native import normalise_pulse_region
    for i in range(3):
        pr = list(z["pr_%d" % i])
        on, fac, a, b = normalise_pulse_region(pr, len(z["T"]))
        amp, info, R = oracle_lib.fit_residual(z["p"][None], z["T"], (fac, a, b))
        assert bits_equal(R[0], z["resid_%d" % i].astype(np.float32))


def test_stats_cases_restated_bit_exact():
    """numpy restatement of comprehensive_stats == reference, all entries."""
    from oracle import restated as R
    z = np.load(os.path.join(GOLDEN, "stats_cases.npz"))
    for i in range(int(z["n"])):
        X, w = z["X_%d" % i], z["w_%d" % i]
        thr, isint = z["thr_%d" % i], z["thr_is_int_%d" % i]
        ct = int(thr[0]) if isint[0] else float(thr[0])
        st = int(thr[1]) if isint[1] else float(thr[1])
        t = R.comprehensive_stats(R.weighted_cube(X, w), w, ct, st)
        ref = z["test_%d" % i]
        assert bits_equal(np.where(np.isnan(t), 0, t), np.where(np.isnan(ref), 0, ref)), i
        assert np.array_equal(np.isnan(t), np.isnan(ref))


def test_stats_cases_c_oracle(oracle_lib):
    """C oracle stats == reference (std/mean/ptp exact; fftmax to 1e-9)."""
    from oracle import restated as R
    z = np.load(os.path.join(GOLDEN, "stats_cases.npz"))
    for i in range(int(z["n"])):
        X, w = z["X_%d" % i], z["w_%d" % i]
        thr = z["thr_%d" % i]
        Xw = R.weighted_cube(X, w)
        valid = w != 0
        sd, mn, pt, ff = oracle_lib.diagnostics(Xw, valid)
        rsd, rmn, rpt, rff = R.diagnostics(Xw, valid)
        assert bits_equal(sd, rsd) and bits_equal(mn, rmn) and bits_equal(pt, rpt)
        assert np.allclose(ff, rff, rtol=1e-9, atol=0, equal_nan=True)
        t = oracle_lib.test_values(valid, sd, mn, pt, ff, thr[0], thr[1])
        ref = z["test_%d" % i]
        fin = np.isfinite(ref)
        assert np.array_equal(np.isnan(t), np.isnan(ref))
        assert np.all(np.abs(t[fin] - ref[fin]) <= 1e-9 * np.maximum(1, np.abs(ref[fin])))
        assert np.array_equal((t >= 1), (ref >= 1))


def test_long_stats_cases_restated_and_c_oracle(oracle_lib):
    """nbin 512..4096 (the bench profile lengths): the numpy restatement and the
    C oracle reproduce the reference's comprehensive_stats — std/mean/ptp and
    the test values' zap decisions bit for bit, fftmax within 1e-9 relative."""
    from oracle import restated as R
    z, cases = long_stats_cases()
    for i, (X, w, _) in enumerate(cases):
        ct, st = thresholds(z, i)
        Xw = R.weighted_cube(X, w)
        valid = w != 0
        t = R.comprehensive_stats(Xw, w, ct, st)
        ref = z["test_%d" % i]
        assert bits_equal(np.where(np.isnan(t), 0, t), np.where(np.isnan(ref), 0, ref)), i
        sd, mn, pt, ff = oracle_lib.diagnostics(Xw, valid)
        for got, nm in ((sd, "std"), (mn, "mean"), (pt, "ptp")):
            want = z["diag_%s_%d" % (nm, i)]
            assert bits_equal(np.where(valid, got, 0), np.where(valid, want, 0).astype(got.dtype)), (i, nm)
        assert np.allclose(ff, z["diag_fft_%d" % i], rtol=1e-9, atol=0), i
        tc = oracle_lib.test_values(valid, sd, mn, pt, ff, ct, st)
        fin = np.isfinite(ref)
        assert np.array_equal(np.isnan(tc), np.isnan(ref))
        assert np.all(np.abs(tc[fin] - ref[fin]) <= 1e-9 * np.maximum(1, np.abs(ref[fin])))
        assert np.array_equal(tc >= 1, ref >= 1), i


def test_zap_plot_matches_reference(oracle_lib, tmp_path, monkeypatch):
    """-z (iterative_cleaner.py:164-171): the host plot of the oracle's test
    values is pixel-identical to the PNG the reference wrote."""
    import argparse

    import matplotlib.pyplot as plt

    from iterative_cleaner_amd import cleaner, synth
    z = np.load(os.path.join(GOLDEN, "zap_plot_case.npz"))
    data, w0, shift = synth.make_cube(8, 24, 64, 61, 0.2)
    out = oracle_lib.clean_loop(data[:, 0], w0, shift)
    monkeypatch.chdir(tmp_path)
    plt.close("all")
    cleaner._plot_zap(out["test"], "zap.ar", argparse.Namespace(chanthresh=5, subintthresh=5))
    img = plt.imread("zap.ar_5_5.png")
    plt.close("all")
    assert img.shape == z["image"].shape and np.array_equal(img, z["image"])


@pytest.mark.parametrize("path", clean_fixtures(), ids=lambda p: os.path.basename(p)[6:-4])
def test_clean_loop_c_oracle(path, oracle_lib):
    """Whole loop: templates, amps, info, weights, loops bit-exact vs clean()."""
    z, meta, raw, w0, shift, args = load_clean_case(path)
    pr = None if args["pulse_region"] == [0, 0, 1] else args["pulse_region"]
    if pr is not None:
        from iterative_cleaner_amd._native import normalise_pulse_region
        _, fac, a, b = normalise_pulse_region(pr, meta["nbin"])
        pr = (fac, a, b)
    out = oracle_lib.clean_loop(raw, w0, shift, args["chanthresh"], args["subintthresh"],
                                args["max_iter"], pr, want_details=True, data_f64=meta.get("data_f64", False),
                                **case_kwargs(z, meta))
    nit = int(z["n_iter"])
    assert out["loops"] == int(z["loops"])
    for k in range(1, nit + 1):
        assert bits_equal_nan(out["T"][k - 1], z["T_%d" % k]), "template of loop %d" % k
    assert bits_equal(out["amp"].ravel(), z["amp_%d" % nit])
    assert bits_equal(out["info"].ravel(), z["info_%d" % nit])
    assert bits_equal(out["weights"], z["weights_%d" % nit])
    assert bits_equal_nan(out["std"], z["diag_std_%d" % nit])
    assert bits_equal_nan(out["mean"], z["diag_mean_%d" % nit])
    assert bits_equal_nan(out["ptp"], z["diag_ptp_%d" % nit])
    ref = z["test_%d" % nit]
    fin = np.isfinite(ref)
    assert np.array_equal(np.isnan(out["test"]), np.isnan(ref))
    assert np.all(np.abs(out["test"][fin] - ref[fin]) <= 1e-9 * np.maximum(1, np.abs(ref[fin])))


def test_first_iteration_residual_and_diagnostics(oracle_lib):
    """Iteration-1 residual cube (f32, dedispersed) bit-exact on the small fixtures."""
    for path in clean_fixtures():
        z, meta, raw, w0, shift, args = load_clean_case(path)
        if "residual_ded_1" not in z.files or args["pulse_region"] != [0, 0, 1] or meta.get("frac_delay") \
                or meta.get("stored_dedispersed"):
            continue
        D = oracle_lib.fit_cube(raw, w0, shift)
        T = oracle_lib.template(raw, w0, shift)
        assert np.array_equal(z["residual_ded_1"].astype(np.float32), z["residual_ded_1"], equal_nan=True)
        assert bits_equal(T, z["T_1"])
        amp, info, R = oracle_lib.fit_residual(D.reshape(-1, meta["nbin"]), T)
        assert bits_equal(amp, z["amp_1"])
        # (an f64 get_data binding hands back the same f32 amplitudes, widened)
        assert bits_equal(R.reshape(raw.shape), z["residual_ded_1"].astype(np.float32))


def test_numpy_template_matches_c(oracle_lib):
    """archive stand-in (numpy) template ops == C restatement, incl. 2 super-blocks."""
    from iterative_cleaner_amd import archive as ica
    from iterative_cleaner_amd import synth
    data, w0, shift = synth.make_cube(5, 300, 64, 31, 0.2)
    w = w0.copy()
    w[1, 7] = 0.0
    w[3, 290] = 0.5
    ar = ica.Archive(data, w, shift)
    ar.pscrunch()
    ar.remove_baseline()
    ar.dedisperse()
    ar.fscrunch()
    ar.tscrunch()
    T_np = ar.get_Profile(0, 0, 0).get_amps() * 10000
    T_c = oracle_lib.template(data[:, 0], w, shift)
    assert bits_equal(T_np, T_c)


@pytest.mark.parametrize("name", ["s12x48x128", "s8x32x64_pol4", "s12x40x128_pr"])
def test_reference_like_cpu_baseline(name):
    """The CPU baseline timed by bench.py reproduces the reference's result."""
    from oracle import reference_like
    from iterative_cleaner_amd import archive as ica
    from iterative_cleaner_amd import synth
    z, meta, raw, w0, shift, args = load_clean_case(os.path.join(GOLDEN, "clean_%s.npz" % name))
    data, w0_, shift_ = synth.make_cube(meta["nsub"], meta["nchan"], meta["nbin"], meta["seed"],
                                        meta["rfi"], npol=meta["npol"])
    ar = ica.Archive(data, w0_, shift_)
    ar.pscrunch()
    test, weights, loops = reference_like.clean_loop(ar, args["chanthresh"], args["subintthresh"],
                                                     args["max_iter"], args["pulse_region"])
    nit = int(z["n_iter"])
    assert loops == int(z["loops"])
    assert bits_equal(weights, z["weights_%d" % nit])
    assert nan_equal(test, z["test_%d" % nit])


@pytest.mark.parametrize("nbin", [64, 100, 1024, 4096])
def test_closed_form_c_oracle_matches_numpy_statement(nbin, oracle_lib):
    """fit_mode 1's definition (oracle/restated.py closed_form_fit: numpy
    pairwise sums) and the C oracle agree bit for bit, including an all-zero
    template (a = 0), a zero profile and a NaN profile (status 5)."""
    from oracle import restated as R

    from iterative_cleaner_amd import synth
    data, w0, shift = synth.make_cube(4, 24, nbin, 5, 0.2)
    D = oracle_lib.fit_cube(data[:, 0], w0, shift).reshape(-1, nbin)
    D[3] = 0.0
    D[5, 7] = np.nan
    T = oracle_lib.template(data[:, 0], w0, shift)
    for k, TT in enumerate((T, np.zeros_like(T))):
        for sh in (None, shift):   # the dot in the stored (dispersed) order of each row's channel
            a1, i1, R1 = oracle_lib.fit_closed(D, TT, shift=sh)
            a2, i2, R2 = R.closed_form_fit(D, TT, shift=sh)
            assert bits_equal(a1, a2) and bits_equal(i1, i2) and bits_equal(R1, R2)
        if k == 0:
            assert i1[5] == 5 and not R1[5].any()
        else:
            assert not a1.any() and np.array_equal(R1, -D, equal_nan=True)
