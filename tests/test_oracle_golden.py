"""Pin the CPU oracle to the reference: every golden fixture was produced by
running /root/reference/iterative_cleaner.py itself (tests/golden/make_golden.py).
These run on CPU; they make the oracle a trustworthy checker for the GPU."""
import os

import numpy as np
import pytest

from helpers import GOLDEN, bits_equal, clean_fixtures, load_clean_case, nan_equal


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
                                args["max_iter"], pr, want_details=True)
    nit = int(z["n_iter"])
    assert out["loops"] == int(z["loops"])
    for k in range(1, nit + 1):
        assert bits_equal(out["T"][k - 1], z["T_%d" % k]), "template of loop %d" % k
    assert bits_equal(out["amp"].ravel(), z["amp_%d" % nit])
    assert bits_equal(out["info"].ravel(), z["info_%d" % nit])
    assert bits_equal(out["weights"], z["weights_%d" % nit])
    assert bits_equal(out["std"], z["diag_std_%d" % nit])
    assert bits_equal(out["mean"], z["diag_mean_%d" % nit])
    assert bits_equal(out["ptp"], z["diag_ptp_%d" % nit])
    ref = z["test_%d" % nit]
    fin = np.isfinite(ref)
    assert np.array_equal(np.isnan(out["test"]), np.isnan(ref))
    assert np.all(np.abs(out["test"][fin] - ref[fin]) <= 1e-9 * np.maximum(1, np.abs(ref[fin])))


def test_first_iteration_residual_and_diagnostics(oracle_lib):
    """Iteration-1 residual cube (f32, dedispersed) bit-exact on the small fixtures."""
    for path in clean_fixtures():
        z, meta, raw, w0, shift, args = load_clean_case(path)
        if "residual_ded_1" not in z.files or args["pulse_region"] != [0, 0, 1]:
            continue
        D = oracle_lib.fit_cube(raw, w0, shift)
        T = oracle_lib.template(raw, w0, shift)
        assert bits_equal(T, z["T_1"])
        amp, info, R = oracle_lib.fit_residual(D.reshape(-1, meta["nbin"]), T)
        assert bits_equal(amp, z["amp_1"])
        assert bits_equal(R.reshape(raw.shape), z["residual_ded_1"])


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
