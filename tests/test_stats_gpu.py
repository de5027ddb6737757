"""comprehensive_stats (iterative_cleaner.py:181-226) on the GPU through the
C-ABI entry ic_comprehensive_stats, against the outputs the REFERENCE itself
produced on the same inputs (tests/golden/stats_cases.npz: nbin 8..256 edge
cases; stats_cases_long.npz: nbin 512..4096, the bench profile lengths).
std / mean / ptp bit-exact; fftmax within 1e-9 relative (our FFT is not
pocketfft); test values within 1e-9 and the zap decisions (test >= 1) equal."""
import os

import numpy as np
import pytest

from helpers import GOLDEN, bits_equal, long_stats_cases, thresholds

pytestmark = pytest.mark.gpu


def _check(test, diags, ref_test, valid, ref_diags=None):
    fin = np.isfinite(ref_test)
    assert np.array_equal(np.isnan(test), np.isnan(ref_test))
    assert np.array_equal(np.isinf(test), np.isinf(ref_test))
    assert np.all(np.abs(test[fin] - ref_test[fin]) <= 1e-9 * np.maximum(1, np.abs(ref_test[fin])))
    assert np.array_equal(test >= 1, ref_test >= 1)
    if ref_diags is not None:
        sd, mn, pt, ff = diags
        for got, want in ((sd, ref_diags[0]), (mn, ref_diags[1]), (pt, ref_diags[2])):
            assert bits_equal(np.where(valid, got, 0), np.where(valid, want, 0).astype(got.dtype))
        assert np.allclose(ff, ref_diags[3], rtol=1e-9, atol=0)


def test_stats_cases_match_reference():
    from iterative_cleaner_amd import _native
    z = np.load(os.path.join(GOLDEN, "stats_cases.npz"))
    for i in range(int(z["n"])):
        X, w = z["X_%d" % i], z["w_%d" % i]
        ct, st = thresholds(z, i)
        test, diags = _native.comprehensive_stats(X, w, ct, st, diagnostics=True)
        _check(test, diags, z["test_%d" % i], w != 0)


def test_long_stats_cases_match_reference():
    from iterative_cleaner_amd import _native
    z, cases = long_stats_cases()
    for i, (X, w, _) in enumerate(cases):
        ct, st = thresholds(z, i)
        test, diags = _native.comprehensive_stats(X, w, ct, st, diagnostics=True)
        ref = tuple(z["diag_%s_%d" % (nm, i)] for nm in ("std", "mean", "ptp", "fft"))
        _check(test, diags, z["test_%d" % i], w != 0, ref)


@pytest.mark.parametrize("nbin", [100, 1000, 2048, 4096])
def test_stats_match_c_oracle_larger(nbin, oracle_lib):
    """Many profiles per line (real median/MAD selections) at the long profile
    lengths and two non-power-of-two ones (the generic kernel)."""
    from oracle import restated as R

    from iterative_cleaner_amd import _native
    rng = np.random.default_rng(nbin)
    nsub, nchan = 24, 70
    X = rng.standard_normal((nsub, nchan, nbin)).astype(np.float32)
    X[3, :, rng.integers(0, nbin, 7)] += 60
    X[:, 11, :] += (20 * np.sin(np.arange(nbin) * 0.3)).astype(np.float32)
    w = np.ones((nsub, nchan), np.float32)
    w[:, 5] = 0
    w[7, 9] = 0.5
    test, diags = _native.comprehensive_stats(X, w, 5, 5, diagnostics=True)
    Xw = R.weighted_cube(X, w)
    sd, mn, pt, ff = oracle_lib.diagnostics(Xw, w != 0)
    ref = oracle_lib.test_values(w != 0, sd, mn, pt, ff, 5, 5)
    _check(test, diags, ref, w != 0, (sd, mn, pt, ff))


@pytest.mark.parametrize("grp", ["0", "4", "8"])
def test_line_medians_per_block_match(grp, oracle_lib):
    """The per-line median/MAD in its two forms: one wave per line, and a block
    of W waves per line (k_linestats_grp, taken by default for few lines of
    >= 1024 values; rowstat_minlen=1 forces it onto every line here).
    Both must reproduce the reference's selections: the edge cases of
    stats_cases.npz (NaN, empty, tied lines), and long rows (nchan 3000) with
    ties, zapped entries and outliers against the C oracle."""
    from oracle import restated as R

    from iterative_cleaner_amd import _native
    opt = dict(rowstat_waves=int(grp), rowstat_minlen=1)
    z = np.load(os.path.join(GOLDEN, "stats_cases.npz"))
    for i in range(int(z["n"])):
        X, w = z["X_%d" % i], z["w_%d" % i]
        ct, st = thresholds(z, i)
        test, diags = _native.comprehensive_stats(X, w, ct, st, diagnostics=True, **opt)
        _check(test, diags, z["test_%d" % i], w != 0)
    rng = np.random.default_rng(77)
    for nsub, nchan, nbin in ((5, 3000, 32), (3, 1999, 16)):
        X = rng.standard_normal((nsub, nchan, nbin)).astype(np.float32)
        X[:, ::7, :] = np.round(X[:, ::7, :])           # ties
        X[1, rng.integers(0, nchan, 40), :] += 80       # outliers
        w = np.ones((nsub, nchan), np.float32)
        w[:, rng.integers(0, nchan, 200)] = 0
        w[2, :nchan // 2] = 0                           # a half-zapped row
        test, diags = _native.comprehensive_stats(X, w, 5, 5, diagnostics=True, **opt)
        Xw = R.weighted_cube(X, w)
        sd, mn, pt, ff = oracle_lib.diagnostics(Xw, w != 0)
        ref = oracle_lib.test_values(w != 0, sd, mn, pt, ff, 5, 5)
        _check(test, diags, ref, w != 0, (sd, mn, pt, ff))
