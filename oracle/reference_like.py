"""Reference-like CPU loop — TEST INFRASTRUCTURE / CPU BASELINE ONLY.

A restatement of the reference cleaning loop (iterative_cleaner.py:83-146)
that makes the reference's own library calls, so its cost profile is the
reference's: per-profile ``scipy.optimize.leastsq`` (ic.py:275-288),
``numpy.ma`` diagnostics (ic.py:206-217) and per-line ``np.ma.median``
scalers (ic.py:229-256), on the repo's archive stand-in.  bench.py times it
as ``cpu_baseline`` (kind "port"); tests check it against the golden
fixtures.  Never imported by the product package.
"""
from __future__ import annotations

import numpy as np
import scipy.optimize


def _fit_profile(prof, template, pulse_region):
    """ic.py:275-288: leastsq of a*T - p from a = 1; bad status -> zeros."""
    resid = lambda a: a * template - prof  # noqa: E731
    a, status = scipy.optimize.leastsq(resid, [1.0])
    out = np.asarray(resid(a))
    if pulse_region != [0, 0, 1]:
        lo, hi = int(pulse_region[1]), int(pulse_region[2])
        out[lo:hi] = out[lo:hi] * pulse_region[0]
    if status not in (1, 2, 3, 4):
        return np.zeros_like(prof)
    return out


def _scaled(diag, axis, thresh):
    """|(x - median) / MAD| / thresh along lines of ``axis`` (ic.py:229-256, :222-223)."""
    out = np.empty_like(diag)
    nlines = diag.shape[1 - axis]
    for q in range(nlines):
        line = diag[:, q] if axis == 0 else diag[q, :]
        with np.errstate(invalid="ignore", divide="ignore"):
            dev = line - np.ma.median(line)
            val = dev / np.ma.median(np.abs(dev))
        if axis == 0:
            out[:, q] = val
        else:
            out[q, :] = val
    return np.abs(out) / thresh


def _test_values(data, chanthresh, subintthresh):
    """ic.py:181-226 on a masked (nsub, nchan, nbin) cube."""
    diags = (np.ma.std(data, axis=2), np.ma.mean(data, axis=2), np.ma.ptp(data, axis=2),
             np.max(np.abs(np.fft.rfft(data - np.expand_dims(data.mean(axis=2), axis=2),
                                       axis=2)), axis=2))
    per_diag = [np.max((_scaled(d, 0, chanthresh), _scaled(d, 1, subintthresh)), axis=0)
                for d in diags]
    return np.median(per_diag, axis=0)


def clean_loop(ar, chanthresh=5, subintthresh=5, max_iter=5, pulse_region=(0, 0, 1)):
    """Run the loop on a pscrunched stand-in Archive; returns (test, weights, loops)."""
    pulse_region = list(pulse_region)
    w_orig = ar.get_weights()
    history = [ar.get_weights()]
    nbin = ar.get_nbin()
    keep = w_orig.astype(bool)
    mask = np.repeat(~keep[:, :, None], nbin, axis=2)
    weights = w_orig
    test = None
    loops = None
    it = 0
    while it < max_iter:
        it += 1
        # template from the previous loop's weights (ic.py:88-94)
        tmpl_ar = ar.clone()
        for (s, c), w in np.ndenumerate(weights):
            tmpl_ar.get_Integration(s).set_weight(c, float(w))
        tmpl_ar.pscrunch()
        tmpl_ar.remove_baseline()
        tmpl_ar.dedisperse()
        tmpl_ar.fscrunch()
        tmpl_ar.tscrunch()
        template = tmpl_ar.get_Profile(0, 0, 0).get_amps() * 10000
        # fit cube (ic.py:96-101)
        fit_ar = ar.clone()
        fit_ar.pscrunch()
        fit_ar.remove_baseline()
        fit_ar.dedisperse()
        cube = fit_ar.get_data()[:, 0]
        for s in range(cube.shape[0]):
            for c in range(cube.shape[1]):
                fit_ar.get_Profile(s, 0, c).get_amps()[:] = _fit_profile(cube[s, c], template,
                                                                         pulse_region)
        fit_ar.dededisperse()
        data = fit_ar.get_data()[:, 0] * w_orig[:, :, None]
        test = _test_values(np.ma.masked_array(data.astype(np.float32), mask=mask),
                            chanthresh, subintthresh)
        weights = np.where(test >= 1, np.float32(0.0), w_orig).astype(np.float32)
        if any(np.all(weights == h) for h in history):
            loops = it
            it = 1000000
        history.append(weights)
    if it == max_iter:
        loops = max_iter
    return test, weights, loops
