"""Shared helpers for the parity tests (inputs regenerated from committed seeds)."""
import glob
import hashlib
import json
import os

import numpy as np

from iterative_cleaner_amd import synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def clean_fixtures():
    return sorted(glob.glob(os.path.join(GOLDEN, "clean_*.npz")))


def poke_cube(data, meta):
    """The non-finite samples a fixture placed in its synthetic data (make_golden.py poke)."""
    for s_, c_, b_, v_ in meta.get("poke", ()):
        data[s_, :, c_, b_] = float(v_)


def load_clean_case(path):
    """(fixture npz, meta, raw total-intensity cube, w0, shift, args dict)."""
    z = np.load(path)
    meta = json.loads(str(z["meta"]))
    data, w0, shift = synth.make_cube(meta["nsub"], meta["nchan"], meta["nbin"], meta["seed"],
                                      meta["rfi"], npol=meta["npol"])
    poke_cube(data, meta)
    assert hashlib.sha256(data.tobytes()).hexdigest() == str(z["input_sha256"]), \
        "synthetic generator drifted from the golden fixture"
    if meta.get("frac_weights"):
        w0 = synth.fractional_weights(w0)
    if meta.get("weights_zero"):
        w0 = np.zeros_like(w0)
    raw = data[:, 0] if meta["npol"] == 1 else (data[:, 0] + data[:, 1]).astype(np.float32)
    raw = np.ascontiguousarray(raw)
    if meta.get("stored_dedispersed") and meta.get("frac_delay"):
        # the archive as stored: dedispersed by the stand-in's FFT rotation; the
        # session takes it with input_dedispersed (case_kwargs).  (Integer
        # shifts: the host rolls a stored-dedispersed cube back exactly, so the
        # session's input is the dispersed synthetic cube itself.)
        from iterative_cleaner_amd import phase_rotation as pr
        d = case_delay(z, meta)
        raw = pr.rotate(raw, pr.phasors(meta["nbin"], d), 1)
    return z, meta, raw, w0, shift, meta["args"]


def case_delay(z, meta):
    """The fractional delays of a fixture made with frac_delay (FFT
    phase-rotation dedispersion): (nchan,), or (nsub, nchan) with frac_delay2
    (per-Integration periods); else None (integer shifts)."""
    if not meta.get("frac_delay"):
        return None
    d = np.asarray(z["dm_delay"], dtype=np.float64)
    shift = synth.make_cube(1, meta["nchan"], meta["nbin"], 0, 0.0)[2]
    want = synth.per_profile_delays(shift, meta["nbin"], meta["nsub"]) if meta.get("frac_delay2") \
        else synth.fractional_delays(shift, meta["nbin"])
    assert np.array_equal(d, want), "delay generator drifted"
    return d


def case_kwargs(z, meta):
    """Session keywords of a fixture's dedispersion: delay and input_dedispersed."""
    d = case_delay(z, meta)
    return dict(delay=d, input_dedispersed=bool(meta.get("stored_dedispersed")) and d is not None)


def bits_equal(a, b):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    return a.shape == b.shape and a.dtype == b.dtype and a.tobytes() == b.tobytes()


def bits_equal_nan(a, b):
    """bits_equal, except that a NaN matches any NaN: the sign and payload of a
    NaN that an invalid operation produces are the hardware's (x86's default
    NaN is negative, the GPU's positive), not part of numpy's semantics."""
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    na, nb = np.isnan(a), np.isnan(b)
    return bool(np.array_equal(na, nb)) and a[~na].tobytes() == b[~nb].tobytes()


def nan_equal(a, b):
    return bool(np.all((a == b) | (np.isnan(a) & np.isnan(b))))


def long_stats_cases():
    """The seeded comprehensive_stats inputs of tests/golden/stats_cases_long.npz
    (generator in make_golden.py; the fixture pins their hashes)."""
    import importlib
    import sys
    if GOLDEN not in sys.path:
        sys.path.insert(0, GOLDEN)
    mg = importlib.import_module("make_golden")
    z = np.load(os.path.join(GOLDEN, "stats_cases_long.npz"))
    cases = mg.long_stats_cases()
    for i, (X, w, _) in enumerate(cases):
        assert hashlib.sha256(np.ascontiguousarray(X).tobytes()).hexdigest() == str(z["X_sha256_%d" % i]), \
            "long stats generator drifted from the golden fixture (case %d)" % i
    return z, cases


def thresholds(z, i):
    """(chanthresh, subintthresh) of a stats fixture case, int where the reference had an int."""
    thr, isint = z["thr_%d" % i], z["thr_is_int_%d" % i]
    return (int(thr[0]) if isint[0] else float(thr[0]), int(thr[1]) if isint[1] else float(thr[1]))


def check_whole_loop(oracle_lib, raw, w0, shift, one, max_iter=5, residual=False, delay=None):
    """The whole cleaning loop of a full-size archive run independently by the
    (threaded) C oracle, compared with the GPU run `one` (ic_run + ic_get_fit /
    diagnostics / template [/ residual]) profile by profile: the loop count, the
    per-iteration change and zero counts, the final template, every profile's
    leastsq amplitude and status, std / mean / ptp and the weights bit for bit,
    fftmax within 1e-9 relative, and the test values - the oracle's own, from the
    oracle's diagnostics - within 1e-9 (only fftmax's last bits differ).  delay:
    the FFT dedispersion mode's fractional delays (orc_rotate).  The reference:
    iterative_cleaner.py:83-146 (fit :259-288, statistics :181-226)."""
    ref = oracle_lib.clean_loop(raw, w0, shift, max_iter=max_iter, want_details=True, want_residual=residual,
                                delay=delay)
    assert one["loops"] == ref["loops"] and one["n_iter"] == len(one["changed"])
    k = one["n_iter"]
    assert np.array_equal(one["changed"], ref["changed"][:k]), "changed weights per loop"
    assert np.array_equal(one["nzero"], ref["nzero"][:k]), "zero weights per loop"
    assert bits_equal(one["T"], ref["T"][k - 1]), "final template"
    assert bits_equal(one["amp"], ref["amp"]), "leastsq amplitudes (%d differ)" % int((one["amp"] != ref["amp"]).sum())
    assert bits_equal(one["info"], ref["info"]), "leastsq status"
    for name in ("std", "mean", "ptp"):
        a, b = one[name], ref[name]
        assert a.dtype == b.dtype and nan_equal(a, b), name
        fin = ~np.isnan(b)
        assert bits_equal(a[fin], b[fin]), name
    g, f = one["fft"], ref["fft"]
    assert np.all((g == f) | (np.abs(g - f) <= 1e-9 * np.abs(f)) | (np.isnan(g) & np.isnan(f))), "fftmax"
    t, u = one["test"], ref["test"]
    assert np.all((t == u) | (np.abs(t - u) <= 1e-9) | (np.isnan(t) & np.isnan(u))), "test values"
    assert bits_equal(one["weights"], ref["weights"]), "weights (%d differ)" % int((one["weights"] != ref["weights"]).sum())
    if residual:
        assert nan_equal(one["residual"], ref["residual"]), "residual cube (-u)"
    return ref
