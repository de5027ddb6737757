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


def load_clean_case(path):
    """(fixture npz, meta, raw total-intensity cube, w0, shift, args dict)."""
    z = np.load(path)
    meta = json.loads(str(z["meta"]))
    data, w0, shift = synth.make_cube(meta["nsub"], meta["nchan"], meta["nbin"], meta["seed"],
                                      meta["rfi"], npol=meta["npol"])
    assert hashlib.sha256(data.tobytes()).hexdigest() == str(z["input_sha256"]), \
        "synthetic generator drifted from the golden fixture"
    if meta.get("frac_weights"):
        w0 = synth.fractional_weights(w0)
    raw = data[:, 0] if meta["npol"] == 1 else (data[:, 0] + data[:, 1]).astype(np.float32)
    return z, meta, np.ascontiguousarray(raw), w0, shift, meta["args"]


def case_delay(z, meta):
    """The fractional per-channel delays of a fixture made with frac_delay (FFT
    phase-rotation dedispersion), else None (integer shifts)."""
    if not meta.get("frac_delay"):
        return None
    d = np.asarray(z["dm_delay"], dtype=np.float64)
    assert np.array_equal(d, synth.fractional_delays(synth.make_cube(1, meta["nchan"], meta["nbin"], 0, 0.0)[2],
                                                     meta["nbin"])), "delay generator drifted"
    return d


def bits_equal(a, b):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    return a.shape == b.shape and a.dtype == b.dtype and a.tobytes() == b.tobytes()


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
