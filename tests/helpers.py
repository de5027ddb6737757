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
    raw = data[:, 0] if meta["npol"] == 1 else (data[:, 0] + data[:, 1]).astype(np.float32)
    return z, meta, np.ascontiguousarray(raw), w0, shift, meta["args"]


def bits_equal(a, b):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    return a.shape == b.shape and a.dtype == b.dtype and a.tobytes() == b.tobytes()


def nan_equal(a, b):
    return bool(np.all((a == b) | (np.isnan(a) & np.isnan(b))))
