#!/usr/bin/env python
"""Generate golden fixtures by running the REFERENCE implementation.

Runs only in the build container (``/root/reference`` is absent on the GPU
box).  The reference ``iterative_cleaner.py`` is imported with a stub
``psrchive`` module whose ``Archive_load`` is this repo's NumPy stand-in
(``iterative_cleaner_amd.archive``); nothing of the reference is copied.
Its own functions are instrumented (wrapped, not modified) to record the
per-iteration intermediates of ``clean()`` (iterative_cleaner.py:65-178):

  T (template, :94), leastsq (x, info) per profile (:278), the f32
  residual cube (:101), the weighted masked cube's diagnostics
  (:206-217), channel/subint-scaled diagnostics (:222-223), test (:225),
  weights after set_weights_archive (:125), loops and stdout.

Also recorded: direct calls of ``comprehensive_stats`` on edge-case inputs
and of ``scipy.optimize.leastsq`` through ``remove_profile1d`` on edge-case
profiles.  Output: ``tests/golden/*.npz`` (plain arrays, no pickles).

usage: python tests/golden/make_golden.py [--out tests/golden]
"""
from __future__ import annotations

import argparse
import contextlib
import hashlib
import io
import json
import os
import sys
import tempfile
import types

sys.dont_write_bytecode = True
os.environ.setdefault("MPLBACKEND", "Agg")

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

import numpy as np                                   # noqa: E402
import scipy.optimize                                # noqa: E402

from iterative_cleaner_amd import archive as ica     # noqa: E402
from iterative_cleaner_amd import synth              # noqa: E402

REF_DIR = "/root/reference"


def import_reference():
    stub = types.ModuleType("psrchive")
    stub.Archive_load = ica.Archive_load
    sys.modules["psrchive"] = stub
    if REF_DIR not in sys.path:
        sys.path.insert(0, REF_DIR)
    import iterative_cleaner as ic  # noqa: WPS433  (reference, read-only)
    return ic


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def ref_args(ic, extra=()):
    old = sys.argv
    try:
        sys.argv = ["iterative_cleaner.py", "dummy.ar", *extra]
        return ic.parse_arguments()
    finally:
        sys.argv = old


class Recorder:
    """Wrap the reference's own functions to capture intermediates."""

    def __init__(self, ic):
        self.ic = ic
        self.iters = []
        self._cur = None
        self._orig = {}

    def __enter__(self):
        ic = self.ic
        for name in ("remove_profile_inplace", "comprehensive_stats",
                     "set_weights_archive", "channel_scaler", "subint_scaler"):
            self._orig[name] = getattr(ic, name)
        self._orig["leastsq"] = scipy.optimize.leastsq
        rec = self

        def leastsq(func, x0, *a, **k):
            res = rec._orig["leastsq"](func, x0, *a, **k)
            if rec._cur is not None:
                rec._cur["amp"].append(float(np.asarray(res[0])[0]))
                rec._cur["info"].append(int(res[1]))
            return res

        def remove_profile_inplace(ar, template, pulse_region):
            rec._cur = {"T": np.array(template, dtype=np.float32), "amp": [], "info": []}
            out = rec._orig["remove_profile_inplace"](ar, template, pulse_region)
            rec._cur["residual_ded"] = ar.get_data()[:, 0].copy()
            return out

        def comprehensive_stats(data, args, axis):
            cur = rec._cur
            cur["X"] = np.ma.getdata(data).copy()
            cur["X_mask"] = np.ma.getmaskarray(data)[:, :, 0].copy()
            diags = [np.ma.std(data, axis=2), np.ma.mean(data, axis=2),
                     np.ma.ptp(data, axis=2),
                     np.max(np.abs(np.fft.rfft(
                         data - np.expand_dims(data.mean(axis=2), axis=2), axis=2)), axis=2)]
            for nm, d in zip(("std", "mean", "ptp", "fft"), diags):
                cur["diag_" + nm] = np.ma.getdata(d).copy()
                cur["diag_" + nm + "_mask"] = np.ma.getmaskarray(d).copy()
                cs = rec._orig["channel_scaler"](d)
                ss = rec._orig["subint_scaler"](d)
                cur["chan_" + nm] = np.ma.getdata(cs).copy()
                cur["sub_" + nm] = np.ma.getdata(ss).copy()
            out = rec._orig["comprehensive_stats"](data, args, axis)
            cur["test"] = np.asarray(out).copy()
            return out

        def set_weights_archive(archive, test_results):
            out = rec._orig["set_weights_archive"](archive, test_results)
            if rec._cur is not None and "test" in rec._cur and "weights" not in rec._cur:
                rec._cur["weights"] = archive.get_weights().copy()
                rec.iters.append(rec._cur)
                rec._cur = None
            return out

        ic.remove_profile_inplace = remove_profile_inplace
        ic.comprehensive_stats = comprehensive_stats
        ic.set_weights_archive = set_weights_archive
        scipy.optimize.leastsq = leastsq
        return self

    def __exit__(self, *exc):
        for name, fn in self._orig.items():
            if name == "leastsq":
                scipy.optimize.leastsq = fn
            else:
                setattr(self.ic, name, fn)
        return False


def _load_f64(path):
    """The stand-in as a psrchive build whose get_data returns f64."""
    ar = ica.Archive_load(path)
    ar.get_data_dtype = np.float64
    return ar


def run_clean_case(ic, name, nsub, nchan, nbin, seed, rfi, extra_args=(),
                   keep_cubes=True, npol=1, workdir=None, out_dir=HERE, residual_full=True, data_f64=False,
                   frac_weights=False, frac_delay=False, poke=(), weights_zero=False, frac_delay2=False,
                   stored_dedispersed=False):
    data, weights, shift = synth.make_cube(nsub, nchan, nbin, seed, rfi, npol=npol)
    if weights_zero:                  # every profile zapped before the first loop
        weights = np.zeros_like(weights)
    for (s_, c_, b_, v_) in poke:      # non-finite samples placed in the data
        data[s_, :, c_, b_] = v_
    if frac_weights:
        weights = synth.fractional_weights(weights)
    path = os.path.join(workdir, "%s.ar" % name)
    delay = synth.fractional_delays(shift, nbin) if frac_delay else None
    if frac_delay2:            # per-(subint, channel): psrchive's per-Integration folding period
        frac_delay = True
        delay = synth.per_profile_delays(shift, nbin, nsub)
    ar = ica.Archive(data, weights, shift, filename=path, dm_delay=delay)
    if stored_dedispersed:     # the archive is stored dedispersed: its dedisperse is a no-op
        ar.dedisperse()
    ar.unload(path)
    loader = _load_f64 if data_f64 else ica.Archive_load
    ar = loader(path)
    args = ref_args(ic, ["-l", *extra_args])
    buf = io.StringIO()
    cwd = os.getcwd()
    os.chdir(workdir)
    stub = sys.modules["psrchive"]
    stub.Archive_load = loader          # the reference's reload (:150) sees the same binding
    try:
        with Recorder(ic) as rec, contextlib.redirect_stdout(buf):
            out_ar = ic.clean(ar, args, path)
    finally:
        stub.Archive_load = ica.Archive_load
        os.chdir(cwd)
    stdout = buf.getvalue()
    loops = None
    for line in stdout.splitlines():
        if line.startswith("RFI removal stops after"):
            loops = int(line.split()[-2])
        if line.startswith("Cleaning was interrupted"):
            loops = int(line.split("(")[-1].rstrip(")"))
    arrays = {
        "input_sha256": np.array(sha(data)),
        "final_weights": out_ar.get_weights(),
        "stdout": np.array(stdout),
        "n_iter": np.array(len(rec.iters)),
        "loops": np.array(loops if loops is not None else -1),
        "meta": np.array(json.dumps({
            "name": name, "nsub": nsub, "nchan": nchan, "nbin": nbin, "seed": seed,
            "rfi": rfi, "npol": npol, "extra_args": list(extra_args), "data_f64": bool(data_f64),
            "frac_weights": bool(frac_weights), "frac_delay": bool(frac_delay),
            **({"frac_delay2": True} if frac_delay2 else {}),
            **({"stored_dedispersed": True} if stored_dedispersed else {}),
            "args": {k: v for k, v in vars(args).items() if k != "archive"},
            "numpy": np.__version__, "scipy": scipy.__version__,
            **({"poke": [[int(a_), int(b_), int(c_), repr(float(v_))] for (a_, b_, c_, v_) in poke]}
               if poke else {}),
            **({"weights_zero": True} if weights_zero else {})})),
    }
    for k, it in enumerate(rec.iters, start=1):
        arrays["T_%d" % k] = it["T"]
        arrays["amp_%d" % k] = np.array(it["amp"], dtype=np.float64)
        arrays["info_%d" % k] = np.array(it["info"], dtype=np.int32)
        arrays["test_%d" % k] = it["test"]
        arrays["weights_%d" % k] = it["weights"]
        for nm in ("std", "mean", "ptp", "fft"):
            arrays["diag_%s_%d" % (nm, k)] = it["diag_" + nm]
            arrays["diag_%s_mask_%d" % (nm, k)] = it["diag_" + nm + "_mask"]
            if keep_cubes:
                arrays["chan_%s_%d" % (nm, k)] = it["chan_" + nm]
                arrays["sub_%s_%d" % (nm, k)] = it["sub_" + nm]
        if keep_cubes and k == 1:
            arrays["residual_ded_%d" % k] = it["residual_ded"]
            arrays["X_%d" % k] = it["X"]
        else:
            arrays["residual_ded_sha_%d" % k] = np.array(sha(it["residual_ded"]))
            arrays["X_sha_%d" % k] = np.array(sha(it["X"]))
    if frac_delay:
        arrays["dm_delay"] = delay
    if "-u" in extra_args:
        # the residual archive the reference unloads (iterative_cleaner.py:106-108, :161-162)
        res = ica.Archive_load("%s_residual_%s.ar" % (path, loops))
        rdata = res.get_data()
        arrays["residual_sha256"] = np.array(sha(rdata))
        arrays["residual_weights"] = res.get_weights()
        arrays["residual_shape"] = np.array(rdata.shape)
        if residual_full:
            arrays["residual_data"] = rdata
        else:
            arrays["residual_subint0"] = rdata[0]
    fn = os.path.join(out_dir, "clean_%s.npz" % name)
    np.savez_compressed(fn, **arrays)
    print("wrote %s  iters=%d loops=%s" % (fn, len(rec.iters), loops))


def stats_cases(rng):
    """Edge-case inputs for comprehensive_stats (iterative_cleaner.py:181-226)."""
    cases = []
    for ci in range(24):
        nsub = int(rng.integers(3, 14))
        nchan = int(rng.integers(4, 30))
        nbin = int(rng.choice([8, 16, 24, 64, 100, 128, 136, 256]))
        X = rng.standard_normal((nsub, nchan, nbin)).astype(np.float32)
        X *= np.float32(10.0 ** rng.uniform(-3, 3))
        w = np.ones((nsub, nchan), np.float32)
        kind = ci % 8
        if kind == 1:      # zero-weight channels and subints
            w[:, rng.integers(0, nchan)] = 0
            w[rng.integers(0, nsub), :] = 0
        if kind == 2:      # dead all-zero channel with weight 1
            X[:, rng.integers(0, nchan), :] = 0
        if kind == 3:      # fractional weights
            w = rng.choice([0.0, 0.25, 0.5, 1.0, 1.5], size=(nsub, nchan)).astype(np.float32)
        if kind == 4:      # many identical profiles -> MAD == 0 lines
            X[:, :, :] = X[0:1, 0:1, :]
            X[rng.integers(0, nsub), rng.integers(0, nchan)] += 3
        if kind == 5:      # strong RFI outliers
            X[rng.integers(0, nsub, 4), rng.integers(0, nchan, 4)] *= 50
        if kind == 6:      # more than half of a channel zero-weight
            c = rng.integers(0, nchan)
            w[: nsub // 2 + 1, c] = 0
        if kind == 7:      # quantised data (ties in medians)
            X = np.round(X * 2) / 2
            X = X.astype(np.float32)
        thr = [(5, 5), (3.0, 3.0), (1.5, 4.0), (5, 2.5)][ci % 4]
        cases.append((X, w, thr))
    return cases


def run_stats_cases(ic, out_dir=HERE):
    rng = np.random.default_rng(12345)
    arrays = {}
    for i, (X, w, (ct, st)) in enumerate(stats_cases(rng)):
        args = argparse.Namespace(chanthresh=ct, subintthresh=st)
        data = X.copy()
        data = ic.apply_weights(data, w)
        mask = np.bitwise_not(np.expand_dims(w, 2).astype(bool)).repeat(X.shape[2], axis=2)
        mdata = np.ma.masked_array(data, mask=mask)
        with np.errstate(all="ignore"):
            test = ic.comprehensive_stats(mdata, args, axis=2)
        arrays["X_%d" % i] = X
        arrays["w_%d" % i] = w
        arrays["thr_%d" % i] = np.array([ct, st], dtype=np.float64)
        arrays["thr_is_int_%d" % i] = np.array([isinstance(ct, int), isinstance(st, int)])
        arrays["test_%d" % i] = np.asarray(test)
    arrays["n"] = np.array(len(stats_cases(np.random.default_rng(12345))))
    fn = os.path.join(out_dir, "stats_cases.npz")
    np.savez_compressed(fn, **arrays)
    print("wrote", fn)


LONG_NBINS = (512, 1024, 2048, 4096)


def long_stats_cases():
    """comprehensive_stats inputs at the bench profile lengths (nbin 512..4096):
    regenerated from this seeded generator by the tests (the fixture keeps the
    input hashes and the reference's outputs, not the 0.1-1 MB inputs)."""
    cases = []
    for ni, nbin in enumerate(LONG_NBINS):
        for kind in range(5):
            rng = np.random.default_rng(9000 + 10 * ni + kind)
            nsub = int(rng.integers(3, 8))
            nchan = int(rng.integers(4, 12))
            X = rng.standard_normal((nsub, nchan, nbin)).astype(np.float32)
            X *= np.float32(10.0 ** rng.uniform(-2, 2))
            w = np.ones((nsub, nchan), np.float32)
            if kind == 1:      # zero-weight channel + subint, fractional weights
                w[:, rng.integers(0, nchan)] = 0
                w[rng.integers(0, nsub), :] = 0
                w[rng.integers(0, nsub), rng.integers(0, nchan)] = 0.5
            if kind == 2:      # narrowband sinusoid (FFT maximum off DC), dead channel
                ph = (np.arange(nbin) + 0.5) / nbin
                X[:, 1, :] += (30 * np.sin(2 * np.pi * 17.0 * ph)).astype(np.float32)
                X[:, 2, :] = 0
            if kind == 3:      # impulsive spikes (ptp / mean outliers)
                X[rng.integers(0, nsub), :, rng.integers(0, nbin, 9)] += 200
            if kind == 4:      # quantised (ties in medians, exact sums)
                X = (np.round(X * 4) / 4).astype(np.float32)
            thr = [(5, 5), (3.0, 3.0), (1.5, 4.0), (5, 2.5), (5, 5)][kind]
            cases.append((X, w, thr))
    return cases


def run_long_stats_cases(ic, out_dir=HERE):
    arrays = {}
    cases = long_stats_cases()
    for i, (X, w, (ct, st)) in enumerate(cases):
        args = argparse.Namespace(chanthresh=ct, subintthresh=st)
        data = ic.apply_weights(X.copy(), w)
        mask = np.bitwise_not(np.expand_dims(w, 2).astype(bool)).repeat(X.shape[2], axis=2)
        mdata = np.ma.masked_array(data, mask=mask)
        with np.errstate(all="ignore"):
            test = ic.comprehensive_stats(mdata, args, axis=2)
            diags = [np.ma.std(mdata, axis=2), np.ma.mean(mdata, axis=2), np.ma.ptp(mdata, axis=2),
                     np.max(np.abs(np.fft.rfft(
                         mdata - np.expand_dims(mdata.mean(axis=2), axis=2), axis=2)), axis=2)]
        arrays["X_sha256_%d" % i] = np.array(sha(X))
        arrays["w_%d" % i] = w
        arrays["thr_%d" % i] = np.array([ct, st], dtype=np.float64)
        arrays["thr_is_int_%d" % i] = np.array([isinstance(ct, int), isinstance(st, int)])
        arrays["test_%d" % i] = np.asarray(test)
        for nm, d in zip(("std", "mean", "ptp", "fft"), diags):
            arrays["diag_%s_%d" % (nm, i)] = np.ma.getdata(d).copy()
    arrays["n"] = np.array(len(cases))
    fn = os.path.join(out_dir, "stats_cases_long.npz")
    np.savez_compressed(fn, **arrays)
    print("wrote", fn)


def run_zap_plot_case(ic, out_dir=HERE):
    """clean() with -z: the reference's zap PNG (iterative_cleaner.py:164-171)."""
    import matplotlib.pyplot as plt
    with tempfile.TemporaryDirectory() as wd:
        data, weights, shift = synth.make_cube(8, 24, 64, 61, 0.2)
        path = "zap.ar"                      # relative: the plot title carries the name
        args = ref_args(ic, ["-l", "-q", "-z"])
        cwd = os.getcwd()
        os.chdir(wd)
        plt.close("all")
        try:
            ica.Archive(data, weights, shift, filename=path).unload(path)
            ic.clean(ica.Archive_load(path), args, path)
            img = plt.imread("%s_%s_%s.png" % (path, args.chanthresh, args.subintthresh))
        finally:
            os.chdir(cwd)
        plt.close("all")
        np.savez_compressed(os.path.join(out_dir, "zap_plot_case.npz"), image=img,
                            input_sha256=np.array(sha(data)))
        print("wrote zap_plot_case.npz", img.shape)


def leastsq_cases(rng):
    cases = []
    for nbin in (64, 128, 256, 1024, 4096):
        reps = {64: 60, 128: 60, 256: 60, 1024: 20, 4096: 8}[nbin]
        phase = (np.arange(nbin) + 0.5) / nbin
        pulse = np.exp(-0.5 * ((phase - 0.3) / 0.02) ** 2)
        for r in range(reps):
            T = (pulse * 10000 * rng.gamma(2, 0.5)).astype(np.float32)
            p = (rng.gamma(2, 0.5) * pulse + rng.standard_normal(nbin)).astype(np.float32)
            kind = r % 12
            if kind == 1: p = np.zeros(nbin, np.float32)
            if kind == 2: T = np.zeros(nbin, np.float32)
            if kind == 3: p = np.full(nbin, 3.25, np.float32)
            if kind == 4: p = (T * np.float32(rng.uniform(-2, 2))).astype(np.float32)
            if kind == 5: p = (p * np.float32(10.0 ** rng.uniform(-6, 6))).astype(np.float32)
            if kind == 6: T = (T * np.float32(10.0 ** rng.uniform(-6, 6))).astype(np.float32)
            if kind == 7: p = (T * np.float32(1e-7) + p * np.float32(1e-12)).astype(np.float32)
            if kind == 8: T = rng.standard_normal(nbin).astype(np.float32)
            if kind == 9: p[rng.integers(0, nbin, 5)] += 1e4
            if kind == 10: T = (T - T.mean()).astype(np.float32)
            if kind == 11:
                T = np.zeros(nbin, np.float32)
                T[rng.integers(0, nbin)] = 1.0
            cases.append((T, p))
    return cases


def run_leastsq_cases(ic, out_dir=HERE):
    rng = np.random.default_rng(777)
    Ts, ps, xs, infos, resid = [], [], [], [], []
    for T, p in leastsq_cases(rng):
        rec = {}
        orig = scipy.optimize.leastsq

        def spy(func, x0, *a, **k):
            res = orig(func, x0, *a, **k)
            rec["x"], rec["info"] = float(np.asarray(res[0])[0]), int(res[1])
            return res
        scipy.optimize.leastsq = spy
        try:
            with contextlib.redirect_stdout(io.StringIO()), np.errstate(all="ignore"):
                _, r = ic.remove_profile1d(p, 0, 0, T, [0, 0, 1])
        finally:
            scipy.optimize.leastsq = orig
        Ts.append(T); ps.append(p); xs.append(rec["x"]); infos.append(rec["info"])
        resid.append(np.asarray(r, dtype=np.float64))
    arrays = {"x": np.array(xs), "info": np.array(infos, np.int32)}
    sizes = np.array([len(t) for t in Ts])
    arrays["nbin"] = sizes
    arrays["T"] = np.concatenate(Ts)
    arrays["p"] = np.concatenate(ps)
    arrays["resid"] = np.concatenate(resid)
    fn = os.path.join(out_dir, "leastsq_cases.npz")
    np.savez_compressed(fn, **arrays)
    print("wrote %s (%d profiles)" % (fn, len(xs)))


def leastsq_nonfinite_cases():
    """Profiles outside the usual range: non-finite samples (NaN / +-Inf in the
    profile or the template) and exact large multiples of the template, for
    which scipy's leastsq returns status 8 (the reference then prints "Bad
    status ..." and zeroes the residual, iterative_cleaner.py:284-286)."""
    cases = []
    rng = np.random.default_rng(4711)
    for nbin in (64, 256, 1024):
        phase = (np.arange(nbin) + 0.5) / nbin
        pulse = np.exp(-0.5 * ((phase - 0.3) / 0.02) ** 2)
        T = (pulse * 1.3e4).astype(np.float32)
        noise = rng.standard_normal(nbin).astype(np.float32)
        for kind in range(14):
            t, p = T.copy(), noise.copy()
            if kind == 0: p[5] = np.nan
            if kind == 1: p[nbin // 3] = np.inf
            if kind == 2: p[nbin // 2] = -np.inf
            if kind == 3: p[:] = np.nan
            if kind == 4: t[7] = np.nan
            if kind == 5: t[nbin // 3] = np.inf
            if kind == 6: p = (T * np.float32(1e12)).astype(np.float32)
            if kind == 7: p = (T * np.float32(-4.1e11)).astype(np.float32)
            if kind == 12: p = (T * np.float32(1e13)).astype(np.float32)
            if kind == 13: p = (T * np.float32(1e11)).astype(np.float32)
            if kind == 8: p = (T * np.float32(1e10)).astype(np.float32); p[3] += np.float32(1e-3)
            if kind == 9: t = (pulse * 1.6e-11).astype(np.float32); p = (t * np.float32(6.8e10)).astype(np.float32)
            if kind == 10: t = (pulse * 3.4e4).astype(np.float32); p = (t * np.float32(2.8e11)).astype(np.float32)
            if kind == 11: p = np.full(nbin, np.float32(3e38)); p[::2] = np.float32(-3e38)
            cases.append((t, p))
    return cases


def run_leastsq_nonfinite(ic, out_dir=HERE):
    Ts, ps, xs, infos, resid, printed = [], [], [], [], [], []
    for T, p in leastsq_nonfinite_cases():
        rec = {}
        orig = scipy.optimize.leastsq

        def spy(func, x0, *a, **k):
            res = orig(func, x0, *a, **k)
            rec["x"], rec["info"] = float(np.asarray(res[0])[0]), int(res[1])
            return res
        scipy.optimize.leastsq = spy
        buf = io.StringIO()
        try:
            with contextlib.redirect_stdout(buf), np.errstate(all="ignore"):
                _, r = ic.remove_profile1d(p, 0, 0, T, [0, 0, 1])
        finally:
            scipy.optimize.leastsq = orig
        Ts.append(T); ps.append(p); xs.append(rec["x"]); infos.append(rec["info"])
        resid.append(np.asarray(r, dtype=np.float64))
        printed.append(buf.getvalue())
    arrays = {"x": np.array(xs), "info": np.array(infos, np.int32), "nbin": np.array([len(t) for t in Ts]),
              "T": np.concatenate(Ts), "p": np.concatenate(ps), "resid": np.concatenate(resid),
              "stdout": np.array(printed)}
    fn = os.path.join(out_dir, "leastsq_nonfinite.npz")
    np.savez_compressed(fn, **arrays)
    import collections
    print("wrote %s (%d profiles, statuses %s)" % (fn, len(xs), dict(collections.Counter(infos))))


def run_pulse_region_case(ic, out_dir=HERE):
    """remove_profile1d with an active pulse region (K6: (factor, start, end))."""
    rng = np.random.default_rng(4242)
    nbin = 128
    T = (np.exp(-0.5 * (((np.arange(nbin) + .5) / nbin - .3) / .02) ** 2) * 1e4).astype(np.float32)
    p = (0.7 * T / 1e4 + rng.standard_normal(nbin)).astype(np.float32)
    out = {}
    for i, pr in enumerate(([0.5, 30.0, 50.0], [0.0, 10.0, 20.0], [2.0, 100.0, 300.0])):
        with contextlib.redirect_stdout(io.StringIO()):
            _, r = ic.remove_profile1d(p, 0, 0, T, pr)
        out["pr_%d" % i] = np.array(pr)
        out["resid_%d" % i] = np.asarray(r, dtype=np.float64)
    out["T"], out["p"] = T, p
    fn = os.path.join(out_dir, "pulse_region_cases.npz")
    np.savez_compressed(fn, **out)
    print("wrote", fn)


def run_cli_case(ic, out_dir=HERE):
    """main() end to end: output naming, final weights, bad parts, log/no-log."""
    with tempfile.TemporaryDirectory() as wd:
        data, weights, shift = synth.make_cube(10, 40, 128, 21, 0.2)
        path = os.path.join(wd, "cli.ar")
        ica.Archive(data, weights, shift, filename=path).unload(path)
        buf = io.StringIO()
        old = sys.argv
        cwd = os.getcwd()
        os.chdir(wd)
        try:
            sys.argv = ["iterative_cleaner.py", "-l", "--bad_chan", "0.3",
                        "--bad_subint", "0.3", "-c", "3", "-s", "3", path]
            with contextlib.redirect_stdout(buf):
                ic.main(ic.parse_arguments())
        finally:
            sys.argv = old
            os.chdir(cwd)
        outp = os.path.join(wd, "cli_cleaned.ar")
        out_ar = ica.Archive_load(outp)
        np.savez_compressed(os.path.join(out_dir, "cli_case.npz"),
                            weights=out_ar.get_weights(),
                            stdout=np.array(buf.getvalue().replace(wd, "<WD>")),
                            input_sha256=np.array(sha(data)))
        print("wrote cli_case.npz")


def run_cli_std_name_case(ic, out_dir=HERE):
    """main() with -o std -q (round 4): the NAME.FREQ.MJD.ar output name
    (iterative_cleaner.py:52-56) and its weights."""
    with tempfile.TemporaryDirectory() as wd:
        data, weights, shift = synth.make_cube(5, 16, 64, 24, 0.2)
        path = os.path.join(wd, "std.ar")
        ica.Archive(data, weights, shift, filename=path).unload(path)
        old = sys.argv
        cwd = os.getcwd()
        os.chdir(wd)
        try:
            sys.argv = ["iterative_cleaner.py", "-l", "-q", "-o", "std", path]
            ic.main(ic.parse_arguments())
        finally:
            sys.argv = old
            os.chdir(cwd)
        names = sorted(f for f in os.listdir(wd) if f != "std.ar")
        assert len(names) == 1, names
        out_ar = ica.Archive_load(os.path.join(wd, names[0]))
        np.savez_compressed(os.path.join(out_dir, "cli_std_name_case.npz"), name=np.array(names[0]),
                            weights=out_ar.get_weights(), input_sha256=np.array(sha(data)))
        print("wrote cli_std_name_case.npz (%s)" % names[0])


def run_cli_memory_case(ic, out_dir=HERE):
    """main() with --memory and -o on a 4-pol archive (round 4): clean() does not
    pscrunch the archive in memory and does not reload it (:66-70, :147-149), so
    the named output keeps its 4 polarisations with the new weights."""
    with tempfile.TemporaryDirectory() as wd:
        data, weights, shift = synth.make_cube(6, 32, 64, 23, 0.2, npol=4)
        path = os.path.join(wd, "mem.ar")
        ica.Archive(data, weights, shift, filename=path).unload(path)
        buf = io.StringIO()
        old = sys.argv
        cwd = os.getcwd()
        os.chdir(wd)
        try:
            sys.argv = ["iterative_cleaner.py", "-l", "--memory", "-o", "mem_out.ar", path]
            with contextlib.redirect_stdout(buf):
                ic.main(ic.parse_arguments())
        finally:
            sys.argv = old
            os.chdir(cwd)
        out_ar = ica.Archive_load(os.path.join(wd, "mem_out.ar"))
        out = out_ar.get_data()
        np.savez_compressed(os.path.join(out_dir, "cli_memory_case.npz"),
                            weights=out_ar.get_weights(), data_shape=np.array(out.shape),
                            data_sha256=np.array(sha(np.ascontiguousarray(out))),
                            stdout=np.array(buf.getvalue().replace(wd, "<WD>")),
                            input_sha256=np.array(sha(data)))
        print("wrote cli_memory_case.npz")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=HERE)
    ap.add_argument("--skip-big", action="store_true")
    ap.add_argument("--only", default="", help="comma list: long,stats_long,zap,nonfinite,f64,fft,edge,cli_memory,"
                                                "fft2 (later rounds' fixtures only)")
    a = ap.parse_args()
    ic = import_reference()
    only = set(filter(None, a.only.split(",")))
    if only:
        if "long" in only:
            run_long_cases(ic, a.out)
        if "stats_long" in only:
            run_long_stats_cases(ic, a.out)
        if "zap" in only:
            run_zap_plot_case(ic, a.out)
        if "nonfinite" in only:
            run_leastsq_nonfinite(ic, a.out)
        if "f64" in only:
            run_f64_cases(ic, a.out)
        if "fft" in only:
            run_fft_cases(ic, a.out)
        if "edge" in only:
            run_edge_cases(ic, a.out)
        if "fft2" in only:
            run_fft2_cases(ic, a.out)
        if "cli_memory" in only:
            run_cli_memory_case(ic, a.out)
            run_cli_std_name_case(ic, a.out)
        return
    with tempfile.TemporaryDirectory() as wd:
        run_clean_case(ic, "s12x48x128", 12, 48, 128, 3, 0.05, workdir=wd, out_dir=a.out)
        run_clean_case(ic, "s16x64x256_rfi30", 16, 64, 256, 4, 0.30, workdir=wd, out_dir=a.out)
        run_clean_case(ic, "s10x40x100_thr3", 10, 40, 100, 7, 0.2,
                       extra_args=("-c", "3", "-s", "3", "-m", "7"), workdir=wd, out_dir=a.out)
        run_clean_case(ic, "s8x32x64_pol4", 8, 32, 64, 8, 0.2, npol=4,
                       extra_args=("-p",), workdir=wd, out_dir=a.out)
        run_clean_case(ic, "s12x40x128_pr", 12, 40, 128, 9, 0.1,
                       extra_args=("-r", "0.5", "30", "50"), workdir=wd, out_dir=a.out)
        if not a.skip_big:
            run_clean_case(ic, "C1", 64, 256, 256, 0, 0.05, keep_cubes=False,
                           workdir=wd, out_dir=a.out)
            run_clean_case(ic, "s64x256x256_rfi30", 64, 256, 256, 0, 0.30, keep_cubes=False,
                           workdir=wd, out_dir=a.out)
    run_stats_cases(ic, a.out)
    run_leastsq_cases(ic, a.out)
    run_pulse_region_case(ic, a.out)
    run_cli_case(ic, a.out)
    run_long_cases(ic, a.out)
    run_long_stats_cases(ic, a.out)
    run_zap_plot_case(ic, a.out)
    run_leastsq_nonfinite(ic, a.out)
    run_f64_cases(ic, a.out)
    run_fft_cases(ic, a.out)
    run_edge_cases(ic, a.out)
    run_cli_memory_case(ic, a.out)
    run_cli_std_name_case(ic, a.out)
    run_fft2_cases(ic, a.out)


def run_fft2_cases(ic, out_dir=HERE):
    """Round 6: archives as psrchive holds them.  Per-(subint, channel) delays
    (each Integration's own folding period: every dedisperse / dededisperse is
    the FFT rotation by that profile's delay), and archives stored dedispersed
    (dedisperse at ic.py:91 / :100 a no-op, only :104 rotates), with integer
    shifts and with fractional delays."""
    with tempfile.TemporaryDirectory() as wd:
        run_clean_case(ic, "s12x48x128_fft_pp", 12, 48, 128, 3, 0.05, frac_delay2=True, workdir=wd,
                       out_dir=out_dir)
        run_clean_case(ic, "s6x48x1024_fft_pp_u", 6, 48, 1024, 43, 0.05, extra_args=("-u",), frac_delay2=True,
                       keep_cubes=False, workdir=wd, out_dir=out_dir)
        run_clean_case(ic, "s8x40x256_fft_ded", 8, 40, 256, 21, 0.2, frac_delay=True, stored_dedispersed=True,
                       keep_cubes=False, workdir=wd, out_dir=out_dir)
        run_clean_case(ic, "s6x40x128_fft_pp_ded_u", 6, 40, 128, 22, 0.2, extra_args=("-u",), frac_delay2=True,
                       stored_dedispersed=True, keep_cubes=False, workdir=wd, out_dir=out_dir)
        run_clean_case(ic, "s10x40x128_ded_u", 10, 40, 128, 23, 0.2, extra_args=("-u",), stored_dedispersed=True,
                       keep_cubes=False, workdir=wd, out_dir=out_dir)


def run_edge_cases(ic, out_dir=HERE):
    """Degenerate archives (round 4): one subint, one channel, 2 x 3; NaN / +-Inf samples; every weight 0; thresholds that zap everything; FFT-mode one subint and NaN / Inf; f64 data with NaN / -Inf and -u."""
    with tempfile.TemporaryDirectory() as wd:
        run_clean_case(ic, "s1x40x64_edge", 1, 40, 64, 5, 0.2, workdir=wd, out_dir=out_dir)
        run_clean_case(ic, "s6x1x128_edge", 6, 1, 128, 5, 0.2, workdir=wd, out_dir=out_dir)
        run_clean_case(ic, "s2x3x64_edge", 2, 3, 64, 5, 0.2, workdir=wd, out_dir=out_dir)
        run_clean_case(ic, "s8x24x128_nonfinite_edge", 8, 24, 128, 6, 0.2, workdir=wd, out_dir=out_dir,
                       poke=((1, 3, 10, np.nan), (4, 7, 100, np.inf), (6, 11, 0, -np.inf)))
        run_clean_case(ic, "s4x16x64_w0_edge", 4, 16, 64, 5, 0.2, workdir=wd, out_dir=out_dir, weights_zero=True)
        run_clean_case(ic, "s6x24x128_allzap_edge", 6, 24, 128, 5, 0.2, extra_args=("-c", "0.001", "-s", "0.001"),
                       workdir=wd, out_dir=out_dir)
        run_clean_case(ic, "s1x40x64_fft_edge", 1, 40, 64, 5, 0.2, frac_delay=True, workdir=wd, out_dir=out_dir)
        run_clean_case(ic, "s8x24x128_fft_nonfinite_edge", 8, 24, 128, 6, 0.2, frac_delay=True, workdir=wd,
                       out_dir=out_dir, poke=((1, 3, 10, np.nan), (4, 7, 100, np.inf)))
        run_clean_case(ic, "s8x24x128_f64_nonfinite_edge", 8, 24, 128, 6, 0.2, data_f64=True, extra_args=("-u",),
                       workdir=wd, out_dir=out_dir, poke=((2, 5, 40, -np.inf), (5, 9, 3, np.nan)))


def run_fft_cases(ic, out_dir=HERE):
    """clean() on archives with fractional delays: every dedisperse /
    dededisperse (ic.py:91, :100, :104) is the stand-in's FFT phase rotation
    (iterative_cleaner_amd/phase_rotation.py)."""
    with tempfile.TemporaryDirectory() as wd:
        run_clean_case(ic, "s12x48x128_fft", 12, 48, 128, 3, 0.05, frac_delay=True, workdir=wd, out_dir=out_dir)
        run_clean_case(ic, "s8x32x64_pol4_fft", 8, 32, 64, 8, 0.2, npol=4, extra_args=("-p",),
                       frac_delay=True, keep_cubes=False, workdir=wd, out_dir=out_dir)
        run_clean_case(ic, "s6x48x1024_fft_u", 6, 48, 1024, 43, 0.05, extra_args=("-u",), frac_delay=True,
                       keep_cubes=False, workdir=wd, out_dir=out_dir)
        run_clean_case(ic, "s12x40x256_fft_pr", 12, 40, 256, 9, 0.1, extra_args=("-r", "0.5", "30", "50"),
                       frac_delay=True, keep_cubes=False, workdir=wd, out_dir=out_dir)
        run_clean_case(ic, "s4x32x4096_fft_rfi30", 4, 32, 4096, 47, 0.30, frac_delay=True, keep_cubes=False,
                       workdir=wd, out_dir=out_dir)
        run_clean_case(ic, "s6x48x128_fft_f64", 6, 48, 128, 5, 0.1, frac_delay=True, data_f64=True,
                       frac_weights=True, keep_cubes=False, workdir=wd, out_dir=out_dir)


def run_f64_cases(ic, out_dir=HERE):
    """clean() through a binding whose get_data returns f64 (ic.py:111-112, :206-209
    then run in f64), with fractional weights (f64 products differ from f32)."""
    with tempfile.TemporaryDirectory() as wd:
        run_clean_case(ic, "s12x48x128_f64", 12, 48, 128, 3, 0.05, data_f64=True, frac_weights=True,
                       workdir=wd, out_dir=out_dir)
        run_clean_case(ic, "s12x48x128_fracw", 12, 48, 128, 3, 0.05, frac_weights=True, keep_cubes=False,
                       workdir=wd, out_dir=out_dir)
        run_clean_case(ic, "s6x48x1024_f64", 6, 48, 1024, 43, 0.05, keep_cubes=False, data_f64=True,
                       workdir=wd, out_dir=out_dir)
        run_clean_case(ic, "s8x40x100_f64_thr3", 8, 40, 100, 7, 0.2, extra_args=("-c", "3", "-s", "3"),
                       keep_cubes=False, data_f64=True, workdir=wd, out_dir=out_dir)


def run_long_cases(ic, out_dir=HERE):
    """clean() at the bench profile lengths (C4's 512, C2/C3's 1024, C5's 4096)."""
    with tempfile.TemporaryDirectory() as wd:
        run_clean_case(ic, "s6x48x512_u", 6, 48, 512, 44, 0.05, extra_args=("-u",),
                       keep_cubes=False, workdir=wd, out_dir=out_dir)
        run_clean_case(ic, "s6x48x1024", 6, 48, 1024, 43, 0.05, keep_cubes=False,
                       workdir=wd, out_dir=out_dir)
        run_clean_case(ic, "s16x128x1024", 16, 128, 1024, 41, 0.05, keep_cubes=False,
                       workdir=wd, out_dir=out_dir)
        run_clean_case(ic, "s4x32x2048_rfi30", 4, 32, 2048, 45, 0.30, keep_cubes=False,
                       workdir=wd, out_dir=out_dir)
        run_clean_case(ic, "s4x32x4096_rfi30", 4, 32, 4096, 47, 0.30, keep_cubes=False,
                       workdir=wd, out_dir=out_dir)
        run_clean_case(ic, "s4x32x4096_rfi30_m3u", 4, 32, 4096, 40, 0.30, extra_args=("-u", "-m", "3"),
                       keep_cubes=False, workdir=wd, out_dir=out_dir, residual_full=False)


if __name__ == "__main__":
    main()
