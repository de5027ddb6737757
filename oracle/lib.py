"""ctypes binding of the C oracle (oracle/ic_oracle.c) — TEST INFRASTRUCTURE ONLY."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libic_oracle.so")
_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH) or \
            os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(HERE, "ic_oracle.c")):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


class OrcParams(C.Structure):
    _fields_ = [("nsub", C.c_int32), ("nchan", C.c_int32), ("nbin", C.c_int32),
                ("max_iter", C.c_int32), ("chanthresh", C.c_double),
                ("subintthresh", C.c_double), ("pr_on", C.c_int32),
                ("pr_factor", C.c_double), ("pr_start", C.c_int32), ("pr_end", C.c_int32),
                ("baseline_duty", C.c_double), ("fit_mode", C.c_int32), ("data_f64", C.c_int32),
                ("dedisp_mode", C.c_int32), ("input_dedispersed", C.c_int32),
                ("delay_per_profile", C.c_int32)]


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = C.CDLL(LIB_PATH)
        _lib.orc_lmdif1.restype = C.c_int
        _lib.orc_lmdif1.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_double),
                                    C.POINTER(C.c_int), C.c_void_p]
        _lib.orc_fit_residual.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_int,
                                          C.c_double, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                          C.c_void_p]
        _lib.orc_fit_closed.argtypes = list(_lib.orc_fit_residual.argtypes) + [C.c_void_p, C.c_int]
        _lib.orc_baseline.argtypes = [C.c_int] * 3 + [C.c_void_p] * 3 + [C.c_double, C.c_void_p, C.c_void_p]
        _lib.orc_fit_cube.argtypes = [C.c_int] * 3 + [C.c_void_p] * 3 + [C.c_double, C.c_void_p]
        _lib.orc_template.argtypes = [C.c_int] * 3 + [C.c_void_p] * 3 + [C.c_double, C.c_void_p]
        _lib.orc_diagnostics.argtypes = [C.c_int, C.c_int] + [C.c_void_p] * 6
        _lib.orc_test.argtypes = [C.c_int, C.c_int] + [C.c_void_p] * 5 + [C.c_double, C.c_double, C.c_void_p]
        _lib.orc_test_f64.argtypes = _lib.orc_test.argtypes
        _lib.orc_diagnostics_f64.argtypes = [C.c_int, C.c_int] + [C.c_void_p] * 6
        _lib.orc_sum_f32.restype = C.c_float
        _lib.orc_sum_f32.argtypes = [C.c_void_p, C.c_int]
        _lib.orc_sum_f64.restype = C.c_double
        _lib.orc_sum_f64.argtypes = [C.c_void_p, C.c_int]
        _lib.orc_clean_loop.restype = C.c_int
        _lib.orc_clean_loop.argtypes = [C.POINTER(OrcParams)] + [C.c_void_p] * 17
        _lib.orc_twiddles.argtypes = [C.c_int, C.c_void_p]
        _lib.orc_phasors.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        _lib.orc_rotate.argtypes = [C.c_int] * 3 + [C.c_void_p] * 3 + [C.c_int, C.c_void_p]
        _lib.orc_rotate_ex.argtypes = [C.c_int] * 3 + [C.c_void_p] * 3 + [C.c_int] * 3 + [C.c_void_p]
    return _lib


def f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def lmdif1(T, p):
    T, p = f32(T), f32(p)
    x = C.c_double()
    nfev = C.c_int()
    info = lib().orc_lmdif1(len(T), _p(T), _p(p), C.byref(x), C.byref(nfev), None)
    return x.value, info, nfev.value


def fit_residual(D, T, pr=None):
    """D: (P, nbin) fit cube; returns (amp, info, R f32 dedispersed)."""
    D = f32(D).reshape(-1, np.shape(D)[-1])
    T = f32(T)
    P, n = D.shape
    amp = np.empty(P, np.float64)
    info = np.empty(P, np.int32)
    R = np.empty((P, n), np.float32)
    on, fac, a, b = (0, 1.0, 0, 0) if pr is None else (1, float(pr[0]), int(pr[1]), int(pr[2]))
    lib().orc_fit_residual(P, n, _p(T), _p(D), on, fac, a, b, _p(amp), _p(info), _p(R))
    return amp, info, R


def fit_closed(D, T, pr=None, shift=None):
    """fit_mode 1 (closed form): (amp, info, R f32 dedispersed) of the (P, nbin) fit
    cube; shift (nchan,): the rows' channel shifts (row k is channel k % nchan),
    whose stored order the dot is summed in (None: 0)."""
    D = f32(D).reshape(-1, np.shape(D)[-1])
    T = f32(T)
    P, n = D.shape
    amp = np.empty(P, np.float64)
    info = np.empty(P, np.int32)
    R = np.empty((P, n), np.float32)
    on, fac, a, b = (0, 1.0, 0, 0) if pr is None else (1, float(pr[0]), int(pr[1]), int(pr[2]))
    sh = None if shift is None else np.ascontiguousarray(shift, np.int32).reshape(-1)
    lib().orc_fit_closed(P, n, _p(T), _p(D), on, fac, a, b, _p(amp), _p(info), _p(R), _p(sh),
                         0 if sh is None else int(sh.size))
    return amp, info, R


def baseline(raw, W, shift, duty=0.15):
    raw = f32(raw)
    nsub, nchan, n = raw.shape
    base = np.empty((nsub, nchan), np.float32)
    win = np.empty(nsub, np.int32)
    lib().orc_baseline(nsub, nchan, n, _p(raw), _p(f32(W)), _p(np.ascontiguousarray(shift, np.int32)),
                       duty, _p(base), _p(win))
    return base, win


def fit_cube(raw, w0, shift, duty=0.15):
    raw = f32(raw)
    D = np.empty_like(raw)
    lib().orc_fit_cube(*raw.shape, _p(raw), _p(f32(w0)), _p(np.ascontiguousarray(shift, np.int32)),
                       duty, _p(D))
    return D


def template(raw, W, shift, duty=0.15):
    raw = f32(raw)
    T = np.empty(raw.shape[-1], np.float32)
    lib().orc_template(*raw.shape, _p(raw), _p(f32(W)), _p(np.ascontiguousarray(shift, np.int32)),
                       duty, _p(T))
    return T


def twiddles(n):
    """(2, n) f64 twiddle table of the FFT rotation (orc_twiddles)."""
    tw = np.empty((n, 2), np.float64)
    lib().orc_twiddles(n, _p(tw))
    return np.ascontiguousarray(tw.T)


def phasors(n, delay):
    """(2, nchan, n/2 + 1) f64 phasor table (orc_phasors)."""
    d = np.ascontiguousarray(delay, np.float64).reshape(-1)
    ph = np.empty((d.size, n // 2 + 1, 2), np.float64)
    lib().orc_phasors(n, d.size, _p(d), _p(ph))
    return np.ascontiguousarray(np.moveaxis(ph, -1, 0))


def rotate(cube, delay, sign=1, base=None, identity=False):
    """FFT phase rotation (fractional dedispersion) of a (nsub, nchan, n) cube:
    rot(f32(cube - base)) by +delay (sign 1) or -delay (sign -1); delay (nchan,)
    per channel or (nsub, nchan) per profile (orc_rotate_ex); identity: the
    no-op dedisperse of an archive stored dedispersed (f32(cube - base))."""
    cube = f32(cube)
    nsub, nchan, n = cube.shape
    out = np.empty_like(cube)
    d = np.ascontiguousarray(delay, np.float64)
    per_profile = d.size == nsub * nchan and d.ndim == 2
    if not per_profile:
        d = d.reshape(nchan)
    lib().orc_rotate_ex(nsub, nchan, n, _p(cube), _p(None if base is None else f32(base)), _p(d),
                        1 if per_profile else 0, 1 if identity else 0, int(sign), _p(out))
    return out


def diagnostics(X, valid):
    X = f32(X)
    shp = X.shape[:-1]
    P, n = int(np.prod(shp)), X.shape[-1]
    v = np.ascontiguousarray(valid, dtype=np.uint8).reshape(P)
    sd, mn, ff = (np.empty(P, np.float64) for _ in range(3))
    pt = np.empty(P, np.float32)
    lib().orc_diagnostics(P, n, _p(X), _p(v), _p(sd), _p(mn), _p(pt), _p(ff))
    return sd.reshape(shp), mn.reshape(shp), pt.reshape(shp), ff.reshape(shp)


def diagnostics_f64(X, valid):
    """Diagnostics of f64 data (data_f64): X is the f64 weighted cube."""
    X = np.ascontiguousarray(X, dtype=np.float64)
    shp = X.shape[:-1]
    P, n = int(np.prod(shp)), X.shape[-1]
    v = np.ascontiguousarray(valid, dtype=np.uint8).reshape(P)
    sd, mn, pt, ff = (np.empty(P, np.float64) for _ in range(4))
    lib().orc_diagnostics_f64(P, n, _p(X), _p(v), _p(sd), _p(mn), _p(pt), _p(ff))
    return sd.reshape(shp), mn.reshape(shp), pt.reshape(shp), ff.reshape(shp)


def test_values(valid, std, mean, ptp, fft, ct, st):
    """Scaled test values; ptp f32 (f32 data) or f64 (f64 data: scaled in f64)."""
    nsub, nchan = np.shape(valid)
    out = np.empty((nsub, nchan), np.float64)
    d64 = np.asarray(ptp).dtype == np.float64
    fn = lib().orc_test_f64 if d64 else lib().orc_test
    fn(nsub, nchan, _p(np.ascontiguousarray(valid, np.uint8)),
       _p(np.ascontiguousarray(std, np.float64)), _p(np.ascontiguousarray(mean, np.float64)),
       _p(np.ascontiguousarray(ptp, np.float64) if d64 else f32(ptp)), _p(np.ascontiguousarray(fft, np.float64)),
       float(ct), float(st), _p(out))
    return out


def clean_loop(raw, w0, shift, chanthresh=5.0, subintthresh=5.0, max_iter=5, pulse_region=None,
               duty=0.15, want_residual=False, want_details=False, fit_mode=0, data_f64=False, delay=None,
               input_dedispersed=False):
    """Whole loop; returns dict(test, weights, loops, changed, nzero, [...]).
    delay (nchan,) or (nsub, nchan) f64 bins: fractional dedispersion by FFT
    phase rotation (dedisp_mode 1) instead of the integer `shift`;
    input_dedispersed: raw is stored dedispersed (its dedisperse a no-op)."""
    raw = f32(raw)
    nsub, nchan, n = raw.shape
    P = nsub * nchan
    pr_on, fac, a, b = 0, 1.0, 0, 0
    if pulse_region is not None:
        pr_on, fac, a, b = 1, float(pulse_region[0]), int(pulse_region[1]), int(pulse_region[2])
    per_profile = delay is not None and np.ndim(delay) == 2
    prm = OrcParams(nsub, nchan, n, max_iter, float(chanthresh), float(subintthresh), pr_on, fac, a, b, duty,
                    int(fit_mode), 1 if data_f64 else 0, 0 if delay is None else 1,
                    1 if input_dedispersed else 0, 1 if per_profile else 0)
    if delay is not None:
        delay = np.ascontiguousarray(delay, np.float64).reshape((nsub, nchan) if per_profile else (nchan,))
    test = np.empty((nsub, nchan), np.float64)
    weights = np.empty((nsub, nchan), np.float32)
    loops = np.zeros(1, np.int32)
    changed = np.zeros(max(max_iter, 1), np.int32)
    nzero = np.zeros(max(max_iter, 1), np.int32)
    R = np.empty((nsub, nchan, n), np.float32) if want_residual else None
    T_all = np.empty((max(max_iter, 1), n), np.float32) if want_details else None
    amp = np.empty(P, np.float64) if want_details else None
    info = np.empty(P, np.int32) if want_details else None
    sd = np.empty(P, np.float64) if want_details else None
    mn = np.empty(P, np.float64) if want_details else None
    pt = np.empty(P, np.float64) if want_details else None
    ff = np.empty(P, np.float64) if want_details else None
    lib().orc_clean_loop(C.byref(prm), _p(raw), _p(f32(w0)), _p(np.ascontiguousarray(shift, np.int32)),
                         _p(test), _p(weights), _p(loops), _p(changed), _p(nzero), _p(R), _p(T_all),
                         _p(amp), _p(info), _p(sd), _p(mn), _p(pt), _p(ff), _p(delay))
    out = dict(test=test, weights=weights, loops=int(loops[0]), changed=changed[:max_iter],
               nzero=nzero[:max_iter])
    if want_residual:
        out["residual"] = R
    if want_details:
        out.update(T=T_all, amp=amp.reshape(nsub, nchan), info=info.reshape(nsub, nchan),
                   std=sd.reshape(nsub, nchan), mean=mn.reshape(nsub, nchan),
                   ptp=(pt if data_f64 else pt.astype(np.float32)).reshape(nsub, nchan),
                   fft=ff.reshape(nsub, nchan))
    return out
