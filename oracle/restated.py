"""NumPy restatement of the cleaning statistics — TEST INFRASTRUCTURE ONLY.

Written without numpy.ma: every masked-array rule the reference relies on is
spelled out so that the C oracle and the HIP kernels can follow the same
text.  Reference lines: comprehensive_stats iterative_cleaner.py:181-226,
channel_scaler :229-241, subint_scaler :244-256, apply_weights :291-297,
mask :114-117.  numpy 2.2.6 sources followed: numpy/ma/core.py (mean
:5416-5460, var/std :5510-5600, ptp :6110, domained division :1170-1240,
masked unary :990-1020), numpy/ma/extras.py median :716-880.
"""
from __future__ import annotations

import numpy as np

TINY = np.finfo(np.float64).tiny


# --------------------------------------------------------------------------
# numpy pairwise summation (numpy/_core/src/umath/loops_utils.h.src)
# --------------------------------------------------------------------------
def _pw(a: np.ndarray, lo: int, n: int) -> np.ndarray:
    """Pairwise sum of a[..., lo:lo+n] in a's dtype, numpy's exact order."""
    dt = a.dtype.type
    if n < 8:
        res = np.zeros(a.shape[:-1], dtype=a.dtype)       # res = 0.
        for i in range(n):
            res = (res + a[..., lo + i]).astype(a.dtype)
        return res
    if n <= 128:
        r = [a[..., lo + j].copy() for j in range(8)]
        i = 8
        lim = n - (n % 8)
        while i < lim:
            for j in range(8):
                r[j] = (r[j] + a[..., lo + i + j]).astype(a.dtype)
            i += 8
        res = (((r[0] + r[1]).astype(a.dtype) + (r[2] + r[3]).astype(a.dtype)).astype(a.dtype)
               + ((r[4] + r[5]).astype(a.dtype) + (r[6] + r[7]).astype(a.dtype)).astype(a.dtype)
               ).astype(a.dtype)
        while i < n:
            res = (res + a[..., lo + i]).astype(a.dtype)
            i += 1
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return (_pw(a, lo, n2) + _pw(a, lo + n2, n - n2)).astype(dt)


def pairwise_sum(a: np.ndarray) -> np.ndarray:
    """np.add.reduce along the last (contiguous) axis: 0 + pairwise(a)."""
    n = a.shape[-1]
    zero = np.zeros(a.shape[:-1], dtype=a.dtype)
    return (zero + _pw(a, 0, n)).astype(a.dtype)


# --------------------------------------------------------------------------
# diagnostics (iterative_cleaner.py:206-217)
# --------------------------------------------------------------------------
def diagnostics(X: np.ndarray, valid: np.ndarray):
    """X: weighted cube f32 (nsub, nchan, nbin); valid: (nsub, nchan) bool.

    Returns (std f64, mean f64, ptp f32, fftmax f64) *data* arrays exactly as
    the numpy.ma results hold them (invalid entries: std 0, mean 0,
    ptp 1e20, fftmax = max|rfft(X)| of the unshifted invalid profile).
    """
    X = np.asarray(X, dtype=np.float32)
    n = X.shape[-1]
    s32 = pairwise_sum(X)                                       # f32
    mean = np.where(valid, s32.astype(np.float64) / n, 0.0)
    d = X.astype(np.float64) - mean[..., None]
    var = pairwise_sum(d * d) / n
    std = np.where(valid, np.sqrt(var), 0.0)
    ptp = np.where(valid, (X.max(axis=-1) - X.min(axis=-1)).astype(np.float32),
                   np.float32(1e20)).astype(np.float32)
    fin = np.where(valid[..., None], d, X.astype(np.float64))
    fft = np.max(np.abs(np.fft.rfft(fin, axis=-1)), axis=-1)
    return std, mean, ptp, fft


# --------------------------------------------------------------------------
# medians (numpy/ma/extras.py _median 1-D path; numpy.median)
# --------------------------------------------------------------------------
def _mid_median(sorted_vals: np.ndarray, dtype) -> "np.generic":
    """Median of ascending ``sorted_vals`` (no NaN) in dtype: odd → 0+mid,
    even → (0+lo+hi)/2, all in dtype (numpy's sum-then-true_divide)."""
    cnt = sorted_vals.shape[0]
    dt = np.dtype(dtype).type
    idx, odd = divmod(cnt, 2)
    if odd:
        return dt(dt(0) + sorted_vals[idx])
    s = dt(dt(dt(0) + sorted_vals[idx - 1]) + sorted_vals[idx])
    return dt(s / dt(2))


def median_valid(vals: np.ndarray, dtype):
    """np.ma.median of a line's valid values (NaN if any NaN)."""
    v = np.asarray(vals, dtype=dtype)
    if v.size == 0:
        return None
    if np.isnan(v).any():
        return np.dtype(dtype).type(np.nan)
    return _mid_median(np.sort(v), dtype)


def median_plain(vals: np.ndarray):
    v = np.asarray(vals, dtype=np.float64)
    if np.isnan(v).any():
        return np.float64(np.nan)
    return _mid_median(np.sort(v), np.float64)


# --------------------------------------------------------------------------
# scalers + combine (iterative_cleaner.py:221-256)
# --------------------------------------------------------------------------
def scale_line_masked(d: np.ndarray, valid: np.ndarray, thresh) -> np.ndarray:
    """Final f64 value of |scaler(D)|/thresh for one line of a masked diag."""
    dt = d.dtype.type
    out = np.empty(d.shape, dtype=np.float64)
    thr = np.float64(thresh)
    with np.errstate(all="ignore"):
        # invalid entries keep their data through - and / (numpy.ma restores da
        # where masked); np.abs (a plain ufunc + __array_wrap__) then takes |.|
        # of masked data too, and the masked /thresh keeps it: value = |d|
        out[~valid] = np.float64(0.0) + np.abs(d[~valid]).astype(np.float64)
        if valid.any():
            med = median_valid(d[valid], d.dtype)
            r = (d - med).astype(d.dtype)
            mad = median_valid(np.abs(r[valid]), d.dtype)
            q = (r / mad).astype(d.dtype)
            dom = ~np.isfinite(q) | (np.abs(r).astype(np.float64) * TINY
                                     >= np.float64(np.abs(mad)))
            a = np.abs(q)
            res = a.astype(np.float64) / thr
            dom2 = ~np.isfinite(res) | (a.astype(np.float64) * TINY >= np.abs(thr))
            v = np.where(dom, np.float64(0.0) + np.abs(dt(0) + r).astype(np.float64),
                         np.where(dom2, np.float64(0.0) + a.astype(np.float64), res))
            out[valid] = v[valid]
    return out


def scale_line_plain(d: np.ndarray, thresh) -> np.ndarray:
    with np.errstate(all="ignore"):
        med = median_plain(d)
        r = d - med
        mad = median_plain(np.abs(r))
        q = r / mad
        return np.abs(q) / np.float64(thresh)


def comprehensive_stats(X: np.ndarray, w0: np.ndarray, chanthresh, subintthresh,
                        return_parts: bool = False):
    """test (nsub, nchan) f64 for the weighted cube X and original weights."""
    valid = np.asarray(w0) != 0
    std, mean, ptp, fft = diagnostics(X, valid)
    nsub, nchan = valid.shape
    scaled = []
    parts = {}
    for name, D, masked in (("std", std, True), ("mean", mean, True),
                            ("ptp", ptp, True), ("fft", fft, False)):
        ch = np.empty((nsub, nchan), np.float64)
        sb = np.empty((nsub, nchan), np.float64)
        for c in range(nchan):
            ch[:, c] = (scale_line_masked(D[:, c], valid[:, c], chanthresh) if masked
                        else scale_line_plain(D[:, c], chanthresh))
        for s in range(nsub):
            sb[s, :] = (scale_line_masked(D[s, :], valid[s, :], subintthresh) if masked
                        else scale_line_plain(D[s, :], subintthresh))
        scaled.append(np.maximum(ch, sb))
        parts[name] = (D, ch, sb)
    st = np.stack(scaled)                                    # (4, nsub, nchan)
    with np.errstate(all="ignore"):
        srt = np.sort(st, axis=0)                            # NaN last
        test = (np.float64(0.0) + srt[1] + srt[2]) / 2.0
        test = np.where(np.isnan(st).any(axis=0), np.nan, test)
    if return_parts:
        return test, parts
    return test


def weighted_cube(R: np.ndarray, w0: np.ndarray) -> np.ndarray:
    """apply_weights (iterative_cleaner.py:291-297): f32(R * w0)."""
    return (np.asarray(R, np.float32) * np.asarray(w0, np.float32)[..., None]).astype(np.float32)


# --------------------------------------------------------------------------
# fit_mode 1 (IC_FIT_CLOSED): the closed-form amplitude, stated in numpy
# --------------------------------------------------------------------------
def closed_form_fit(D: np.ndarray, T: np.ndarray, shift=None):
    """a = np.sum(np.roll(T*p, sh)) / np.sum(T*T) per fit-cube row (numpy
    pairwise f64 sums along the contiguous bin axis): the products of the
    dedispersed row are summed in the archive's stored (dispersed) sample order,
    sample j pairing with the dedispersed bin (j - sh) mod nbin, sh the row's
    channel shift (shift: (nchan,) or None = 0; round 6: the dedispersed order
    before); a = 0 for an all-zero template; status 1, or 5 (residual zeroed)
    when a is not finite.  Returns (amp, info, R f32)."""
    T64 = np.asarray(T, np.float32).astype(np.float64)
    D64 = np.asarray(D, np.float32).astype(np.float64).reshape(-1, T64.size)
    TT = np.sum(T64 * T64)
    with np.errstate(all="ignore"):
        prod = D64 * T64[None, :]
        if shift is not None:
            sh = np.asarray(shift, np.int64).reshape(-1)
            rows = np.arange(prod.shape[0]) % sh.size
            j = (np.arange(T64.size)[None, :] - sh[rows][:, None]) % T64.size
            prod = np.ascontiguousarray(np.take_along_axis(prod, j, axis=-1))
        dot = np.sum(prod, axis=-1)
        amp = dot / TT if TT != 0.0 else np.zeros_like(dot)
        info = np.where(np.isfinite(amp), 1, 5).astype(np.int32)
        R = np.where(info[:, None] == 1, amp[:, None] * T64[None, :] - D64, 0.0).astype(np.float32)
    return amp, info, R



def fft_phase_shift(x: np.ndarray, delay, sign: int = 1) -> np.ndarray:
    """psrchive's published dedispersion of a profile (Profile::rotate_phase ->
    fft::shift): forward real FFT, harmonic k times exp(+-2 pi i k s / N),
    inverse real FFT, as numpy states it (pocketfft, complex128), rounded to
    f32.  x (..., nchan, N) f32, delay (nchan,) bins; sign +1 dedisperses
    (y[j] = x[j + s]), -1 dededisperses.  The stand-in's written-order
    rotation (iterative_cleaner_amd/phase_rotation.py, orc_rotate, k_rotate)
    computes in f32, as psrchive does, and agrees with this to within 4 f32
    epsilons of the profile's largest |sample|; real psrchive (FFTW in f32) is
    not available, so that parity is UNPINNED."""
    x = np.asarray(x, dtype=np.float32)
    n = x.shape[-1]
    k = np.arange(n // 2 + 1)
    s = np.asarray(delay, dtype=np.float64)[:, None]
    X = np.fft.rfft(x.astype(np.float64), axis=-1)
    return np.fft.irfft(X * np.exp(sign * 2j * np.pi * k * s / n), n=n, axis=-1).astype(np.float32)
