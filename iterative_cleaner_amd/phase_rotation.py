"""Fractional dedispersion of the archive stand-in: psrchive's FFT phase rotation
with a written, reproducible arithmetic order.

psrchive dedisperses a profile by rotating it in phase through its Fourier
transform (Pulsar::Profile::rotate_phase -> fft::shift: forward real FFT,
multiply harmonic k by exp(i 2 pi k s / nbin), inverse real FFT, 1/nbin).  The
reference calls it through ``dedisperse()`` / ``dededisperse()``
(iterative_cleaner.py:91, :100, :104).  psrchive is absent here, so real-data
parity is unpinned; this module DEFINES the stand-in's rotation so that the
GPU kernel (k_rotate, ic_kernels.hip), the C restatement the tests check
against (orc_rotate in the oracle/ directory) and this numpy version agree bit for
bit.

Definition, for a profile x of N = 2M samples (N a power of two) and a delay
of s bins (``y[j] = x[j + s]`` for integer s; ``dedisperse`` rotates by +s,
``dededisperse`` by -s).  The arithmetic is IEEE single precision, as psrchive's
(its FTransform runs FFTW's single-precision plans on the f32 amplitudes):

1. x' = f32(x - base) (base 0 when no baseline is subtracted), then
   z[j] = (x'[2j], x'[2j+1]), j < M.
2. Z = FFT_M(z): Stockham autosort, stages of radix R = 8 while three or
   more of the log2 M levels remain, then one of radix 4 or 2; Ns = the
   product of the earlier radices.  Butterfly j < M/R: k = j mod Ns,
   a_q = z[j + q M/R]; from the second stage on (Ns > 1) b_q = a_q * w_q for
   q >= 1 with w_q = tw[q k N/(R Ns)] and the product (a.r w.r - a.i w.i,
   a.r w.i + a.i w.r), else b = a; y = DFT_R(b); out[(j - k) R + k + p Ns] = y_p.
   DFT_2: y0 = b0 + b1, y1 = b0 - b1.  DFT_4: c0 = b0 + b2, c1 = b0 - b2,
   c2 = b1 + b3, c3 = -i (b1 - b3) = (d.i, -d.r); y0 = c0 + c2, y1 = c1 + c3,
   y2 = c0 - c2, y3 = c1 - c3.  DFT_8: c_q = b_q + b_(q+4), c_(q+4) = b_q -
   b_(q+4) (q < 4); c5 = ((c5.r + c5.i) s, (c5.i - c5.r) s), c6 = (c6.i, -c6.r),
   c7 = ((c7.i - c7.r) s, -((c7.r + c7.i) s)) with s = f32(f64(sqrt(2)/2)); the
   even outputs y_(2p) = DFT_4(c0..c3)_p, the odd y_(2p+1) = DFT_4(c4..c7)_p.
3. For k = 1 .. M/2, q = M - k: the half-length spectrum of the inverse from
   Z_k, Z_q in one linear map (:func:`_pair`: the real spectrum, the phasors
   (P.r, sign * P.i) and the inverse's packing composed), stored conjugated,
   the conjugate's imaginary part as (-a) + (-b) of the two terms' imaginary
   parts (k = M/2 pairs with itself: the k values are stored last).
   DC and Nyquist: X_0 = Z_0.r + Z_0.i, X_M = Z_0.r - Z_0.i (real),
   Y_0 = X_0 P_0.r, Y_M = X_M P_M.r, stored (Y_0 + Y_M)/2, -((Y_0 - Y_M)/2).
4. r = FFT_M(stored) (same stages); out[2j] = r[j].r * (1/M),
   out[2j+1] = (-r[j].i) * (1/M).

Every step is a single IEEE f32 operation in the written order (no fused
multiply-add).  Tables: tw[q] = exp(-2 pi i q / N), evaluated in x87 long
double (cosl/sinl), rounded to f64 (:func:`twiddles`, the table k_diag's FFT
shares) and then to f32; the phasors P[k] = exp(+2 pi i k s / N) of a delay s,
evaluated by the f64 formula of :func:`phasors` (the GPU's ic_phasor,
ic_internal.h) and rounded to f32, so that the library's per-channel table and
its per-profile evaluation (psrchive's per-Integration folding period: one
delay per subint and channel) give the same bits.

History: rounds 2-5 ran radix-2 stages in f64; round 6 redefined the stages
as radix 8 (98 operations per 8 points instead of 120), the pair step as one
linear map, and then the arithmetic as f32, which is psrchive's own
precision and lets k_rotate run every complex operation as packed f32 pairs
(v_pk_add_f32 / v_pk_mul_f32: half the f64 instruction count) with half the
LDS traffic.  The result is within a few f32 ulps of the profile's largest
sample of numpy's f64 ``irfft(rfft(x) * exp(2j pi k s / N))`` (oracle/restated.py
fft_phase_shift, tests/test_phase_rotation.py), as psrchive's FFTW-f32 rotation
is.
"""
from __future__ import annotations

import numpy as np

__all__ = ["PI_L", "twiddles", "phasors", "rotate", "is_supported"]

PI_L = np.longdouble("3.141592653589793238462643383279502884")


def is_supported(nbin: int) -> bool:
    """The rotation needs a power-of-two nbin (the GPU kernel: 64 .. 4096)."""
    return nbin >= 4 and (nbin & (nbin - 1)) == 0


def twiddles(nbin: int) -> np.ndarray:
    """(2, nbin) f64: cos / sin of -2 pi q / nbin (long double, then f64)."""
    q = np.arange(nbin).astype(np.longdouble)
    ang = (np.longdouble(-2.0) * PI_L) * q / np.longdouble(nbin)
    return np.stack([np.cos(ang).astype(np.float64), np.sin(ang).astype(np.float64)])


# Taylor coefficients of sin((pi/2) z) and cos((pi/2) z):
# (-1)^j (pi/2)^(2j+1) / (2j+1)!  and  (-1)^j (pi/2)^(2j) / (2j)!, j = 0 .. 8,
# each the f64 nearest the exact value
_PH_S = tuple(float.fromhex(h) for h in (
    "0x1.921fb54442d18p+0", "-0x1.4abbce625be53p-1", "0x1.466bc6775aae2p-4", "-0x1.32d2cce62bd86p-8",
    "0x1.50783487ee782p-13", "-0x1.e3074fde8871fp-19", "0x1.e8f434d018d63p-25", "-0x1.6fadb9f155744p-31",
    "0x1.aaec32af93359p-38"))
_PH_C = tuple(float.fromhex(h) for h in (
    "0x1.0000000000000p+0", "-0x1.3bd3cc9be45dep+0", "0x1.03c1f081b5ac4p-2", "-0x1.55d3c7e3cbffap-6",
    "0x1.e1f506891babbp-11", "-0x1.a6d1f2a204a8cp-16", "0x1.f9d38a3763cc3p-22", "-0x1.b6e24f44b128fp-28",
    "0x1.20c62c2f2d7f5p-34"))


def phasors(nbin: int, delays) -> np.ndarray:
    """(2, *delays.shape, nbin/2 + 1) f64: exp(+2 pi i k s / nbin) for every
    delay s (bins) and harmonic k <= nbin/2, in this f64 operation order:

    * Veltkamp split s = sh + sl (c = s * 8193; sh = c - (c - s); sl = s - sh):
      sh has 40 significant bits, so k*sh and k*sl are exact (k < 2^13);
    * t = k sh - nbin rint(k sh / nbin)   (exact; |t| <= nbin/2)
    * y = (t + k sl) * (4 / nbin)          quarter turns, one rounding
    * q = rint(y); z = y - q               (exact; |z| <= 1/2)
    * w = z*z; sin = z * (S0 + w (S1 + ... w S8)); cos = C0 + w (C1 + ... w C8)
    * quadrant q mod 4: (cos, sin), (-sin, cos), (-cos, -sin), (sin, -cos).

    That is P0(k); the phasor itself (the GPU's ic_phasor) is P0(k) for k < 64
    and for multiples of 64, else the product P0(k mod 64) * P0(k - k mod 64)
    with separately rounded operations (re = a.re b.re - a.im b.im, im = a.re
    b.im + a.im b.re), so that a profile's phasors take 64 + nbin/128
    polynomial evaluations.  Within 7e-16 of the exact phasor
    (tests/test_phase_rotation.py checks it against x87 long double)."""
    m = nbin // 2
    k = np.arange(m + 1, dtype=np.float64)
    s = np.asarray(delays, dtype=np.float64)[..., None]
    nn = float(nbin)
    c = s * 8193.0
    sh = c - (c - s)
    sl = s - sh
    xh = k * sh
    xl = k * sl
    t = xh - nn * np.rint(xh * (1.0 / nn))
    y = (t + xl) * (4.0 / nn)
    q = np.rint(y)
    z = y - q
    w = z * z
    sp = np.full_like(z, _PH_S[8])
    cp = np.full_like(z, _PH_C[8])
    for j in range(7, -1, -1):
        sp = _PH_S[j] + w * sp
        cp = _PH_C[j] + w * cp
    sn = z * sp
    qi = q.astype(np.int64) & 3
    re = np.where(qi == 0, cp, np.where(qi == 1, -sn, np.where(qi == 2, -cp, sn)))
    im = np.where(qi == 0, sn, np.where(qi == 1, cp, np.where(qi == 2, -sn, -cp)))
    # the product form: P(k) = P0(k mod 64) P0(k - k mod 64) where both parts are nonzero
    ki = np.arange(m + 1)
    lo, hi = ki & 63, ki - (ki & 63)
    sel = (lo != 0) & (hi != 0)
    if sel.any():
        ar, ai = re[..., lo[sel]], im[..., lo[sel]]
        br, bi = re[..., hi[sel]], im[..., hi[sel]]
        re = re.copy()
        im = im.copy()
        re[..., sel] = ar * br - ai * bi
        im[..., sel] = ar * bi + ai * br
    return np.stack([re, im])


S8 = np.float32(0.7071067811865476)   # f32 of f64(sqrt(2)/2) = Re exp(-i pi/4) of the f32 twiddle table


def _dft4(ar, ai):
    """DFT of 4 points (lists of arrays) in the definition's order (module docstring)."""
    c0r, c0i = ar[0] + ar[2], ai[0] + ai[2]
    c1r, c1i = ar[0] - ar[2], ai[0] - ai[2]
    c2r, c2i = ar[1] + ar[3], ai[1] + ai[3]
    dr, di = ar[1] - ar[3], ai[1] - ai[3]
    c3r, c3i = di, -dr                       # -i (b1 - b3)
    return ([c0r + c2r, c1r + c3r, c0r - c2r, c1r - c3r],
            [c0i + c2i, c1i + c3i, c0i - c2i, c1i - c3i])


def _dft8(ar, ai):
    cr = [ar[q] + ar[q + 4] for q in range(4)] + [ar[q] - ar[q + 4] for q in range(4)]
    ci = [ai[q] + ai[q + 4] for q in range(4)] + [ai[q] - ai[q + 4] for q in range(4)]
    t1, t2 = cr[5] + ci[5], ci[5] - cr[5]    # c5 * exp(-i pi/4)
    cr[5], ci[5] = t1 * S8, t2 * S8
    cr[6], ci[6] = ci[6], -cr[6]             # c6 * -i
    t1, t2 = ci[7] - cr[7], cr[7] + ci[7]    # c7 * exp(-3 i pi/4)
    cr[7], ci[7] = t1 * S8, -(t2 * S8)
    er, ei = _dft4(cr[:4], ci[:4])
    orr, oi = _dft4(cr[4:], ci[4:])
    return ([er[0], orr[0], er[1], orr[1], er[2], orr[2], er[3], orr[3]],
            [ei[0], oi[0], ei[1], oi[1], ei[2], oi[2], ei[3], oi[3]])


def _stockham(vr: np.ndarray, vi: np.ndarray, tw: np.ndarray):
    """FFT of the last axis (M complex points): Stockham stages of radix 8 while
    three or more levels remain, then one of radix 4 or 2 (module docstring)."""
    m = vr.shape[-1]
    n = 2 * m
    lg = m.bit_length() - 1
    ns, done = 1, 0
    while done < lg:
        rem = lg - done
        r = 8 if rem >= 3 else (4 if rem == 2 else 2)
        g = m // r
        j = np.arange(g)
        k = j & (ns - 1)
        ar = [vr[..., q * g:(q + 1) * g] for q in range(r)]
        ai = [vi[..., q * g:(q + 1) * g] for q in range(r)]
        if ns > 1:
            for q in range(1, r):
                idx = q * k * (n // (r * ns))
                wr, wi = tw[0][idx], tw[1][idx]
                ar[q], ai[q] = ar[q] * wr - ai[q] * wi, ar[q] * wi + ai[q] * wr
        if r == 8:
            yr, yi = _dft8(ar, ai)
        elif r == 4:
            yr, yi = _dft4(ar, ai)
        else:
            yr, yi = [ar[0] + ar[1], ar[0] - ar[1]], [ai[0] + ai[1], ai[0] - ai[1]]
        o = (j - k) * r + k
        nr = np.empty_like(vr)
        ni = np.empty_like(vi)
        for p in range(r):
            nr[..., o + p * ns] = yr[p]
            ni[..., o + p * ns] = yi[p]
        vr, vi = nr, ni
        ns *= r
        done += {8: 3, 4: 2, 2: 1}[r]
    return vr, vi


def _pair(zkr, zki, zqr, zqi, c, sn, pkr, pki, pqr, pqi):
    """The half-length inputs of the inverse, conjugated (what it stores):
    conj(Z'_k) and conj(Z'_q) (q = M - k), from the transform's Z_k, Z_q in one
    linear map: with w = exp(-2 pi i k / N) = (c, sn) and the phasors P_k, P_q
    (their imaginary parts signed for the direction), the real spectrum
    X_k = E_k + w O_k, Y = P X and the inverse's packing Z' = E' + i conj(w) H'
    compose to
        Z'_k = A_k Z_k + B_k conj(Z_q),  Z'_q = A_q Z_q - conj(B_k) conj(Z_k),
        A_k = ((1 + sn) P_k + (1 - sn) conj(P_q)) / 2,
        A_q = ((1 + sn) P_q + (1 - sn) conj(P_k)) / 2,
        B_k = i c (P_k - conj(P_q)) / 2.
    Each Z' is the sum of its two terms; its conjugate's imaginary part is the
    sum of the two terms' negated imaginary parts ((-a) + (-b), which differs
    from -(a + b) only in the sign of a zero sum)."""
    h1 = (1.0 + sn) * 0.5
    h2 = (1.0 - sn) * 0.5
    hc = c * 0.5
    akr = h1 * pkr + h2 * pqr
    aki = h1 * pki - h2 * pqi
    aqr = h1 * pqr + h2 * pkr
    aqi = h1 * pqi - h2 * pki
    bkr = -(hc * (pki + pqi))
    bki = hc * (pkr - pqr)
    return ((akr * zkr - aki * zki) + (bkr * zqr + bki * zqi),
            (-(akr * zki + aki * zkr)) + (-(bki * zqr - bkr * zqi)),
            (aqr * zqr - aqi * zqi) + (bki * zki - bkr * zkr),
            (-(aqr * zqi + aqi * zqr)) + (-(bki * zkr + bkr * zki)))


def rotate(x: np.ndarray, ph: np.ndarray, sign: int, tw: np.ndarray | None = None,
           base: np.ndarray | None = None) -> np.ndarray:
    """Rotate profiles x (..., nchan, nbin) f32 by their delays.

    ph: phasors(nbin, delays) for the nchan channels (axis -2 of x), or for
    every profile (delays of x's leading shape, e.g. (nsub, nchan)); sign +1 =
    dedisperse (y[j] = x[j + s]), -1 = dededisperse; base (..., nchan) f32 is
    subtracted first in f32 (remove_baseline's levels)."""
    x = np.asarray(x, dtype=np.float32)
    n = x.shape[-1]
    if not is_supported(n):
        raise ValueError("fractional dedispersion needs a power-of-two nbin (got %d)" % n)
    if tw is None:
        tw = twiddles(n)
    tw = np.asarray(tw, dtype=np.float64).astype(np.float32)   # f32 of the f64 table
    with np.errstate(invalid="ignore", over="ignore"):   # NaN / Inf samples propagate
        return _rotate(x, ph, sign, tw, base)


def _rotate(x, ph, sign, tw, base):
    n = x.shape[-1]
    if base is not None:
        x = (x - np.asarray(base, dtype=np.float32)[..., None]).astype(np.float32)
    m = n // 2
    vr = np.ascontiguousarray(x[..., 0::2])
    vi = np.ascontiguousarray(x[..., 1::2])
    vr, vi = _stockham(vr, vi, tw)
    pr = np.asarray(ph[0]).astype(np.float32)
    pi = np.asarray(ph[1] if sign > 0 else -ph[1]).astype(np.float32)
    k = np.arange(1, m // 2 + 1)
    q = m - k
    zkr, zki, zqr, zqi = vr[..., k], vi[..., k], vr[..., q], vi[..., q]
    zkr2, zki2, zqr2, zqi2 = _pair(zkr, zki, zqr, zqi, tw[0][k], tw[1][k], pr[..., k], pi[..., k], pr[..., q],
                                   pi[..., q])
    x0 = vr[..., 0] + vi[..., 0]
    xm = vr[..., 0] - vi[..., 0]
    y0 = x0 * pr[..., 0]
    ym = xm * pr[..., m]
    ur = np.empty_like(vr)
    ui = np.empty_like(vi)
    ur[..., 0] = (y0 + ym) * 0.5
    ui[..., 0] = -((y0 - ym) * 0.5)
    ur[..., q] = zqr2      # conj(Z'_q), conj(Z'_k) (_pair)
    ui[..., q] = zqi2
    ur[..., k] = zkr2      # k = M/2 pairs with itself: the k values are stored last
    ui[..., k] = zki2
    rr, ri = _stockham(ur, ui, tw)
    inv = np.float32(1.0 / m)
    out = np.empty(x.shape, dtype=np.float32)
    out[..., 0::2] = rr * inv
    out[..., 1::2] = (-ri) * inv
    for a in (vr, vi, ur, ui, rr, ri):
        assert a.dtype == np.float32   # every operation of the definition is f32
    return out
