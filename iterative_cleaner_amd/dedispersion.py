"""How the cleaner dedisperses an archive that is not the stand-in: delays from
the dispersion measure, as psrchive derives them for ``dedisperse()`` /
``dededisperse()`` (iterative_cleaner.py:91, :100, :104), and the choice of the
loop's dedispersion mode.

psrchive dedisperses every Integration on its own: channel c of subint s is
rotated in phase by the cold-plasma delay of its centre frequency relative to
the archive's centre frequency, divided by THAT Integration's folding period
(Pulsar::Dispersion -> Integration -> Profile::rotate_phase).  In bins:

    delay[s, c] = (DM / 2.41e-4) * (1 / f_c^2 - 1 / f_ref^2) / P_s * nbin

(DM in pc cm^-3, f in MHz, P_s in s; 1/2.41e-4 s MHz^2 cm^3 pc^-1 is the
tempo / psrchive / dspsr dispersion constant), in that f64 operation order.
psrchive is not importable here, so this derivation is unpinned against it;
the tests pin what the loop does with the delays.

Mode selection (:func:`plan`):
  * every delay integral (and each channel's the same in every subint)
    -> integer rotation (IC_DEDISP_SHIFT), which is what a phase rotation by
    a whole number of bins is;
  * otherwise             -> psrchive's fractional FFT rotation (IC_DEDISP_FFT):
    one delay per channel when every subint has the same row, else one per
    profile (ic_set_delays2).  nbin must then be a power of two in 64..4096;
    any other nbin raises (the rotation kernels do not serve it, and rounding
    the delays would silently change which profiles get zapped).
"""
from __future__ import annotations

import numpy as np

DISPERSION_CONSTANT = 1.0 / 2.41e-4    # s MHz^2 cm^3 / pc (psrchive, dspsr, tempo)

__all__ = ["DISPERSION_CONSTANT", "delays_from_dm", "plan", "archive_delays", "fft_supported"]


def fft_supported(nbin: int) -> bool:
    """nbin the rotation kernels serve: a power of two in 64..4096."""
    return 64 <= nbin <= 4096 and (nbin & (nbin - 1)) == 0


def delays_from_dm(dm, freqs, fref, periods, nbin) -> np.ndarray:
    """(nsub, nchan) f64 delays in bins (module docstring's formula)."""
    f = np.asarray(freqs, dtype=np.float64).reshape(-1)
    p = np.asarray(periods, dtype=np.float64).reshape(-1)
    fr = float(fref)
    t = (float(dm) * DISPERSION_CONSTANT) * (1.0 / (f * f) - 1.0 / (fr * fr))      # (nchan,) seconds
    return t[None, :] / p[:, None] * float(nbin)


def plan(delay, nbin: int, what: str = "archive"):
    """(shift, delay) for the loop: integer shifts (delay None) when every delay
    is integral, else (zeros, delay) with delay (nchan,) if all rows agree or
    (nsub, nchan).  Raises ValueError for fractional delays at an nbin the
    rotation does not serve, and for non-finite delays."""
    d = np.asarray(delay, dtype=np.float64)
    if d.ndim == 1:
        d = d[None, :]
    if not np.all(np.isfinite(d)):
        raise ValueError("%s: non-finite dedispersion delay" % what)
    nchan = d.shape[1]
    if np.all(d == np.rint(d)):
        rows = np.mod(d, float(nbin)).astype(np.int64)
        if np.all(rows == rows[:1]):
            return rows[0], None
        # integral, but a channel's shift differs between subints: the shift
        # arrays are per channel, so these go through the per-profile rotation
    if not fft_supported(nbin):
        raise ValueError("%s: fractional dedispersion delays need a power-of-two nbin in 64..4096 for the "
                         "FFT phase rotation (nbin=%d); the delays are not rounded" % (what, nbin))
    zeros = np.zeros(nchan, np.int64)
    if np.all(d == d[:1]):
        return zeros, np.ascontiguousarray(d[0])
    return zeros, np.ascontiguousarray(d)


def archive_delays(ar) -> np.ndarray:
    """Delays of a psrchive(-like) archive: ``get_dispersion_measure()``,
    ``get_centre_frequency()``, the channel frequencies of subint 0
    (``get_Profile(0, 0, c).get_centre_frequency()``) and every Integration's
    ``get_folding_period()``."""
    nsub, nchan, nbin = ar.get_nsubint(), ar.get_nchan(), ar.get_nbin()
    freqs = np.array([ar.get_Profile(0, 0, c).get_centre_frequency() for c in range(nchan)], np.float64)
    periods = np.array([ar.get_Integration(s).get_folding_period() for s in range(nsub)], np.float64)
    return delays_from_dm(ar.get_dispersion_measure(), freqs, ar.get_centre_frequency(), periods, nbin)
