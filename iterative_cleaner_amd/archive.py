"""NumPy stand-in for the subset of the psrchive ``Archive`` API that the
surgical cleaner touches (reference calls listed at
iterative_cleaner.py:47-60, :66-125, :150-162, :262-272, :300-330).

psrchive is not installed here (no network), so this module *defines* the
archive semantics that both the reference-driven golden fixtures and the GPU
path must follow.  Every floating-point reduction below has a fixed, written
order so that the HIP kernels can reproduce it bit-for-bit:

* samples and weights are float32 (``get_data``/``get_weights`` return f32
  copies; ``get_data_dtype = np.float64`` models a psrchive build whose
  get_data returns f64 copies of the f32 amplitudes);
* ``get_state``: psrchive's polarisation state names - "Intensity" (one
  polarisation), "PPQQ" (AA, BB), "Coherence" (AA, BB, CR, CI) or "Stokes"
  (I, Q, U, V);
* ``pscrunch``: total intensity = f32(pol0 + pol1) for PPQQ / Coherence data,
  pol 0 (= I) for Stokes data; the state becomes "Intensity";
* ``dedisperse``/``dededisperse``: integer per-channel rotation by
  ``dm_shift[c]`` bins, ``ded[i] = raw[(i + shift) % nbin]``; an archive made
  with fractional delays ``dm_delay`` (f64 bins: ``[c]`` per channel, or
  ``[s, c]`` per profile - psrchive's per-Integration folding period) rotates
  instead by psrchive's FFT phase rotation, in the arithmetic order written in
  :mod:`.phase_rotation` (power-of-two nbin); an archive stored dedispersed
  (``dedispersed=True``) returns its samples as they are from the dedispersed
  view, and only ``dededisperse`` moves them;
* channel sums (baseline total, fscrunch) use the CANONICAL CHANNEL ORDER
  (:func:`chan_sum`): f64, sequential inside super-blocks of ``SUPER_BLOCK``
  channels; the super-block partials are combined by the halving tree of
  :func:`sb_tree`.  A shard that owns one node of that tree (2^d shards own
  the 2^d nodes at depth d) computes its subtree alone, and the top d levels
  combine the shard roots, so channel-sharded runs reproduce single-device
  bits;
* ``remove_baseline``: per subint (psrchive Integration::remove_baseline),
  the off-pulse window of width ``int(duty*nbin)`` is the first argmin of
  the circular window sums of the weighted, dedispersed total profile; each
  profile subtracts f32(mean of its own samples in that window) in f32;
* ``fscrunch``/``tscrunch``: weighted means, f64 accumulation, f32 result,
  weights summed.
"""
from __future__ import annotations

import copy
import os

import numpy as np

SUPER_BLOCK = 256          # channels per canonical-order super-block
BASELINE_DUTY = 0.15       # psrchive BaselineWindow default duty cycle

__all__ = ["Archive", "Archive_load", "Profile", "Integration", "chan_sum", "sb_tree",
           "baseline_width", "window_argmin", "SUPER_BLOCK", "BASELINE_DUTY", "STATES", "default_state",
           "load_channels"]


STATES = ("Intensity", "PPQQ", "Coherence", "Stokes")


def default_state(npol: int) -> str:
    return {1: "Intensity", 2: "PPQQ", 4: "Coherence"}.get(int(npol), "PPQQ")


def sb_tree(parts):
    """Canonical combine of super-block partials ``parts[0..n)`` (n >= 1):
    tree(lo, hi) = parts[lo] if hi - lo == 1 else tree(lo, mid) + tree(mid, hi),
    mid = lo + (hi - lo) // 2."""
    def tree(lo, hi):
        if hi - lo == 1:
            return parts[lo]
        mid = lo + (hi - lo) // 2
        return tree(lo, mid) + tree(mid, hi)
    return tree(0, len(parts))


def chan_sum(terms: np.ndarray, axis: int) -> np.ndarray:
    """Canonical channel reduction of f64 ``terms`` along ``axis``.

    For each super-block b of SUPER_BLOCK channels: part_b = 0.0; part_b += t[c]
    for c in b (ascending).  result = sb_tree(part_0 .. part_{nsb-1}).
    Zero-size → 0.0.
    """
    t = np.moveaxis(np.asarray(terms, dtype=np.float64), axis, 0)
    nchan = t.shape[0]
    if nchan == 0:
        return np.zeros(t.shape[1:], dtype=np.float64)
    parts = []
    for b0 in range(0, nchan, SUPER_BLOCK):
        part = np.zeros(t.shape[1:], dtype=np.float64)
        for c in range(b0, min(b0 + SUPER_BLOCK, nchan)):
            part = part + t[c]
        parts.append(part)
    return sb_tree(parts)


def baseline_width(nbin: int, duty: float = BASELINE_DUTY) -> int:
    return max(1, int(duty * nbin))


def window_argmin(total: np.ndarray, width: int) -> np.ndarray:
    """First argmin (numpy NaN semantics) over j of the circular window sums
    m[j] = sum_{k<width} total[..., (j+k) % nbin], sequential over k, f64."""
    total = np.asarray(total, dtype=np.float64)
    m = np.zeros_like(total)
    for k in range(width):
        m = m + np.roll(total, -k, axis=-1)
    return np.argmin(m, axis=-1)


class _Epoch:
    def __init__(self, mjd: float):
        self.mjd = float(mjd)

    def strtempo(self) -> str:
        return "%.15f" % self.mjd

    def in_days(self) -> float:
        return self.mjd


class Profile:
    """``ar.get_Profile(isub, ipol, ichan)``: amps are a writable f32 view."""

    def __init__(self, ar: "Archive", isub: int, ipol: int, ichan: int):
        self._ar, self._isub, self._ipol, self._ichan = ar, isub, ipol, ichan

    def get_amps(self) -> np.ndarray:
        return self._ar._data[self._isub, self._ipol, self._ichan]

    def get_weight(self) -> float:
        return float(self._ar._weights[self._isub, self._ichan])

    def set_weight(self, w: float) -> None:
        self._ar._weights[self._isub, self._ichan] = w

    def get_nbin(self) -> int:
        return self._ar.get_nbin()


class Integration:
    def __init__(self, ar: "Archive", isub: int):
        self._ar, self._isub = ar, isub

    def set_weight(self, ichan: int, w: float) -> None:
        self._ar._weights[self._isub, ichan] = w

    def get_weight(self, ichan: int) -> float:
        return float(self._ar._weights[self._isub, ichan])

    def get_nchan(self) -> int:
        return self._ar.get_nchan()


class Archive:
    """In-memory pulsar archive: data (nsub, npol, nchan, nbin) float32."""

    def __init__(self, data, weights=None, dm_shift=None, dedispersed=False,
                 filename="synthetic.ar", source="J0000+0000",
                 centre_frequency=1400.0, mjd_start=60000.0, mjd_end=60000.01,
                 baseline_duty=BASELINE_DUTY, state=None, dm_delay=None):
        data = np.asarray(data, dtype=np.float32)
        if data.ndim != 4:
            raise ValueError("data must be (nsub, npol, nchan, nbin)")
        self._data = np.ascontiguousarray(data)
        nsub, npol, nchan, nbin = data.shape
        if state is None:
            state = default_state(npol)
        if state not in STATES or (state == "Intensity") != (npol == 1):
            raise ValueError("bad polarisation state %r for npol=%d" % (state, npol))
        self._state = state
        if weights is None:
            weights = np.ones((nsub, nchan), dtype=np.float32)
        self._weights = np.array(weights, dtype=np.float32).reshape(nsub, nchan)
        if dm_shift is None:
            dm_shift = np.zeros(nchan, dtype=np.int64)
        self._shift = np.mod(np.asarray(dm_shift, dtype=np.int64), nbin).reshape(nchan)
        self._delay = None
        if dm_delay is not None:
            from .phase_rotation import is_supported
            if not is_supported(nbin):
                raise ValueError("fractional dedispersion needs a power-of-two nbin (got %d)" % nbin)
            d = np.array(dm_delay, dtype=np.float64)
            self._delay = d.reshape((nsub, nchan) if d.ndim == 2 else (nchan,))
        self._dedispersed = bool(dedispersed)
        self._filename = filename
        self._source = source
        self._cfreq = float(centre_frequency)
        self._mjd = (float(mjd_start), float(mjd_end))
        self._duty = float(baseline_duty)

    # ---------------------------------------------------------------- shape
    def get_nsubint(self): return self._data.shape[0]
    def get_npol(self): return self._data.shape[1]
    def get_nchan(self): return self._data.shape[2]
    def get_nbin(self): return self._data.shape[3]

    # ---------------------------------------------------------------- access
    get_data_dtype = np.float32

    def get_data(self) -> np.ndarray:
        return self._data.astype(self.get_data_dtype)

    def get_weights(self) -> np.ndarray:
        return self._weights.copy()

    def get_Profile(self, isub, ipol, ichan) -> Profile:
        return Profile(self, int(isub), int(ipol), int(ichan))

    def get_Integration(self, isub) -> Integration:
        return Integration(self, int(isub))

    def get_dm_shift(self) -> np.ndarray:
        return self._shift.copy()

    def get_dm_delay(self):
        """Fractional delays in bins (f64; (nchan,) per channel or (nsub, nchan)
        per profile), or None for an archive dedispersed by integer shifts."""
        return None if self._delay is None else self._delay.copy()

    def _rotate(self, data: np.ndarray, sign: int) -> np.ndarray:
        from .phase_rotation import phasors, rotate
        d = self._delay if self._delay.ndim == 1 else self._delay[:, None, :]   # over (nsub, npol, nchan)
        return rotate(data, phasors(self.get_nbin(), d), sign)

    def get_dedispersed(self) -> bool:
        return self._dedispersed

    def get_filename(self) -> str:
        return self._filename

    def get_source(self) -> str:
        return self._source

    def get_centre_frequency(self) -> float:
        return self._cfreq

    def start_time(self) -> _Epoch:
        return _Epoch(self._mjd[0])

    def end_time(self) -> _Epoch:
        return _Epoch(self._mjd[1])

    def get_baseline_duty(self) -> float:
        return self._duty

    def get_state(self) -> str:
        return self._state

    def __str__(self) -> str:
        # "<format>:<name>"; the CLI (iterative_cleaner.py:49) splits on the first ':'
        return "NumPyArchive:%s" % os.path.splitext(self._filename)[0]

    def clone(self) -> "Archive":
        return copy.deepcopy(self)

    # ---------------------------------------------------------------- transforms
    def pscrunch(self) -> None:
        if self.get_npol() > 1:
            if self._state == "Stokes":
                self._data = np.ascontiguousarray(self._data[:, 0:1])
            else:
                self._data = np.ascontiguousarray(self._data[:, 0:1] + self._data[:, 1:2])
            self._state = "Intensity"

    def _ded_view(self) -> np.ndarray:
        """Samples in the dedispersed frame (a copy if currently dispersed)."""
        if self._dedispersed:
            return self._data
        if self._delay is not None:
            return self._rotate(self._data, +1)
        out = np.empty_like(self._data)
        n = self.get_nbin()
        idx = (np.arange(n)[None, :] + self._shift[:, None]) % n
        for c in range(self.get_nchan()):
            out[:, :, c, :] = self._data[:, :, c, idx[c]]
        return out

    def dedisperse(self) -> None:
        if not self._dedispersed:
            self._data = self._ded_view()
            self._dedispersed = True

    def dededisperse(self) -> None:
        if self._dedispersed and self._delay is not None:
            self._data = self._rotate(self._data, -1)
            self._dedispersed = False
        elif self._dedispersed:
            n = self.get_nbin()
            out = np.empty_like(self._data)
            idx = (np.arange(n)[None, :] - self._shift[:, None]) % n
            for c in range(self.get_nchan()):
                out[:, :, c, :] = self._data[:, :, c, idx[c]]
            self._data = out
            self._dedispersed = False

    def remove_baseline(self) -> None:
        ded = self._ded_view()
        if self.get_npol() > 1:
            tot_src = ded[:, 0] + ded[:, 1]
        else:
            tot_src = ded[:, 0]
        w64 = self._weights.astype(np.float64)
        # total[s, i] = canonical chan sum of w[s,c] * x[s,c,i]
        total = chan_sum(w64[:, :, None] * tot_src.astype(np.float64), axis=1)
        width = baseline_width(self.get_nbin(), self._duty)
        j0 = window_argmin(total, width)                          # (nsub,)
        n = self.get_nbin()
        acc = np.zeros(ded.shape[:3], dtype=np.float64)           # (nsub, npol, nchan)
        for k in range(width):
            cols = (j0 + k) % n
            acc = acc + ded[np.arange(ded.shape[0]), :, :, cols].astype(np.float64)
        base = (acc / width).astype(np.float32)
        self._data = (self._data - base[..., None]).astype(np.float32)

    def fscrunch(self) -> None:
        w64 = self._weights.astype(np.float64)
        wsum = chan_sum(w64, axis=1)                              # (nsub,)
        num = chan_sum(w64[:, None, :, None] * self._data.astype(np.float64), axis=2)
        with np.errstate(divide="ignore", invalid="ignore"):
            prof = np.where(wsum[:, None, None] != 0.0,
                            num / wsum[:, None, None], 0.0).astype(np.float32)
        self._data = np.ascontiguousarray(prof[:, :, None, :])
        self._weights = wsum.astype(np.float32)[:, None]
        self._shift = np.zeros(1, dtype=np.int64)
        if self._delay is not None:
            self._delay = np.zeros(1, dtype=np.float64)

    def tscrunch(self) -> None:
        nsub = self.get_nsubint()
        w64 = self._weights.astype(np.float64)                   # (nsub, nchan)
        wt = np.zeros(w64.shape[1], dtype=np.float64)
        num = np.zeros(self._data.shape[1:], dtype=np.float64)   # (npol, nchan, nbin)
        for s in range(nsub):
            wt = wt + w64[s]
            num = num + w64[s][None, :, None] * self._data[s].astype(np.float64)
        with np.errstate(divide="ignore", invalid="ignore"):
            prof = np.where(wt[None, :, None] != 0.0, num / wt[None, :, None], 0.0)
        self._data = np.ascontiguousarray(prof.astype(np.float32)[None])
        self._weights = wt.astype(np.float32)[None, :]
        if self._delay is not None and self._delay.ndim == 2:
            self._delay = self._delay[:1]

    # ---------------------------------------------------------------- I/O
    def unload(self, path: str) -> None:
        from . import archive_io
        archive_io.save(self, path)


def Archive_load(path: str) -> Archive:
    from . import archive_io
    return archive_io.load(path)


def load_channels(path: str, c0: int, c1: int) -> Archive:
    """Channels [c0, c1) of the archive at `path`, read without loading the rest
    (channel-sharded cleaning: each rank holds its slice only).  The returned
    archive carries ``_chan_range = (c0, c1)`` and ``_nchan_total``."""
    from . import archive_io
    return archive_io.load(path, channels=(c0, c1))
