"""A duck-typed archive with only the psrchive binding's methods that the
reference's clean() path touches (iterative_cleaner.py:47-62, :65-178) and the
ones psrchive's own dedispersion reads: get_dispersion_measure,
get_centre_frequency, Profile.get_centre_frequency, Integration.
get_folding_period, get_dedispersed.  None of the stand-in's extras
(get_dm_shift, get_dm_delay, get_baseline_duty): the cleaner must derive the
dedispersion from the psrchive quantities, as it would for real psrchive.
Test infrastructure."""
from __future__ import annotations

import copy

import numpy as np


class _Profile:
    def __init__(self, ar, isub, ipol, ichan):
        self._ar, self._isub, self._ipol, self._ichan = ar, isub, ipol, ichan

    def get_centre_frequency(self):
        return float(self._ar._freqs[self._ichan])

    def get_amps(self):
        return self._ar._data[self._isub, self._ipol, self._ichan]

    def get_weight(self):
        return float(self._ar._weights[self._isub, self._ichan])


class _Integration:
    def __init__(self, ar, isub):
        self._ar, self._isub = ar, isub

    def get_folding_period(self):
        return float(self._ar._periods[self._isub])

    def set_weight(self, ichan, w):
        self._ar._weights[self._isub, ichan] = w

    def get_weight(self, ichan):
        return float(self._ar._weights[self._isub, ichan])

    def get_nchan(self):
        return self._ar._data.shape[2]


class PsrchiveLike:
    """data (nsub, npol, nchan, nbin) f32 as the archive stores it (dispersed,
    or dedispersed with dedispersed=True); freqs (nchan,) MHz; periods (nsub,) s."""

    def __init__(self, data, weights, dm, freqs, periods, cfreq, dedispersed=False, filename="psr.ar"):
        self._data = np.ascontiguousarray(data, np.float32)
        self._weights = np.array(weights, np.float32)
        self._dm = float(dm)
        self._freqs = np.asarray(freqs, np.float64)
        self._periods = np.asarray(periods, np.float64)
        self._cfreq = float(cfreq)
        self._ded = bool(dedispersed)
        self._filename = filename

    def get_nsubint(self): return self._data.shape[0]
    def get_npol(self): return self._data.shape[1]
    def get_nchan(self): return self._data.shape[2]
    def get_nbin(self): return self._data.shape[3]
    def get_data(self): return self._data.copy()
    def get_weights(self): return self._weights.copy()
    def get_dispersion_measure(self): return self._dm
    def get_centre_frequency(self): return self._cfreq
    def get_dedispersed(self): return self._ded
    def get_filename(self): return self._filename
    def get_source(self): return "J1234+5678"
    def get_state(self): return {1: "Intensity", 2: "PPQQ", 4: "Coherence"}[self.get_npol()]
    def get_Integration(self, isub): return _Integration(self, int(isub))
    def get_Profile(self, isub, ipol, ichan): return _Profile(self, int(isub), int(ipol), int(ichan))
    def clone(self): return copy.deepcopy(self)

    def pscrunch(self):
        if self.get_npol() > 1:
            self._data = np.ascontiguousarray(self._data[:, 0:1] + self._data[:, 1:2])

    def __str__(self):
        return "PSRFITS:%s" % self._filename
