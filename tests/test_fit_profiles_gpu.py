"""remove_profile1d (iterative_cleaner.py:275-288) on the GPU through the C-ABI
entry ic_fit_profiles, against the reference's own leastsq outputs:
tests/golden/leastsq_cases.npz (208 profiles at nbin 64..4096: zero profiles
and templates, constants, exact multiples, scales 1e-6..1e6) and
leastsq_nonfinite.npz (NaN / Inf samples, status-8 fits).  Amplitudes,
statuses and the f32 residuals bit for bit (NaN samples as NaN: the payload
an IEEE op propagates differs between x86 and gfx950)."""
import os

import numpy as np
import pytest

from helpers import GOLDEN, bits_equal

pytestmark = pytest.mark.gpu


def _groups(z):
    off = 0
    by_n = {}
    for k, n in enumerate(z["nbin"]):
        by_n.setdefault(int(n), []).append((k, off))
        off += int(n)
    return by_n


@pytest.mark.parametrize("name", ["leastsq_cases", "leastsq_nonfinite"])
def test_fit_profiles_match_reference_leastsq(name):
    from iterative_cleaner_amd import _native
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    for n, items in _groups(z).items():
        for k, off in items:   # one template per profile: fit each alone
            T = z["T"][off:off + n]
            p = z["p"][off:off + n]
            amp, info, R = _native.fit_profiles(p[None], T)
            assert np.float64(amp[0]).tobytes() == np.float64(z["x"][k]).tobytes(), (name, k, amp[0], z["x"][k])
            assert info[0] == z["info"][k], (name, k, info[0], z["info"][k])
            want = z["resid"][off:off + n].astype(np.float32)
            # NaN samples (non-finite profiles) compare as NaN: which NaN payload an
            # IEEE subtraction propagates is the hardware's (x86 SSE vs gfx950)
            nan = np.isnan(want)
            assert np.array_equal(np.isnan(R[0]), nan), (name, k)
            assert bits_equal(R[0][~nan], want[~nan]), (name, k)


@pytest.mark.parametrize("nbin", [64, 256, 1024, 4096])
def test_fit_profiles_batch_matches_c_oracle(nbin, oracle_lib):
    """Many profiles against one template (rounds + tail), both fit modes."""
    from oracle import restated as R

    from iterative_cleaner_amd import _native, synth
    data, w0, shift = synth.make_cube(6, 300 if nbin < 4096 else 40, nbin, 21, 0.3)
    D = oracle_lib.fit_cube(data[:, 0], w0, shift).reshape(-1, nbin)
    T = oracle_lib.template(data[:, 0], w0, shift)
    D[3] = 0.0
    D[7] *= np.float32(1e-30)
    D[9] = (T * np.float32(1e12)).astype(np.float32)
    amp, info, Rg = _native.fit_profiles(D, T)
    a_o, i_o, R_o = oracle_lib.fit_residual(D, T)
    assert bits_equal(amp, a_o) and bits_equal(info, i_o) and bits_equal(Rg, R_o)
    amp, info, Rg = _native.fit_profiles(D, T, fit_mode=_native.FIT_CLOSED)
    a_c, i_c, R_c = R.closed_form_fit(D, T)
    assert bits_equal(amp, a_c) and bits_equal(info, i_c) and bits_equal(Rg, R_c)
