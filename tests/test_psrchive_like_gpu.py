"""cleaner.clean() on an archive that only has psrchive's methods (real-data
drop-in, iterative_cleaner.py:91, :100, :104): the cleaner derives psrchive's
dedispersion itself - delays from the DM, the channel frequencies and every
Integration's folding period - and takes the fractional FFT rotation (per
profile when the periods differ, ic_set_delays2), the integer rotation only
when every delay is integral, and the stored-dedispersed form when the archive
says so.  The zap mask must equal the C oracle's loop with those delays.
Parity against real psrchive: unpinned (psrchive is not importable here)."""
import numpy as np
import pytest

from helpers import bits_equal
from psrchive_like import PsrchiveLike

pytestmark = pytest.mark.gpu


def _archive(nsub, nchan, nbin, seed, dm, periods, dedispersed=False, npol=2):
    from iterative_cleaner_amd import phase_rotation as pr
    from iterative_cleaner_amd import dedispersion, synth
    data, w0, _ = synth.make_cube(nsub, nchan, nbin, seed, 0.2, npol=npol)
    freqs = 140.0 + np.arange(nchan) * (48.0 / nchan)
    cfreq = 164.0
    delay = dedispersion.delays_from_dm(dm, freqs, cfreq, periods, nbin)
    if dedispersed:       # the archive holds its samples dedispersed (psrchive's own dedisperse)
        data = pr.rotate(data, pr.phasors(nbin, delay[:, None, :]), 1)
    return PsrchiveLike(data, w0, dm, freqs, periods, cfreq, dedispersed=dedispersed), delay


def _clean(ar, monkeypatch, tmp_path):
    from iterative_cleaner_amd import cleaner
    seen = {}
    orig = cleaner.run_loop

    def spy(cube, w0, shift, args, **kw):
        seen.update(kw, shift=np.array(shift), cube_shape=cube.shape)
        return orig(cube, w0, shift, args, **kw)

    monkeypatch.setattr(cleaner, "run_loop", spy)
    monkeypatch.chdir(tmp_path)
    out = cleaner.clean(ar, cleaner.parse_arguments(["-l", "-q", "--memory", "psr.ar"]), "psr.ar")
    return out, seen


def _oracle(oracle_lib, ar0, delay, input_dedispersed=False):
    d = ar0.get_data()
    cube = (d[:, 0] + d[:, 1]).astype(np.float32) if d.shape[1] > 1 else np.ascontiguousarray(d[:, 0])
    nchan = cube.shape[1]
    return oracle_lib.clean_loop(cube, ar0.get_weights(), np.zeros(nchan, np.int32), delay=delay,
                                 input_dedispersed=input_dedispersed)


@pytest.mark.parametrize("nbin", [256, 1024])
def test_per_integration_periods_take_per_profile_rotation(nbin, monkeypatch, tmp_path, oracle_lib):
    nsub, nchan = 9, 96
    periods = 0.0331 * (1.0 + 2e-4 * np.sin(np.arange(nsub)))
    ar, delay = _archive(nsub, nchan, nbin, 71, 26.8, periods)
    ar0 = ar.clone()
    out, seen = _clean(ar, monkeypatch, tmp_path)
    assert seen["delay"] is not None and seen["delay"].shape == (nsub, nchan)
    assert np.array_equal(seen["delay"], delay) and not seen["input_dedispersed"]
    assert np.all(seen["shift"] == 0)
    ref = _oracle(oracle_lib, ar0, delay)
    assert bits_equal(out.get_weights(), ref["weights"])
    # the per-profile rotation matters: one delay row for every subint zaps differently
    # or at least computes different test values
    one = _oracle(oracle_lib, ar0, delay[0])
    assert not np.array_equal(one["test"], ref["test"])


def test_constant_period_takes_channel_table(monkeypatch, tmp_path, oracle_lib):
    nsub, nchan, nbin = 8, 80, 512
    ar, delay = _archive(nsub, nchan, nbin, 72, 15.0, np.full(nsub, 0.0125))
    ar0 = ar.clone()
    out, seen = _clean(ar, monkeypatch, tmp_path)
    assert seen["delay"].shape == (nchan,) and np.array_equal(seen["delay"], delay[0])
    ref = _oracle(oracle_lib, ar0, delay[0])
    assert bits_equal(out.get_weights(), ref["weights"])


def test_stored_dedispersed_archive(monkeypatch, tmp_path, oracle_lib):
    """get_dedispersed(): the reference's dedisperse is a no-op on it, only the
    residual's dededisperse rotates (input_dedispersed)."""
    nsub, nchan, nbin = 7, 64, 256
    periods = 0.05 * (1.0 - 1e-4 * np.arange(nsub))
    ar, delay = _archive(nsub, nchan, nbin, 73, 33.0, periods, dedispersed=True)
    ar0 = ar.clone()
    out, seen = _clean(ar, monkeypatch, tmp_path)
    assert seen["input_dedispersed"] and seen["delay"].shape == (nsub, nchan)
    ref = _oracle(oracle_lib, ar0, delay, input_dedispersed=True)
    assert bits_equal(out.get_weights(), ref["weights"])
    wrong = _oracle(oracle_lib, ar0, delay, input_dedispersed=False)
    assert not np.array_equal(wrong["test"], ref["test"])


def test_zero_dm_takes_integer_rotation(monkeypatch, tmp_path, oracle_lib):
    nsub, nchan, nbin = 6, 48, 100          # integral delays: any nbin
    ar, delay = _archive(nsub, nchan, nbin, 74, 0.0, np.full(nsub, 0.02))
    ar0 = ar.clone()
    out, seen = _clean(ar, monkeypatch, tmp_path)
    assert seen["delay"] is None and np.all(seen["shift"] == 0)
    d = ar0.get_data()
    ref = oracle_lib.clean_loop((d[:, 0] + d[:, 1]).astype(np.float32), ar0.get_weights(), np.zeros(nchan, np.int32))
    assert bits_equal(out.get_weights(), ref["weights"])


def test_rotate_profiles2_matches_oracle_and_channel_table(oracle_lib):
    """ic_rotate_profiles2 (per-profile phasors evaluated on the device) equals
    the oracle's per-profile rotation, and, for rows that are all the same,
    ic_rotate_profiles (the host-built channel table) bit for bit."""
    from iterative_cleaner_amd import _native
    rng = np.random.default_rng(5)
    for nbin in (64, 256, 1024, 2048, 4096):
        nsub, nchan = 4, 9
        d = rng.uniform(-3 * nbin, 3 * nbin, (nsub, nchan))
        d[0, 0], d[1, 1], d[2, 2] = 0.0, 5.0, -0.5
        x = (rng.standard_normal((nsub, nchan, nbin)) * 30).astype(np.float32)
        x[1, 2, 7] = np.nan
        for sign in (1, -1):
            got = _native.rotate_profiles(x, d, sign)
            want = oracle_lib.rotate(x, d, sign)
            assert np.array_equal(got.view(np.uint32), want.view(np.uint32)) or \
                np.all((got == want) | (np.isnan(got) & np.isnan(want))), (nbin, sign)
            rows = np.broadcast_to(d[0], (nsub, nchan)).copy()
            a = _native.rotate_profiles(x, rows, sign)
            b = _native.rotate_profiles(x, d[0], sign)
            assert np.all((a == b) | (np.isnan(a) & np.isnan(b))), (nbin, sign)
            assert np.array_equal(a[~np.isnan(a)].view(np.uint32), b[~np.isnan(b)].view(np.uint32))


@pytest.mark.parametrize("nbin", [128, 1024, 4096])
def test_session_per_profile_delays_match_oracle(nbin, oracle_lib):
    """The loop with ic_set_delays2 (and with input_dedispersed) against the C
    oracle: template, amplitudes, status, weights, diagnostics, residual."""
    from iterative_cleaner_amd import _native, synth
    from helpers import bits_equal_nan
    nsub, nchan = 6, 70
    data, w0, shift = synth.make_cube(nsub, nchan, nbin, 80 + nbin % 7, 0.2)
    raw = np.ascontiguousarray(data[:, 0])
    delay = synth.per_profile_delays(shift, nbin, nsub)
    for ided in (False, True):
        ref = oracle_lib.clean_loop(raw, w0, shift, want_residual=True, want_details=True, delay=delay,
                                    input_dedispersed=ided)
        with _native.GpuSession(nsub, nchan, nbin, 5, device=0, delay=delay, input_dedispersed=ided) as s:
            s.upload(raw, w0, np.zeros(nchan, np.int32))
            out = s.run()
            T = s.template()
            amp, info = s.fit()
            sd, mn, pt, ff = s.diagnostics()
            R = s.residual()
        assert out["loops"] == ref["loops"]
        assert bits_equal(T, ref["T"][out["n_iter"] - 1])
        assert bits_equal(amp, ref["amp"]) and bits_equal(info, ref["info"])
        assert bits_equal(out["weights"], ref["weights"])
        assert bits_equal(sd, ref["std"]) and bits_equal(mn, ref["mean"]) and bits_equal(pt, ref["ptp"])
        assert bits_equal_nan(R, ref["residual"])
