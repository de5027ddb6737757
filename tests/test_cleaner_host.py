"""Host-side rules of the drop-in clean() (no GPU: the loop result is stubbed):
print order of the reference (iterative_cleaner.py:82-145, :284-285), the
polarisation state of the loop input (pscrunch: AA+BB, or I for Stokes data),
and slice-only channel loading for channel-sharded runs."""
import argparse

import numpy as np
import pytest

from iterative_cleaner_amd import archive as ica
from iterative_cleaner_amd import archive_io, cleaner, psrfits, synth


def _fake_loop(out):
    def run_loop(cube, w0, shift, args, **kw):
        nsub, nchan = np.shape(w0)
        res = dict(out)
        res["test"] = np.zeros((nsub, nchan))
        res["weights"] = np.asarray(w0, np.float32)
        return res
    return run_loop


@pytest.mark.parametrize("quiet", [False, True])
def test_bad_status_lines_in_reference_order(monkeypatch, capsys, tmp_path, quiet):
    """remove_profile1d prints "Bad status ..." for every failed fit of every loop,
    between "Loop: x" and "Differences ...", even with -q (ic.py:284-285)."""
    monkeypatch.chdir(tmp_path)
    ica.Archive(*synth.make_cube(3, 4, 16, 1, 0.0)).unload("a.ar")
    out = dict(n_iter=2, converged=True, loops=2, changed=np.array([5, 0]), nzero=np.array([2, 2]),
               bad_fits=np.array([2, 1]))
    monkeypatch.setattr(cleaner, "run_loop", _fake_loop(out))
    argv = ["-l", "a.ar"] + (["-q"] if quiet else [])
    cleaner.clean(ica.Archive_load("a.ar"), cleaner.parse_arguments(argv), "a.ar")
    bad = cleaner.BAD_STATUS
    if quiet:
        want = "%s\n%s\n%s\n" % (bad, bad, bad)
    else:
        want = ("Total number of profiles: 12\nLoop: 1\n%s\n%s\n"
                "Differences to previous weights: 5  RFI fraction: %s\nLoop: 2\n%s\n"
                "Differences to previous weights: 0  RFI fraction: %s\nRFI removal stops after 2 loops.\n"
                % (bad, bad, 2 / 12.0, bad, 2 / 12.0))
    assert capsys.readouterr().out == want


def test_stokes_pscrunch_is_pol0():
    data, w, shift = synth.make_cube(2, 3, 8, 4, 0.0, npol=4)
    ar = ica.Archive(data, w, shift, state="Stokes")
    assert np.array_equal(cleaner._loop_input(ar), data[:, 0])        # I
    ar.pscrunch()
    assert ar.get_state() == "Intensity" and np.array_equal(ar.get_data()[:, 0], data[:, 0])
    coh = ica.Archive(data, w, shift)                                   # AABBCRCI
    assert coh.get_state() == "Coherence" and cleaner._loop_input(coh).shape == data.shape
    coh.pscrunch()
    assert np.array_equal(coh.get_data()[:, 0], (data[:, 0] + data[:, 1]).astype(np.float32))
    with pytest.raises(ValueError):
        ica.Archive(data[:, :1], w, shift, state="Stokes")


def test_psrfits_pol_type_round_trip(tmp_path):
    data, w, shift = synth.make_cube(2, 5, 16, 6, 0.0, npol=4)
    for state, pol_type in (("Stokes", "IQUV"), ("Coherence", "AABBCRCI")):
        path = str(tmp_path / ("%s.sf" % state))
        ica.Archive(data, w, shift, state=state).unload(path)
        assert pol_type in open(path, "rb").read(2880 * 4).decode("ascii", "replace")
        assert ica.Archive_load(path).get_state() == state


@pytest.mark.parametrize("suffix", [".ar", ".sf"])
def test_channel_slice_loading(tmp_path, suffix):
    """load_channels reads only [c0, c1) and equals the whole load, sliced."""
    data, w, shift = synth.make_cube(5, 40, 32, 8, 0.2, npol=2)
    path = str(tmp_path / ("obs" + suffix))
    ica.Archive(data, w, shift).unload(path)
    assert archive_io.probe_shape(path) == (5, 2, 40, 32)
    full = ica.Archive_load(path)
    for c0, c1 in ((0, 13), (13, 40), (7, 8)):
        part = ica.load_channels(path, c0, c1)
        assert part._chan_range == (c0, c1) and part._nchan_total == 40
        assert np.array_equal(part.get_data(), full.get_data()[:, :, c0:c1])
        assert np.array_equal(part.get_weights(), full.get_weights()[:, c0:c1])
        assert np.array_equal(part.get_dm_shift(), full.get_dm_shift()[c0:c1])
        assert part.get_state() == full.get_state()
    with pytest.raises(ValueError):
        ica.load_channels(path, 30, 50)


def test_slice_without_sharding_is_refused():
    args = argparse.Namespace(max_iter=5, chanthresh=5, subintthresh=5, pulse_region=[0, 0, 1])
    with pytest.raises(ValueError):
        cleaner.run_loop(np.zeros((2, 3, 8), np.float32), np.ones((2, 3), np.float32), np.zeros(3, np.int64),
                         args, nchan_total=6)


# ------------------------------------------------------------ psrchive's dedispersion
def test_dedispersion_of_a_psrchive_like_archive():
    """An archive with only psrchive's methods: delays from DM, channel
    frequencies and each Integration's folding period (dedispersion.py);
    per-profile when the periods differ, per-channel when they agree, integer
    shifts when every delay is integral, an error at an nbin the rotation cannot
    serve (never a silent rounding)."""
    from psrchive_like import PsrchiveLike

    from iterative_cleaner_amd import cleaner, dedispersion
    data = np.zeros((4, 1, 6, 128), np.float32)
    w = np.ones((4, 6), np.float32)
    freqs = 150.0 + np.arange(6) * 0.5
    per = np.array([0.1, 0.1000001, 0.0999999, 0.1])
    shift, delay = cleaner._dedispersion(PsrchiveLike(data, w, 12.0, freqs, per, 151.0))
    assert np.array_equal(shift, np.zeros(6)) and delay.shape == (4, 6)
    assert np.array_equal(delay, dedispersion.delays_from_dm(12.0, freqs, 151.0, per, 128))
    shift, delay = cleaner._dedispersion(PsrchiveLike(data, w, 12.0, freqs, np.full(4, 0.1), 151.0))
    assert delay.shape == (6,)
    shift, delay = cleaner._dedispersion(PsrchiveLike(data, w, 0.0, freqs, per, 151.0))
    assert delay is None and np.array_equal(shift, np.zeros(6))
    with pytest.raises(ValueError, match="power-of-two nbin"):
        cleaner._dedispersion(PsrchiveLike(np.zeros((4, 1, 6, 100), np.float32), w, 12.0, freqs, per, 151.0))


def test_stored_dedispersed_integer_archive_rolls_back_exactly():
    """An archive stored dedispersed with integer shifts: the host moves its
    samples back to the dispersed frame (cleaner._to_dispersed), exactly: the
    stand-in's own dedisperse of that gives the stored samples bit for bit."""
    from iterative_cleaner_amd import archive as ica
    from iterative_cleaner_amd import cleaner, synth
    data, w, shift = synth.make_cube(3, 10, 64, 2, 0.2, npol=2)
    src = ica.Archive(data, w, shift)
    src.dedisperse()
    stored = src.get_data()
    back = cleaner._to_dispersed(stored, shift)
    assert np.array_equal(back, data)
    assert cleaner._stored_dedispersed(src) and not cleaner._stored_dedispersed(ica.Archive(data, w, shift))
