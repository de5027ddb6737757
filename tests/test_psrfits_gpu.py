"""The CLI on a synthetic PSRFITS archive (config C1's "synthetic PSRFITS
archive"): load through the hand-rolled reader, clean
on the GPU, write the cleaned archive back as PSRFITS.  The zap mask in the
output's DAT_WTS must equal the C oracle's loop on the decoded int16 samples."""
import numpy as np
import pytest

from helpers import bits_equal

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("extra", [[], ["-p"], ["-u", "-c", "4"]])
def test_cli_psrfits_in_out(tmp_path, monkeypatch, capsys, extra, oracle_lib):
    from iterative_cleaner_amd import archive as ica
    from iterative_cleaner_amd import cleaner, psrfits, synth
    monkeypatch.chdir(tmp_path)
    synth.make_archive(16, 64, 128, seed=41, rfi_frac=0.2, npol=2, filename="obs.sf").unload("obs.sf")
    src = ica.Archive_load("obs.sf")
    dec = src.get_data()
    cube = (dec[:, 0] + dec[:, 1]).astype(np.float32)          # archive.py pscrunch
    cth = 4.0 if "-c" in extra else 5.0
    ref = oracle_lib.clean_loop(cube, src.get_weights(), src.get_dm_shift(), cth, 5.0)
    cleaner.main(cleaner.parse_arguments(["-l", *extra, "obs.sf"]))
    out = capsys.readouterr().out
    assert "Cleaned archive: obs_cleaned.ar" in out
    assert psrfits.is_psrfits("obs_cleaned.ar")
    res = ica.Archive_load("obs_cleaned.ar")
    assert bits_equal(res.get_weights(), ref["weights"])
    assert res.get_npol() == (1 if "-p" in extra else 2)
    if "-p" not in extra:
        assert np.array_equal(res.get_data(), dec)              # samples untouched, quantisation kept
    if "-u" in extra:
        assert any("_residual_" in p.name for p in tmp_path.iterdir())


def test_cli_stokes_archive_cleans_total_intensity(tmp_path, monkeypatch, capsys, oracle_lib):
    """An IQUV (Stokes) PSRFITS archive: psrchive's pscrunch keeps I = pol 0, so
    the loop must clean pol 0 (not pol0 + pol1, the AA+BB rule)."""
    from iterative_cleaner_amd import archive as ica
    from iterative_cleaner_amd import cleaner, synth
    monkeypatch.chdir(tmp_path)
    data, w, shift = synth.make_cube(12, 64, 128, 52, 0.2, npol=4)
    rng = np.random.default_rng(52)
    data[:, 1] = rng.standard_normal(data[:, 1].shape).astype(np.float32)     # Q: noise ...
    data[rng.integers(0, 12, 20), 1, rng.integers(0, 64, 20), :] += 40.0     # ... with Q-only RFI
    ica.Archive(data, w, shift, filename="iquv.sf", state="Stokes").unload("iquv.sf")
    src = ica.Archive_load("iquv.sf")
    assert src.get_state() == "Stokes"
    dec = src.get_data()
    ref = oracle_lib.clean_loop(np.ascontiguousarray(dec[:, 0]), src.get_weights(), src.get_dm_shift())
    wrong = oracle_lib.clean_loop((dec[:, 0] + dec[:, 1]).astype(np.float32), src.get_weights(),
                                  src.get_dm_shift())
    assert not bits_equal(ref["weights"], wrong["weights"])     # the rule matters on this archive
    cleaner.main(cleaner.parse_arguments(["-l", "-q", "iquv.sf"]))
    res = ica.Archive_load("iquv_cleaned.ar")
    assert res.get_state() == "Stokes" and res.get_npol() == 4
    assert bits_equal(res.get_weights(), ref["weights"])


@pytest.mark.parametrize("periods", ["constant", "per_row"])
def test_cli_foreign_psrfits_fractional_dedispersion(tmp_path, monkeypatch, capsys, oracle_lib, periods):
    """A PSRFITS file without the stand-in's columns, with DM / DAT_FREQ / PERIOD:
    dedispersed as psrchive would, by default (no switch): the FFT phase rotation
    by the fractional delays from DM, the channel frequencies and each row's
    folding period (per-profile delays, ic_set_delays2, when the rows' periods
    differ).  The zap mask equals the C oracle's loop with those delays."""
    from iterative_cleaner_amd import archive as ica
    from iterative_cleaner_amd import cleaner, dedispersion, psrfits, synth
    monkeypatch.chdir(tmp_path)
    monkeypatch.delenv("IC_DEDISPERSION", raising=False)
    data, w, shift = synth.make_cube(10, 64, 256, 61, 0.2, npol=2)
    ar = ica.Archive(data, w, np.zeros(64, np.int64), filename="dm.sf")
    ar._chan_freqs = 1300.0 + np.arange(64) * 3.0
    ar._period = 0.0125 if periods == "constant" else 0.0125 * (1.0 + 3e-4 * np.cos(np.arange(10)))
    ar._dm = 20.0
    psrfits.save(ar, "dm.sf", stand_in_meta=False)
    src = psrfits.load("dm.sf")
    delay = src.get_dm_delay()
    assert delay is not None and np.any(delay != np.rint(delay))
    assert delay.shape == ((64,) if periods == "constant" else (10, 64))
    want = dedispersion.delays_from_dm(20.0, ar._chan_freqs, 1400.0, np.broadcast_to(ar._period, (10,)), 256)
    assert np.array_equal(delay, want[0] if periods == "constant" else want)
    dec = src.get_data()
    cube = (dec[:, 0] + dec[:, 1]).astype(np.float32)
    ref = oracle_lib.clean_loop(cube, src.get_weights(), src.get_dm_shift(), delay=delay)
    cleaner.main(cleaner.parse_arguments(["-l", "-q", "dm.sf"]))
    res = ica.Archive_load("dm_cleaned.ar")
    assert bits_equal(res.get_weights(), ref["weights"])
