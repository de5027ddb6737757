"""The forked diagnostics of the exact fit (ic_session.hip fork_diag): after a
fit round the profiles already fitted are measured on a second stream while
the late rounds and the tail run, the rest after the fit.  Every output must be
the same bits as the unforked schedule (option diag_fork 0), at every fork round,
with both tail schedules, at the chain-layout profile lengths (1024, 2048,
4096) and the row-layout ones (256, 512: k_diag_p2), and against the C oracle
on whole subints."""
import numpy as np
import pytest

from helpers import bits_equal, nan_equal

pytestmark = pytest.mark.gpu


def _run(monkeypatch, shape, fork, tail, seed=5, rfi=0.1, split=2):
    from iterative_cleaner_amd import _native, synth
    nsub, nchan, nbin = shape
    data, w0, shift = synth.make_cube(nsub, nchan, nbin, seed, rfi)
    raw = np.ascontiguousarray(data[:, 0])
    with _native.GpuSession(nsub, nchan, nbin, max_iter=5, device=0,
                            options={"diag_fork": fork, "tail_split": split}) as s:
        if tail is not None:
            s.set_fit_tail(tail)
        s.upload(raw, w0, shift)
        out = s.run()
        amp, info = s.fit()
        diag = s.diagnostics()
        stats = s.run_stats()
    return raw, w0, shift, out, amp, info, diag, stats


@pytest.mark.parametrize("shape", [(16, 256, 1024), (6, 256, 2048), (4, 192, 4096), (24, 256, 256),
                                   (16, 300, 512)])
@pytest.mark.parametrize("tail", [0, 512, None])
def test_fork_is_bit_identical(monkeypatch, shape, tail):
    ref = _run(monkeypatch, shape, 0, tail)
    for fork in (1, 3, 5):
        got = _run(monkeypatch, shape, fork, tail)
        _, _, _, o0, a0, i0, d0, _ = ref
        _, _, _, o1, a1, i1, d1, _ = got
        assert o1["loops"] == o0["loops"]
        assert bits_equal(o1["weights"], o0["weights"])
        assert nan_equal(o1["test"], o0["test"]) and bits_equal(o1["test"], o0["test"])
        assert bits_equal(a1, a0) and bits_equal(i1, i0)
        for name, x0, x1 in zip(("std", "mean", "ptp", "fftmax"), d0, d1):
            assert bits_equal(x1, x0), (fork, name)


def test_fork_matches_c_oracle_whole_subints(monkeypatch, oracle_lib):
    """Rounds only, the fork after round 3: the last iteration's fit and std /
    mean / ptp of every profile equal the C oracle's on the same template."""
    raw, w0, shift, out, amp, info, diag, _ = _run(monkeypatch, (12, 512, 1024), 3, 0, seed=9)
    ref = oracle_lib.clean_loop(raw, w0, shift, want_details=True)
    assert out["loops"] == ref["loops"]
    assert bits_equal(out["weights"], ref["weights"])
    assert bits_equal(amp, ref["amp"]) and bits_equal(info, ref["info"])
    for name, x in zip(("std", "mean", "ptp"), diag[:3]):
        assert nan_equal(x, ref[name]) and x.dtype == ref[name].dtype, name
    ff = ref["fft"]
    assert np.all(np.abs(diag[3] - ff) <= 1e-9 * np.abs(ff)), "fftmax"


@pytest.mark.parametrize("shape", [(40, 512, 1024), (30, 512, 512), (12, 512, 2048), (24, 300, 256)])
@pytest.mark.parametrize("split", [0, 1])
def test_tail_split_is_bit_identical(monkeypatch, shape, split):
    """Option tail_split: at the hand-over to k_fit_tail the fork round's
    survivors that are already fitted are measured on the second stream beside
    the tail (their list minus the tail's, marked), the tail's after it.  The
    same bits as the unforked schedule, with the hand-over before and after the
    fork round."""
    ref = _run(monkeypatch, shape, 0, None)
    for fork, tail in ((1, 4096), (3, None), (2, 1024)):
        got = _run(monkeypatch, shape, fork, tail, split=split)
        assert got[3]["loops"] == ref[3]["loops"]
        assert bits_equal(got[3]["weights"], ref[3]["weights"]) and bits_equal(got[3]["test"], ref[3]["test"])
        assert bits_equal(got[4], ref[4]) and bits_equal(got[5], ref[5])
        for name, x0, x1 in zip(("std", "mean", "ptp", "fftmax"), ref[6], got[6]):
            assert bits_equal(x1, x0), (fork, tail, name)
