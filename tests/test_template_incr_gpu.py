"""The incremental template stage (k_chan_delta): from the second iteration on
the window totals and fscrunch partials move through the channels whose weight
changed, exact where every subset sum of a super-block column is exact
(k_chan_partials' ExTrack flags), summed again in canonical order elsewhere.
Every output must be the same bits as the full passes (option template_incr 0),
including on data built to make columns inexact (values spanning more than
2^21 within a column, zeros, subnormals), with fractional weights, channel
shards, and against the C oracle.  (A non-finite sample makes the template
non-finite everywhere; its columns fail ExTrack and take the full sums.)"""
import numpy as np
import pytest

from helpers import bits_equal

pytestmark = pytest.mark.gpu


def _cube(shape, seed, rough):
    from iterative_cleaner_amd import synth
    nsub, nchan, nbin = shape
    data, w0, shift = synth.make_cube(nsub, nchan, nbin, seed, 0.1)
    raw = np.ascontiguousarray(data[:, 0])
    if rough:
        rng = np.random.default_rng(seed)
        ch = rng.choice(nchan, size=max(4, nchan // 16), replace=False)
        raw[:, ch[0::4]] *= np.float32(1e-7)          # a column spans > 2^21
        raw[:, ch[1::4], ::7] = 0.0                      # exact zeros
        raw[:, ch[2::4], ::5] = np.float32(1e-41)        # subnormals
        raw[:, ch[3::4]] *= np.float32(3e5)
    return raw, w0, shift


def _run(monkeypatch, raw, w0, shift, incr, tail=None, max_iter=5):
    from iterative_cleaner_amd import _native
    nsub, nchan, nbin = raw.shape
    with _native.GpuSession(nsub, nchan, nbin, max_iter=max_iter, device=0,
                            options={"template_incr": 1 if incr else 0}) as s:
        if tail is not None:
            s.set_fit_tail(tail)
        s.upload(raw, w0, shift)
        out = s.run()
        T = s.template()
        amp, info = s.fit()
        diag = s.diagnostics()
    return out, T, amp, info, diag


def _same(a, b):
    oa, Ta, aa, ia, da = a
    ob, Tb, ab, ib, db = b
    assert oa["loops"] == ob["loops"] and oa["n_iter"] == ob["n_iter"]
    assert bits_equal(oa["weights"], ob["weights"]) and bits_equal(oa["test"], ob["test"])
    assert np.array_equal(oa["changed"], ob["changed"]) and np.array_equal(oa["nzero"], ob["nzero"])
    assert bits_equal(Ta, Tb) and bits_equal(aa, ab) and bits_equal(ia, ib)
    for x, y in zip(da, db):
        assert bits_equal(x, y)


@pytest.mark.parametrize("shape", [(12, 600, 256), (10, 512, 1024), (6, 300, 100), (8, 520, 512), (6, 300, 1000),
                                   (4, 260, 2048)])
@pytest.mark.parametrize("rough", [False, True])
def test_incremental_template_is_bit_identical(monkeypatch, shape, rough):
    raw, w0, shift = _cube(shape, 11, rough)
    _same(_run(monkeypatch, raw, w0, shift, True), _run(monkeypatch, raw, w0, shift, False))


def test_incremental_template_fractional_weights(monkeypatch):
    from iterative_cleaner_amd import synth
    raw, w0, shift = _cube((8, 520, 256), 3, True)
    w0 = synth.fractional_weights(w0)
    _same(_run(monkeypatch, raw, w0, shift, True), _run(monkeypatch, raw, w0, shift, False))


def test_incremental_template_matches_c_oracle(monkeypatch, oracle_lib):
    raw, w0, shift = _cube((8, 520, 256), 21, True)
    out, T, amp, info, _ = _run(monkeypatch, raw, w0, shift, True, tail=0)
    ref = oracle_lib.clean_loop(raw, w0, shift, want_details=True)
    assert out["loops"] == ref["loops"]
    assert bits_equal(out["weights"], ref["weights"])
    assert bits_equal(T, ref["T"][out["n_iter"] - 1])
    assert bits_equal(amp, ref["amp"]) and bits_equal(info, ref["info"])


def test_incremental_template_channel_shards(monkeypatch):
    """In-process channel shards (the session's grouped transport) with the
    incremental stage reproduce one session with full passes."""
    from iterative_cleaner_amd import sharded
    raw, w0, shift = _cube((8, 1024, 256), 5, True)
    ref = _run(monkeypatch, raw, w0, shift, False)
    res = sharded.clean_cube_local(raw, w0, shift, 4)
    assert res["loops"] == ref[0]["loops"]
    assert bits_equal(res["weights"], ref[0]["weights"])
