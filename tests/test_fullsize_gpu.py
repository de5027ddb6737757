"""Parity at BASELINE.json's full size on bench.py's own C2 workload
(360 x 3200 x 1024, generated in HBM by bench.make_cube_device), where the
whole-loop C oracle would take minutes: size-independent properties plus exact
oracle checks of every stage of the final iteration.

* determinism: two runs give bit-identical masks, test values, amplitudes;
* channel shards: 4 in-process shards give the single session's bits;
* template: the oracle's template of the previous iteration's weights equals
  the GPU's final template (whole archive);
* fit + diagnostics, sampled: for 6 random subints (all 3200 channels: a
  subint's baseline depends on nothing else) the oracle's fit cube + exact
  leastsq against the GPU's template reproduce the GPU's amplitudes/status bit
  for bit, and its diagnostics of those residuals reproduce std/mean/ptp bit for
  bit and fftmax within 1e-9 relative;
* scaling + threshold (whole archive): the oracle's median/MAD test values of
  the GPU's diagnostics equal the GPU's test values, and the weights are
  where(test >= 1, 0, w0) (ic.py:131-137).
"""
import numpy as np
import pytest

from helpers import bits_equal

pytestmark = pytest.mark.gpu

SHAPE = (360, 3200, 1024)


def _run(s):
    out = s.run()
    out["amp"], out["info"] = s.fit()
    out["std"], out["mean"], out["ptp"], out["fft"] = s.diagnostics()
    out["T"] = s.template()
    return out


@pytest.fixture(scope="module")
def c2():
    import bench
    import torch
    from iterative_cleaner_amd import _native
    _native.load_library()
    nsub, nchan, nbin, seed, rfi = bench.WORKLOADS["C2"]
    assert (nsub, nchan, nbin) == SHAPE
    dev = torch.device("cuda", 0)
    cube, w0, shift = bench.make_cube_device(nsub, nchan, nbin, seed, rfi, dev)
    torch.cuda.synchronize()
    outs = []
    with _native.GpuSession(*SHAPE, device=0) as s:
        s.upload_device(cube.data_ptr(), w0.data_ptr(), shift.data_ptr())
        outs = [_run(s), _run(s)]
    host = (cube.cpu().numpy(), w0.cpu().numpy(), shift.cpu().numpy().astype(np.int64))
    del cube, w0, shift
    torch.cuda.empty_cache()
    return host, outs


def test_fullsize_deterministic(c2):
    _, (a, b) = c2
    assert a["loops"] == b["loops"] and np.array_equal(a["changed"], b["changed"])
    for key in ("weights", "test", "amp", "info", "std", "mean", "ptp", "fft", "T"):
        assert bits_equal(a[key], b[key]), key
    assert 0 < int((a["weights"] == 0).sum()) < a["weights"].size // 2


def test_fullsize_channel_shards(c2):
    from iterative_cleaner_amd import sharded
    (raw, w0, shift), (one, _) = c2
    out = sharded.clean_cube_local(raw, w0, shift, 4, want_details=True)
    assert out["loops"] == one["loops"] and np.array_equal(out["changed"], one["changed"])
    for key in ("weights", "test", "amp", "std", "fft", "T"):
        assert bits_equal(out[key], one[key]), key


def test_fullsize_template(c2, oracle_lib):
    from iterative_cleaner_amd import _native
    (raw, w0, shift), (one, _) = c2
    k = one["n_iter"]
    assert k >= 1
    if k == 1:
        w_prev = w0
    elif one["changed"][-1] == 0:
        w_prev = one["weights"]
    else:  # weights after iteration k-1: the same loop stopped one iteration earlier
        with _native.GpuSession(*SHAPE, max_iter=k - 1, device=0) as s:
            s.upload(raw, w0, shift)
            w_prev = s.run()["weights"]
    assert bits_equal(oracle_lib.template(raw, w_prev, shift), one["T"])


def test_fullsize_sampled_fit_and_diagnostics(c2, oracle_lib):
    (raw, w0, shift), (one, _) = c2
    nsub, nchan, nbin = SHAPE
    subs = np.sort(np.random.default_rng(7).choice(nsub, size=6, replace=False))
    D = oracle_lib.fit_cube(raw[subs], w0[subs], shift)                 # dedispersed fit cube
    amp, info, R = oracle_lib.fit_residual(D.reshape(-1, nbin), one["T"])
    assert bits_equal(amp.reshape(6, nchan), one["amp"][subs]), "leastsq amplitudes differ"
    assert bits_equal(info.reshape(6, nchan), one["info"][subs])
    # residual -> dispersed frame (archive.py dededisperse) -> x w0, as ic_oracle.c's loop
    Rd = R.reshape(6, nchan, nbin)
    idx = (np.arange(nbin)[None, :] - shift[:, None]) % nbin
    X = np.take_along_axis(Rd, np.broadcast_to(idx[None], Rd.shape), axis=2)
    X = X * w0[subs][:, :, None]
    sd, mn, pt, ff = oracle_lib.diagnostics(X, w0[subs] != 0)
    assert bits_equal(sd, one["std"][subs]) and bits_equal(mn, one["mean"][subs])
    assert bits_equal(pt, one["ptp"][subs])
    g = one["fft"][subs]
    assert np.all((g == ff) | (np.abs(g - ff) <= 1e-9 * np.abs(ff)))


def test_fullsize_test_values_and_weights(c2, oracle_lib):
    (raw, w0, shift), (one, _) = c2
    test = oracle_lib.test_values(w0 != 0, one["std"], one["mean"], one["ptp"], one["fft"], 5.0, 5.0)
    assert bits_equal(test, one["test"])
    assert bits_equal(np.where(one["test"] >= 1.0, np.float32(0), w0).astype(np.float32), one["weights"])
