"""BASELINE.json's other configurations at full size on one MI355X, generated
in HBM exactly as bench.py does (bench.make_cube_device /
make_block_cube_device):

* C3  1024 x 8192 x 1024 (34 GB): determinism, 8 in-process channel shards
  bit-equal to the single session, the final template against the oracle's
  (whole archive), sampled-subint oracle checks of the exact
  fit and the diagnostics, whole-archive oracle test values and weights;
* C4  128 x 1024 x 512 archives through batch.clean_batch (one lane and two):
  every archive bit-equal to its own single session, and one of them against
  the whole loop of the C oracle (helpers.check_whole_loop);
* C5  256 x 1024 x 4096, 30 % RFI, a seed whose loop runs to max_iter: the
  whole loop against the C oracle, the residual cube (ic_get_residual, what -u
  unloads) included.

C3's sampled checks: the whole-loop oracle at 34 GB would need ~140 GB of host
memory, so each stage of its final iteration is checked on its own (a subint's
fit cube depends on nothing outside it) for sampled subints, and the test
values of the GPU's diagnostics on the whole archive."""
import numpy as np
import pytest

from helpers import bits_equal, check_whole_loop

pytestmark = pytest.mark.gpu


def _details(s, residual=False):
    out = s.run()
    out["amp"], out["info"] = s.fit()
    out["std"], out["mean"], out["ptp"], out["fft"] = s.diagnostics()
    out["T"] = s.template()
    if residual:
        out["residual"] = s.residual()
    return out


def _check_sampled_subints(oracle_lib, raw, w0, shift, one, subs):
    """Fit + residual + diagnostics of whole subints against the oracle, given the
    GPU's final template (bit-exact; fftmax within 1e-9 relative)."""
    nbin = raw.shape[2]
    nchan = raw.shape[1]
    D = oracle_lib.fit_cube(raw[subs], w0[subs], shift)
    amp, info, R = oracle_lib.fit_residual(D.reshape(-1, nbin), one["T"])
    assert bits_equal(amp.reshape(len(subs), nchan), one["amp"][subs]), "leastsq amplitudes differ"
    assert bits_equal(info.reshape(len(subs), nchan), one["info"][subs])
    Rd = R.reshape(len(subs), nchan, nbin)
    idx = (np.arange(nbin)[None, :] - shift[:, None]) % nbin
    Rdisp = np.take_along_axis(Rd, np.broadcast_to(idx[None], Rd.shape), axis=2)   # dededisperse
    if "residual" in one:
        assert bits_equal(Rdisp, one["residual"][subs]), "residual cube (-u) differs"
    X = Rdisp * w0[subs][:, :, None]
    sd, mn, pt, ff = oracle_lib.diagnostics(X, w0[subs] != 0)
    assert bits_equal(sd, one["std"][subs]) and bits_equal(mn, one["mean"][subs])
    assert bits_equal(pt, one["ptp"][subs])
    g = one["fft"][subs]
    assert np.all((g == ff) | (np.abs(g - ff) <= 1e-9 * np.abs(ff)))


def _check_test_values(oracle_lib, w0, one):
    test = oracle_lib.test_values(w0 != 0, one["std"], one["mean"], one["ptp"], one["fft"], 5.0, 5.0)
    assert bits_equal(test, one["test"])
    assert bits_equal(np.where(one["test"] >= 1.0, np.float32(0), w0).astype(np.float32), one["weights"])


# ----------------------------------------------------------------------- C3
@pytest.fixture(scope="module")
def c3():
    import torch

    import bench
    from iterative_cleaner_amd import _native
    nsub, nchan, nbin, seed, rfi = bench.WORKLOADS["C3"]
    dev = torch.device("cuda", 0)
    cube, w0, shift = bench.make_block_cube_device(nsub, nchan, nbin, seed, rfi, 0, nchan, dev)
    torch.cuda.synchronize()
    with _native.GpuSession(nsub, nchan, nbin, device=0) as s:
        s.upload_device(cube.data_ptr(), w0.data_ptr(), shift.data_ptr())
        outs = [_details(s), _details(s)]
    # the weights the final template was built from (iteration k-1's, ic.py:88-94):
    # the same loop stopped one iteration earlier
    k = outs[0]["n_iter"]
    if k == 1:
        w_prev = w0.cpu().numpy()
    elif outs[0]["changed"][-1] == 0:
        w_prev = outs[0]["weights"]
    else:
        with _native.GpuSession(nsub, nchan, nbin, max_iter=k - 1, device=0) as s:
            s.upload_device(cube.data_ptr(), w0.data_ptr(), shift.data_ptr())
            w_prev = s.run()["weights"]
    outs[0]["w_prev"] = w_prev
    host = (cube.cpu().numpy(), w0.cpu().numpy(), shift.cpu().numpy().astype(np.int64))
    del cube, w0, shift
    torch.cuda.empty_cache()
    yield host, outs


def test_c3_deterministic(c3):
    _, (a, b) = c3
    assert a["loops"] == b["loops"] and np.array_equal(a["changed"], b["changed"])
    for key in ("weights", "test", "amp", "info", "std", "mean", "ptp", "fft", "T"):
        assert bits_equal(a[key], b[key]), key
    assert 0 < int((a["weights"] == 0).sum()) < a["weights"].size // 2


def test_c3_eight_channel_shards(c3):
    from iterative_cleaner_amd import sharded
    (raw, w0, shift), (one, _) = c3
    out = sharded.clean_cube_local(raw, w0, shift, 8, want_details=True)
    assert out["loops"] == one["loops"] and np.array_equal(out["changed"], one["changed"])
    for key in ("weights", "test", "amp", "info", "std", "mean", "ptp", "fft", "T"):
        assert bits_equal(out[key], one[key]), key


def test_c3_template(c3, oracle_lib):
    """The final template against the oracle's, whole archive: 32 channel
    super-blocks, the deepest canonical channel tree of the configs
    (tests/test_fullsize_gpu.py does the same for C2)."""
    (raw, w0, shift), (one, _) = c3
    assert bits_equal(oracle_lib.template(raw, one["w_prev"], shift), one["T"])


def test_c3_sampled_subints_and_test_values(c3, oracle_lib):
    (raw, w0, shift), (one, _) = c3
    subs = np.sort(np.random.default_rng(3).choice(raw.shape[0], size=3, replace=False))
    _check_sampled_subints(oracle_lib, raw, w0, shift, one, subs)
    _check_test_values(oracle_lib, w0, one)


# ----------------------------------------------------------------------- C4
@pytest.fixture(scope="module")
def c4():
    import torch

    import bench
    nsub, nchan, nbin, seed, rfi = bench.WORKLOADS["C4"]
    dev = torch.device("cuda", 0)
    archives = []
    for k in range(4):
        cube, w0, shift = bench.make_cube_device(nsub, nchan, nbin, seed + k, rfi, dev)
        archives.append((cube.cpu().numpy(), w0.cpu().numpy(), shift.cpu().numpy().astype(np.int64)))
        del cube, w0, shift
    torch.cuda.empty_cache()
    return archives


@pytest.mark.parametrize("lanes", [1, 2])
def test_c4_batch_equals_single_sessions(c4, lanes, oracle_lib):
    from iterative_cleaner_amd import _native, batch
    nsub, nchan, nbin = c4[0][0].shape
    got = list(batch.clean_batch(iter(c4), (nsub, nchan, nbin), device=0, lanes=lanes))
    assert len(got) == len(c4)
    for k, (raw, w0, shift) in enumerate(c4):
        with _native.GpuSession(nsub, nchan, nbin, device=0) as s:
            s.upload(raw, w0, shift)
            one = _details(s)
        assert got[k]["loops"] == one["loops"] and np.array_equal(got[k]["changed"], one["changed"])
        assert bits_equal(got[k]["weights"], one["weights"]) and bits_equal(got[k]["test"], one["test"])
        if k == 1 and lanes == 1:
            check_whole_loop(oracle_lib, raw, w0, shift, one)


# ----------------------------------------------------------------------- C5
@pytest.fixture(scope="module")
def c5():
    import torch

    import bench
    from iterative_cleaner_amd import _native
    nsub, nchan, nbin, seed, rfi = bench.WORKLOADS["C5"]
    dev = torch.device("cuda", 0)
    cube, w0, shift = bench.make_cube_device(nsub, nchan, nbin, seed, rfi, dev)
    torch.cuda.synchronize()
    with _native.GpuSession(nsub, nchan, nbin, max_iter=5, device=0) as s:
        s.upload_device(cube.data_ptr(), w0.data_ptr(), shift.data_ptr())
        one = _details(s, residual=True)
    host = (cube.cpu().numpy(), w0.cpu().numpy(), shift.cpu().numpy().astype(np.int64))
    del cube, w0, shift
    torch.cuda.empty_cache()
    return host, one


def test_c5_runs_to_max_iter(c5):
    _, one = c5
    assert one["n_iter"] == 5 and one["loops"] == 5 and not one["converged"]
    assert one["weights"].size == 256 * 1024 and (one["weights"] == 0).sum() > 0.05 * one["weights"].size


def test_c5_whole_loop_against_oracle(c5, oracle_lib):
    (raw, w0, shift), one = c5
    check_whole_loop(oracle_lib, raw, w0, shift, one, residual=True)
