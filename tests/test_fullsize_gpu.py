"""Parity at BASELINE.json's full size on bench.py's own C2 workload
(360 x 3200 x 1024, generated in HBM by bench.make_cube_device):

* determinism: two runs give bit-identical masks, test values, amplitudes;
* channel shards: 4 in-process shards give the single session's bits;
* the whole loop against the C oracle run independently on the same archive
  (threaded over profiles, subints and lines; helpers.check_whole_loop): loop
  count, per-loop change / zero counts, final template, every profile's
  leastsq amplitude and status, std / mean / ptp and the weights bit for bit,
  fftmax and the oracle's own test values within 1e-9.
"""
import numpy as np
import pytest

from helpers import bits_equal, check_whole_loop

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


def test_fullsize_whole_loop_against_oracle(c2, oracle_lib):
    (raw, w0, shift), (one, _) = c2
    check_whole_loop(oracle_lib, raw, w0, shift, one)
