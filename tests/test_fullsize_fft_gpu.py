"""Parity of the FFT dedispersion mode at BASELINE.json's full size: bench.py's
own C2 workload (360 x 3200 x 1024, generated in HBM by bench.make_cube_device)
with `bench.py --dedisp fft`'s fractional delays (one per channel) and `--dedisp
fft_pp`'s (one per profile: psrchive's per-Integration folding periods), cleaned by the GPU and by the
threaded C oracle run independently on the same archive (helpers.check_whole_loop:
loop count, per-loop change / zero counts, final template, every profile's
leastsq amplitude and status, std / mean / ptp and the weights bit for bit,
fftmax and the oracle's own test values within 1e-9).  Every dedisperse /
dededisperse (iterative_cleaner.py:91, :100, :104) is the stand-in's f32 FFT
phase rotation (phase_rotation.py); the oracle's is orc_rotate.  Real psrchive:
unpinned."""
import numpy as np
import pytest

from helpers import bits_equal, check_whole_loop

pytestmark = pytest.mark.gpu

SHAPE = (360, 3200, 1024)


@pytest.fixture(scope="module", params=["fft", "fft_pp"])
def c2fft(request):
    import bench
    import torch
    from iterative_cleaner_amd import _native, synth
    _native.load_library()
    nsub, nchan, nbin, seed, rfi = bench.WORKLOADS["C2"]
    assert (nsub, nchan, nbin) == SHAPE
    if request.param == "fft":   # bench.py --dedisp fft / fft_pp
        delay = synth.fractional_delays(np.arange(nchan) % 7, nbin)
    else:
        delay = synth.per_profile_delays(np.arange(nchan) % 7, nbin, nsub)
    dev = torch.device("cuda", 0)
    cube, w0, shift = bench.make_cube_device(nsub, nchan, nbin, seed, rfi, dev)
    torch.cuda.synchronize()
    with _native.GpuSession(*SHAPE, max_iter=5, device=0, delay=delay) as s:
        s.upload_device(cube.data_ptr(), w0.data_ptr(), shift.data_ptr())
        out = s.run()
        out["amp"], out["info"] = s.fit()
        out["std"], out["mean"], out["ptp"], out["fft"] = s.diagnostics()
        out["T"] = s.template()
    host = (cube.cpu().numpy(), w0.cpu().numpy(), shift.cpu().numpy().astype(np.int64))
    del cube, w0, shift
    torch.cuda.empty_cache()
    return host, delay, out


@pytest.mark.timeout(400)
def test_fullsize_fft_whole_loop_against_oracle(c2fft, oracle_lib):
    (raw, w0, shift), delay, one = c2fft
    assert one["loops"] >= 2
    assert 0 < int((one["weights"] == 0).sum()) < one["weights"].size // 2
    check_whole_loop(oracle_lib, raw, w0, shift, one, delay=delay)
