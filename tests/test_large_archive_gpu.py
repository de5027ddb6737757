"""An exact-fit archive of more than 2^24 profiles (2050 x 8192 x 64 =
16 793 600 profiles, 4.3 GB in HBM) on one session.

The fit's round lists count their profiles in full 32-bit words (rl_pack;
an earlier packing held 24 bits and refused such sessions).  The oracle is too
slow at this size, so the single session is checked against itself cleaned
as two in-process channel shards of < 2^24 profiles each (sharded.py), which
must give the same bits (masks, test values, amplitudes and statuses)."""
import numpy as np
import pytest

from helpers import bits_equal

pytestmark = pytest.mark.gpu

SHAPE = (2050, 8192, 64)


def test_more_than_2_24_profiles_match_two_shards():
    import bench
    import torch
    from iterative_cleaner_amd import _native, sharded
    nsub, nchan, nbin = SHAPE
    assert nsub * nchan > 1 << 24 and (nsub * nchan) // 2 < 1 << 24
    _native.load_library()
    dev = torch.device("cuda", 0)
    cube, w0, shift = bench.make_cube_device(nsub, nchan, nbin, 77, 0.05, dev)
    torch.cuda.synchronize()
    with _native.GpuSession(nsub, nchan, nbin, device=0) as s:
        s.upload_device(cube.data_ptr(), w0.data_ptr(), shift.data_ptr())
        one = s.run()
        one["amp"], one["info"] = s.fit()
    raw, w0h, shifth = cube.cpu().numpy(), w0.cpu().numpy(), shift.cpu().numpy().astype(np.int64)
    del cube, w0, shift
    torch.cuda.empty_cache()
    assert one["n_iter"] > 0 and 0 < int((one["weights"] == 0).sum()) < one["weights"].size // 2
    assert int(((one["info"] >= 1) & (one["info"] <= 4)).sum()) > (nsub * nchan) // 2
    two = sharded.clean_cube_local(raw, w0h, shifth, 2, want_details=True)
    assert two["loops"] == one["loops"] and np.array_equal(two["changed"], one["changed"])
    for key in ("weights", "test", "amp", "info"):
        assert bits_equal(two[key], one[key]), key
