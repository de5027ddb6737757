"""Session schedule options (ic_set_option, include/iterative_cleaner.h): range
checks, the modes each option can serve, and the sync timeout's failure path
(a session whose host wait ran out refuses every later call but destroy).
The bit-identity of each schedule is held by the tests of that schedule
(test_diag_fork_gpu, test_template_incr_gpu, test_gpu_parity's fit-cube
layouts, test_stats_gpu's row-median forms)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_option_ranges_and_modes():
    from iterative_cleaner_amd import _native
    with _native.GpuSession(4, 64, 256, device=0) as s:
        defaults = {name: s.get_option(name) for name in _native.OPTIONS}
        assert defaults == {"fit_tail": 8192, "diag_fork": 3, "fork_delay": 1, "template_incr": 1,
                            "fit_tiled": 1, "rowstat_waves": 8, "rowstat_minlen": 1024, "diag_chain": 1,
                            "sync_timeout_ms": 600000, "fit_schedule": 0, "tail_split": 2, "rot_stats": 1}
        for name, bad in (("fit_tail", -1), ("diag_fork", 65), ("diag_fork", -1), ("fork_delay", 9),
                          ("template_incr", 2), ("fit_tiled", -1), ("rowstat_waves", 2),
                          ("rowstat_minlen", 0), ("diag_chain", 3), ("sync_timeout_ms", 0),
                          ("fit_schedule", 1), ("fit_schedule", 2), ("tail_split", 3), ("rot_stats", 2),
                          ("rot_stats", -1)):
            with pytest.raises(_native.NativeError, match="IC_OPT"):
                s.set_option(name, bad)
            assert s.get_option(name) == defaults[name]
        s.set_option("diag_fork", 5)
        assert s.get_option("diag_fork") == 5
        with pytest.raises(ValueError):
            s.set_option("no_such_option", 1)
        # options 11 and 12 were the lanes schedule's until round 4: unknown now
        for opt in (11, 12):
            with pytest.raises(_native.NativeError, match="unknown option %d" % opt):
                s._check(s.lib.ic_set_option(s.h, opt, 1), "ic_set_option")
    # the fork serves the exact fit only (either dedispersion); the tiled cube
    # every exact fit and the closed form with integer dedispersion
    with _native.GpuSession(4, 64, 256, device=0, fit_mode=_native.FIT_CLOSED) as s:
        with pytest.raises(_native.NativeError, match="DIAG_FORK"):
            s.set_option("diag_fork", 3)
        s.set_option("diag_fork", 0)
    with _native.GpuSession(4, 64, 256, device=0, delay=np.zeros(64)) as s:
        assert s.get_option("diag_fork") == 3 and s.get_option("template_incr") == 1
        assert s.get_option("fit_tiled") == 1
        for name in ("template_incr", "fit_tiled", "diag_fork", "rot_stats"):
            s.set_option(name, 0)
            s.set_option(name, 1)
    with _native.GpuSession(4, 64, 256, device=0, delay=np.zeros(64), fit_mode=_native.FIT_CLOSED) as s:
        assert s.get_option("fit_tiled") == 0
        with pytest.raises(_native.NativeError, match="FIT_TILED"):
            s.set_option("fit_tiled", 1)


def test_sync_timeout_fails_the_session():
    """A 1 ms host-wait limit on a C2-sized archive (its preparation alone
    takes > 1 ms): ic_run fails, every later call on the session fails with
    IC_ESTATE, destroy succeeds (leaking the buffers its queued kernels use),
    and the device drains."""
    import torch

    from iterative_cleaner_amd import _native
    nsub, nchan, nbin = 360, 3200, 1024
    dev = torch.device("cuda", 0)
    cube = torch.zeros((nsub, nchan, nbin), dtype=torch.float32, device=dev)
    w0 = torch.ones((nsub, nchan), dtype=torch.float32, device=dev)
    shift = torch.zeros(nchan, dtype=torch.int32, device=dev)
    s = _native.GpuSession(nsub, nchan, nbin, device=0)
    s.upload_device(cube.data_ptr(), w0.data_ptr(), shift.data_ptr())
    torch.cuda.synchronize()
    s.set_option("sync_timeout_ms", 1)
    with pytest.raises(_native.NativeError, match="rc=-2"):
        s.run(fetch=False)
    for call in (lambda: s.run(fetch=False), s.fit, s.template, lambda: s.set_option("fit_tail", 0),
                 lambda: s.upload_device(cube.data_ptr(), w0.data_ptr(), shift.data_ptr())):
        with pytest.raises(_native.NativeError, match="rc=-4"):
            call()
    s.close()
    torch.cuda.synchronize()   # the leaked session's queued kernels finish
