"""Host-side checks of bench.py's measurement plumbing (no GPU).

The bench line prices its dominant kernel against HBM traffic and VALU issue
counts taken from committed rocprofv3 PMC summaries under profiles/; they are
quoted only when they were measured on the HIP sources being timed.  These
tests keep the committed summaries in step with the sources.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def test_committed_pmc_traffic_matches_sources():
    traffic, src = bench.pmc_traffic("C2", "k_fit_pass")
    assert src is not None, "no profiles/*pmc_traffic*.json for the current HIP sources (tools/profile_c2.sh)"
    assert traffic > 0


def test_committed_pmc_valu_matches_sources():
    kernels, src = bench.pmc_valu("C2")
    assert src is not None, "no profiles/*pmc_valu*.json for the current HIP sources (tools/pmc_valu.sh)"
    for name in ("k_fit_pass", "k_diag"):
        v = kernels[name]
        assert v["launches"] > 0 and v["valu_insts_per_launch"] > 0
        assert 0.0 < v["f64_share_of_valu"] <= 1.0


def _run(**kw):
    run = {"n_iter": 3, "changed": [120000, 900, 0], "fit_profile_sweeps": 1000, "fit_tail_sweeps": 10,
           "window_moves": 360}
    run.update(kw)
    return run


def test_algorithmic_bytes_of_the_fit_sweep():
    run = _run()
    assert bench.algorithmic_bytes("k_fit_pass", 2, 3, 1024, 30, run, 1) == 4 * 1024 * 1000
    assert bench.algorithmic_bytes("k_fit_tail", 2, 3, 1024, 3, run, 2) == 4 * 1024 * 10 * 2
    assert bench.algorithmic_bytes("k_fit_state", 2, 3, 1024, 30, run, 1) == 2 * 188 * 1000


def test_template_stage_charges_only_what_it_reads():
    """C2 (360 x 3200 x 1024, 3 loops): prepare's pass and iteration 1's pass
    with the fit-cube write read / write whole cubes; the later iterations read
    the changed channels and the subints whose window moved.  At round 3's
    measured 3.72 ms per clean for every template-stage launch the rate must
    sit under the HBM peak (round 3's per-launch model said 8.9 TB/s)."""
    nsub, nchan, nbin = 360, 3200, 1024
    N = nsub * nchan * nbin
    run = _run()
    b = bench.algorithmic_bytes("k_chan_partials", nsub, nchan, nbin, 6, run, 1)
    assert b == (4 * N + 8 * N + 4 * nbin * (120000 + 900) + 4 * nchan * nbin * 360
                 + 16 * nsub * 13 * nbin * 3)
    assert b / 3.722e-3 / 1e9 < bench.HBM_PEAK_GBS
    # the fast mode writes no fit cube
    assert bench.algorithmic_bytes("k_chan_partials", nsub, nchan, nbin, 6, run, 1, exact=False) == b - 4 * N
    # one diagnostics pass per iteration, however many launches (the fork)
    assert bench.algorithmic_bytes("k_diag", nsub, nchan, nbin, 6, run, 2) == 2 * 3 * (4 * N + 44 * nsub * nchan)


def test_rates_above_peak_refuse_the_line():
    pk = {"k_chan_partials": {"sweep_gbs": 8936.1}, "k_fit_pass": {"sweep_gbs": 4660.0}, "k_window": {"sweep_gbs": None}}
    over, resident = bench.check_kernel_rates(pk, 4 * 360 * 3200 * 1024)
    assert over == {"k_chan_partials": 8936.1} and resident == {}
    # a cube the Infinity Cache holds may be re-read on-die faster than HBM: reported, not refused
    over, resident = bench.check_kernel_rates(pk, 4 * 64 * 256 * 256)
    assert over == {} and resident == {"k_chan_partials": 8936.1}


def test_rotation_bytes():
    """k_rotate (fractional dedispersion): 8 B per rotated sample; preparation
    rotates the raw cube and the fit cube, every iteration the residual, and
    the carried template rows of the subints whose window moved.  Its SURVEY
    §8(d) share is the residual's dededispersion alone (8N per iteration)."""
    nsub, nchan, nbin = 4, 6, 128
    N = nsub * nchan * nbin
    run = _run(window_moves=5)
    assert bench.algorithmic_bytes("k_rotate", nsub, nchan, nbin, 7, run, 2) == \
        2 * (8 * N * (2 + 3) + 8 * nchan * nbin * 5)
    assert bench.s8d_bytes("k_rotate", nsub, nchan, nbin, 7, 3, 2) == 8 * N * 3 * 2
