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


def test_algorithmic_bytes_of_the_fit_sweep():
    stats = {"fit_profile_sweeps": 1000, "fit_tail_sweeps": 10}
    assert bench.algorithmic_bytes("k_fit_pass", 2, 3, 1024, 30, stats, 1) == 4 * 1024 * 1000
    assert bench.algorithmic_bytes("k_fit_tail", 2, 3, 1024, 3, stats, 2) == 4 * 1024 * 10 * 2
