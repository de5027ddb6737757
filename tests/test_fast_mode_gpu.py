"""fit_mode 1 (IC_FIT_CLOSED, include/iterative_cleaner.h): the north star's
closed-form amplitude fused with the residual and the diagnostics.  This is
NOT the reference's arithmetic (leastsq, iterative_cleaner.py:277-278), so it
is checked against its own statement: the C oracle's orc_fit_closed, itself
pinned to the numpy expression np.sum(np.roll(T*p, sh))/np.sum(T*T) (the
products summed in the stored sample order; oracle/restated.py,
tests/test_oracle_golden.py).  Bit-exact: amplitudes, status, residual, masks,
std/mean/ptp; fftmax within 1e-9 relative, test values within 1e-9."""
import numpy as np
import pytest

from helpers import bits_equal

pytestmark = pytest.mark.gpu

CASES = [
    # (nsub, nchan, nbin, seed, rfi, extra)
    (7, 300, 64, 11, 0.2, {}),
    (5, 33, 100, 12, 0.3, {}),                 # non power-of-two nbin (generic kernel)
    (9, 70, 128, 15, 0.3, {"chanthresh": 3.0, "subintthresh": 2.5}),
    (8, 64, 256, 16, 0.2, {"pulse_region": [0.25, 40, 90]}),
    (6, 50, 512, 17, 0.2, {}),
    (5, 70, 1024, 18, 0.2, {}),
    (4, 30, 2048, 19, 0.3, {}),
    (6, 40, 4096, 13, 0.3, {}),
]


def _close(a, b, tol):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    same = (a == b) | (np.isnan(a) & np.isnan(b))
    fin = np.isfinite(a) & np.isfinite(b)
    return bool(np.all(same | (fin & (np.abs(a - b) <= tol * np.maximum(1.0, np.abs(b))))))


@pytest.mark.parametrize("case", CASES, ids=lambda c: "%dx%dx%d" % c[:3])
def test_closed_form_loop_matches_c_oracle(case, oracle_lib):
    from iterative_cleaner_amd import _native, synth
    nsub, nchan, nbin, seed, rfi, extra = case
    data, w0, shift = synth.make_cube(nsub, nchan, nbin, seed, rfi)
    raw = np.ascontiguousarray(data[:, 0])
    args = dict(max_iter=5, chanthresh=5, subintthresh=5, pulse_region=[0, 0, 1])
    args.update(extra)
    pr = None
    if args["pulse_region"] != [0, 0, 1]:
        _, fac, a, b = _native.normalise_pulse_region(args["pulse_region"], nbin)
        pr = (fac, a, b)
    ref = oracle_lib.clean_loop(raw, w0, shift, args["chanthresh"], args["subintthresh"], args["max_iter"], pr,
                                want_residual=True, want_details=True, fit_mode=1)
    with _native.GpuSession(nsub, nchan, nbin, args["max_iter"], args["chanthresh"], args["subintthresh"],
                            args["pulse_region"], device=0, fit_mode=_native.FIT_CLOSED) as s:
        s.upload(raw, w0, shift)
        out = s.run()
        T = s.template()
        amp, info = s.fit()
        sd, mn, pt, ff = s.diagnostics()
        R = s.residual()
        st = s.run_stats()
    assert st["fit_rounds"] == 0 and st["fit_profile_sweeps"] == 0 and st["fit_tail_sweeps"] == 0
    assert out["loops"] == ref["loops"]
    assert bits_equal(T, ref["T"][out["n_iter"] - 1])
    assert bits_equal(amp, ref["amp"]) and bits_equal(info, ref["info"])
    assert bits_equal(out["weights"], ref["weights"])
    assert np.array_equal(out["changed"], ref["changed"][:out["n_iter"]])
    assert bits_equal(sd, ref["std"]) and bits_equal(mn, ref["mean"]) and bits_equal(pt, ref["ptp"])
    assert _close(ff, ref["fft"], 1e-9)
    assert _close(out["test"], ref["test"], 1e-9)
    assert bits_equal(R, ref["residual"])


def test_closed_form_pols_upload_and_shards(oracle_lib):
    """The fast mode keeps no fit cube: ic_upload_pols then pscrunches through a
    temporary buffer; channel shards (in-process group) reproduce one session."""
    from iterative_cleaner_amd import _native, synth
    nsub, nchan, nbin = 6, 600, 256
    data, w0, shift = synth.make_cube(nsub, nchan, nbin, 77, 0.2, npol=2)
    raw = (data[:, 0] + data[:, 1]).astype(np.float32)
    ref = oracle_lib.clean_loop(raw, w0, shift, fit_mode=1)
    with _native.GpuSession(nsub, nchan, nbin, device=0, fit_mode=_native.FIT_CLOSED) as s:
        s.upload_pols(data, w0, shift)
        out = s.run()
    assert out["loops"] == ref["loops"] and bits_equal(out["weights"], ref["weights"])
    import threading
    world = 2
    chans, _ = _native.shard_layout(nsub, nchan, world)
    results = [None] * world
    with _native.ShardGroup(world) as g:
        sess = [_native.ShardSession(nsub, nchan, nbin, r, world, group=g, device=0, fit_mode=_native.FIT_CLOSED)
                for r in range(world)]
        for r, (c0, c1) in enumerate(chans):
            sess[r].upload(np.ascontiguousarray(raw[:, c0:c1]), np.ascontiguousarray(w0[:, c0:c1]), shift[c0:c1])

        def go(r):
            results[r] = sess[r].run()
        th = [threading.Thread(target=go, args=(r,)) for r in range(world)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for x in sess:
            x.close()
    merged = np.concatenate([results[r]["weights"] for r in range(world)], axis=1)
    assert bits_equal(merged, ref["weights"])
