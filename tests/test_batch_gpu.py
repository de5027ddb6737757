"""GPU tests of the batch scheduler (config C4): archives cleaned through the
double-buffered asynchronous uploads (ic_upload_async) and the page-locked
staging ring must give exactly the results of one synchronous session per
archive, in order; misuse of the upload queue fails loudly."""
import numpy as np
import pytest

from helpers import bits_equal, bits_equal_nan

pytestmark = pytest.mark.gpu

SHAPE = (6, 96, 128)


def _archives(n):
    from iterative_cleaner_amd import synth
    out = []
    for k in range(n):
        data, w0, shift = synth.make_cube(*SHAPE, seed=200 + k, rfi_frac=0.1 + 0.05 * (k % 3))
        out.append((np.ascontiguousarray(data[:, 0]), w0, shift))
    return out


def _one(cube, w0, shift):
    from iterative_cleaner_amd import _native
    with _native.GpuSession(*SHAPE, device=0) as s:
        s.upload(cube, w0, shift)
        return s.run()


def test_clean_batch_matches_single_sessions():
    from iterative_cleaner_amd import batch
    arcs = _archives(7)
    got = list(batch.clean_batch(iter(arcs), SHAPE, device=0))
    assert len(got) == len(arcs)
    for (cube, w0, shift), out in zip(arcs, got):
        ref = _one(cube, w0, shift)
        assert out["loops"] == ref["loops"] and np.array_equal(out["changed"], ref["changed"])
        assert bits_equal(out["weights"], ref["weights"]) and bits_equal(out["test"], ref["test"])


@pytest.mark.parametrize("lanes", [2, 3])
def test_clean_batch_concurrent_lanes_match_single_sessions(lanes):
    """Several sessions cleaning concurrently on their own streams: same bits,
    results in input order."""
    from iterative_cleaner_amd import batch
    arcs = _archives(8)
    got = list(batch.clean_batch(iter(arcs), SHAPE, device=0, lanes=lanes))
    assert len(got) == len(arcs)
    for (cube, w0, shift), out in zip(arcs, got):
        ref = _one(cube, w0, shift)
        assert out["loops"] == ref["loops"] and np.array_equal(out["changed"], ref["changed"])
        assert bits_equal(out["weights"], ref["weights"]) and bits_equal(out["test"], ref["test"])


@pytest.mark.parametrize("lanes", [1, 2])
def test_clean_batch_non_finite_archive_leaves_no_trace(lanes):
    """An archive with NaN / Inf samples (every test value NaN, nothing zapped)
    between ordinary ones: the sessions the batch reuses carry nothing of it
    into the next archive, and it gives one session's results itself."""
    from iterative_cleaner_amd import batch
    arcs = _archives(5)
    bad = arcs[2][0].copy()
    bad[1, 7, 10] = np.nan
    bad[3, 40, 100] = np.inf
    arcs[2] = (bad, arcs[2][1], arcs[2][2])
    got = list(batch.clean_batch(iter(arcs), SHAPE, device=0, lanes=lanes))
    assert len(got) == len(arcs)
    for k, ((cube, w0, shift), out) in enumerate(zip(arcs, got)):
        ref = _one(cube, w0, shift)
        assert out["loops"] == ref["loops"] and np.array_equal(out["changed"], ref["changed"]), k
        assert bits_equal(out["weights"], ref["weights"]) and bits_equal_nan(out["test"], ref["test"]), k
    assert np.isnan(got[2]["test"]).any()


def test_pipeline_on_pinned_arrays_and_queue_rules():
    from iterative_cleaner_amd import _native, batch
    arcs = _archives(3)
    pinned = []
    for cube, w0, shift in arcs:
        trio = (_native.PinnedArray(cube.shape), _native.PinnedArray(w0.shape),
                _native.PinnedArray(shift.shape, np.int32))
        trio[0].array[:] = cube
        trio[1].array[:] = w0
        trio[2].array[:] = shift
        pinned.append(trio)
    items = [tuple(p.array for p in trio) for trio in pinned]
    with _native.GpuSession(*SHAPE, device=0) as s:
        # the same archive twice in a row, then the others: the slots rotate correctly
        outs = list(batch.pipeline(s, [items[0], items[0], items[1], items[2], items[1]]))
        refs = [_one(*arcs[i]) for i in (0, 0, 1, 2, 1)]
        for out, ref in zip(outs, refs):
            assert bits_equal(out["weights"], ref["weights"]) and out["loops"] == ref["loops"]
        # at most two pending uploads; synchronous uploads refuse while any is pending
        s.upload_async(*items[0])
        s.upload_async(*items[1])
        with pytest.raises(_native.NativeError):
            s.upload_async(*items[2])
        with pytest.raises(_native.NativeError):
            s.upload(*arcs[2])
        a = s.run()
        b = s.run()
        assert bits_equal(a["weights"], refs[0]["weights"]) and bits_equal(b["weights"], refs[2]["weights"])
        # queue drained: a synchronous upload works again, and a re-run repeats the last archive
        s.upload(*arcs[2])
        assert bits_equal(s.run()["weights"], refs[3]["weights"])
        assert bits_equal(s.run()["weights"], refs[3]["weights"])
    for trio in pinned:
        for p in trio:
            p.close()


@pytest.mark.parametrize("npol", [1, 2, 4])
def test_device_pscrunch_matches_host_pscrunch(npol):
    """ic_upload_pols: the GPU's f32(pol0 + pol1) gives exactly the loop of the
    host-pscrunched cube (archive.py pscrunch), including a second run after
    the fit-cube buffer served as scratch."""
    from iterative_cleaner_amd import _native, synth
    data, w0, shift = synth.make_cube(5, 72, 256, seed=77, rfi_frac=0.2, npol=npol)
    host = data[:, 0] if npol == 1 else (data[:, 0] + data[:, 1]).astype(np.float32)
    with _native.GpuSession(5, 72, 256, device=0) as s:
        s.upload(np.ascontiguousarray(host), w0, shift)
        ref = s.run()
        amp_ref, _ = s.fit()
        R_ref = s.residual()
    with _native.GpuSession(5, 72, 256, device=0) as s:
        for _ in range(2):
            s.upload_pols(data, w0, shift)
            out = s.run()
            amp, _ = s.fit()
            assert bits_equal(out["weights"], ref["weights"]) and bits_equal(out["test"], ref["test"])
            assert bits_equal(amp, amp_ref) and bits_equal(s.residual(), R_ref)
