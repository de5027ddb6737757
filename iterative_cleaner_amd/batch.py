"""Batch scheduler for many archives of one shape on one GPU (config C4,
SURVEY.md §8(e)/(f) rank 4).

The reference cleans its archive list one after the other, reloading and
re-processing each (iterative_cleaner.py:59-62).  Here one session is reused
for every archive of a shape, and the host->device copy of archive k+1 runs on
the session's copy stream while archive k is cleaned (ic_upload_async, two
device input slots).  Host staging goes through a ring of page-locked buffers
filled by a loader thread, so reading/decoding archive k+2 overlaps too.
Under torchrun every rank runs its own batch (dist.shard of the list): no
collective.
"""
from __future__ import annotations

import queue
import threading

import numpy as np

from . import _native


def pipeline(session, items, fetch=True):
    """Clean every (cube, w0, shift) of `items` on `session`, overlapping each
    archive's upload with the previous archive's cleaning.  The arrays must stay
    valid until their result is yielded (page-locked for the copies to overlap).
    Yields the ic_run dicts in order."""
    it = iter(items)
    first = next(it, None)
    if first is None:
        return
    session.upload_async(*first)
    for nxt in it:
        session.upload_async(*nxt)
        yield session.run(fetch)
    yield session.run(fetch)


class _Ring:
    """`n` page-locked (cube, w0, shift) slots."""

    def __init__(self, n, nsub, nchan, nbin):
        self.slots = [(_native.PinnedArray((nsub, nchan, nbin), np.float32),
                       _native.PinnedArray((nsub, nchan), np.float32),
                       _native.PinnedArray((nchan,), np.int32)) for _ in range(n)]

    def arrays(self, i):
        return tuple(p.array for p in self.slots[i])

    def close(self):
        for slot in self.slots:
            for p in slot:
                p.close()


def clean_batch(loader, shape, device=0, ring=3, max_iter=5, chanthresh=5.0, subintthresh=5.0,
                pulse_region=(0, 0, 1), baseline_duty=0.15):
    """Clean the archives produced by `loader` (an iterable of (cube, w0, shift)
    host arrays of one (nsub, nchan, nbin) shape; shift is reduced mod nbin).
    A loader thread copies them into a ring of page-locked slots; the GPU
    pipeline overlaps each upload with the previous cleaning.  Yields one
    ic_run dict per archive, in order."""
    nsub, nchan, nbin = (int(x) for x in shape)
    if ring < 3:
        raise ValueError("ring must hold >= 3 slots (loading, copying, cleaning)")
    free = queue.Queue()
    full = queue.Queue(maxsize=ring)
    stop = threading.Event()
    error = []
    rg = _Ring(ring, nsub, nchan, nbin)
    for i in range(ring):
        free.put(i)

    def load():
        try:
            for cube, w0, shift in loader:
                i = free.get()
                if stop.is_set():
                    return
                c, w, s = rg.arrays(i)
                np.copyto(c, np.asarray(cube, np.float32).reshape(nsub, nchan, nbin))
                np.copyto(w, np.asarray(w0, np.float32).reshape(nsub, nchan))
                np.copyto(s, np.mod(np.asarray(shift), nbin).astype(np.int32).reshape(nchan))
                full.put(i)
        except Exception as e:  # noqa: BLE001 - re-raised in the consumer
            error.append(e)
        finally:
            full.put(None)

    th = threading.Thread(target=load, daemon=True)
    th.start()

    def staged():
        while True:
            i = full.get()
            if i is None:
                return
            order.append(i)
            yield rg.arrays(i)

    order = []
    try:
        with _native.GpuSession(nsub, nchan, nbin, max_iter, chanthresh, subintthresh, pulse_region,
                                baseline_duty, device=device) as sess:
            for k, out in enumerate(pipeline(sess, staged())):
                free.put(order[k])          # archive k's slot is free once its run returned
                yield out
        if error:
            raise error[0]
    finally:
        stop.set()
        for _ in range(ring):
            free.put(0)
        th.join(timeout=60)
        rg.close()
