"""Batch scheduler for many archives of one shape on one GPU (config C4,
SURVEY.md §8(e)/(f) rank 4).

The reference cleans its archive list one after the other, reloading and
re-processing each (iterative_cleaner.py:59-62).  Here one session is reused
for every archive of a shape, and the host->device copy of archive k+1 runs on
the session's copy stream while archive k is cleaned (ic_upload_async, two
device input slots).  Host staging goes through a ring of page-locked buffers
filled by a loader thread, so reading/decoding archive k+2 overlaps too.

A C4 archive (128 x 1024 x 512) is too small to fill an MI355X on its own:
its later fit rounds, the tail and the small reductions leave most CUs idle.
`lanes` > 1 runs that many sessions, each on its own HIP streams and host
thread (ctypes drops the GIL during ic_run), pulling archives from one queue,
so the kernels of different archives overlap on the GPU.  Results come back in
input order.  Under torchrun every rank runs its own batch (dist.shard of the
list): no collective.
"""
from __future__ import annotations

import queue
import sys
import threading
import time

import numpy as np

from . import _native

# how long closing the lanes waits, in all, for the workers' current ic_run calls (seconds)
JOIN_TIMEOUT_S = 600.0

# sessions of lanes that were still inside ic_run when the lanes closed, with
# every host array their queued copies and runs may still read: kept alive
# (never freed, never destroyed) for the life of the process
_LEAKED = []


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


_EXITED = -2   # a worker's last message (run_lanes)


def run_lanes(sessions, items, fetch=True, stop=None, join_timeout=None):
    """Clean every (cube, w0, shift) of `items` on `len(sessions)` sessions of one
    shape concurrently (one host thread per session, shared work queue; each
    session overlaps its next upload with its current run).  The arrays must
    stay valid until their result is yielded.  Yields the ic_run dicts in input
    order.  One session: exactly `pipeline`.

    On a worker error, or when the consumer stops early (generator closed), the
    lanes stop: the `stop` event (created here if not given) is set, queued work
    is dropped, and the generator returns only after every worker thread has
    exited - a worker finishes at most the run it is in, so no thread is inside
    ic_run when the caller closes the sessions.  The workers share one deadline
    (`join_timeout`, default JOIN_TIMEOUT_S): a lane still inside ic_run then is
    leaked, its session marked (`_ic_leaked`, handle dropped so nothing
    destroys it under the running call) and, with the arrays it was handed,
    kept in _LEAKED."""
    if len(sessions) == 1:
        yield from pipeline(sessions[0], items, fetch)
        return
    stop = stop if stop is not None else threading.Event()
    work = queue.Queue(maxsize=2 * len(sessions))
    done = queue.Queue()

    held = [[] for _ in sessions]   # per lane: the arrays of its uploads not yet consumed by a run

    def worker(lane, sess):
        pending = None   # index uploaded to this session, not yet run
        try:
            while not stop.is_set():
                try:
                    item = work.get_nowait()
                except queue.Empty:
                    if pending is not None:   # nothing queued: run what we hold
                        done.put((pending, sess.run(fetch)))
                        pending = None
                        continue
                    item = work.get()
                if item is None or stop.is_set():
                    break
                idx, arrays = item
                held[lane].append(arrays)
                del held[lane][:-3]             # an upload is consumed by the second run after it
                sess.upload_async(*arrays)
                if pending is not None:
                    done.put((pending, sess.run(fetch)))
                pending = idx
            if pending is not None and not stop.is_set():
                done.put((pending, sess.run(fetch)))
        except BaseException as e:  # noqa: BLE001 - re-raised by the consumer
            stop.set()
            done.put((-1, e))
        finally:
            done.put((_EXITED, lane))   # the consumer counts the live workers down without polling

    threads = [threading.Thread(target=worker, args=(q, sess), daemon=True) for q, sess in enumerate(sessions)]
    for th in threads:
        th.start()
    n = 0
    feed_error = []

    def put(item):
        while not stop.is_set():
            try:
                work.put(item, timeout=0.1)
                return True
            except queue.Full:
                continue
        return False

    def feed():
        nonlocal n
        try:
            for arrays in items:
                if not put((n, arrays)):
                    return
                n += 1
        except BaseException as e:  # noqa: BLE001
            feed_error.append(e)
            stop.set()
        finally:
            for _ in threads:
                if not put(None):
                    break

    feeder = threading.Thread(target=feed, daemon=True)
    feeder.start()
    ready, nxt, live = {}, 0, len(threads)
    try:
        while True:
            if nxt in ready:
                yield ready.pop(nxt)
                nxt += 1
                continue
            if live == 0:
                feeder.join()   # past its items (or stopped): it returns within one put timeout
                break
            idx, out = done.get()
            if idx == _EXITED:
                live -= 1
                continue
            if idx < 0:
                raise out
            ready[idx] = out
        if feed_error:
            raise feed_error[0]
        if ready or nxt != n:
            raise RuntimeError("batch lanes lost archives %d..%d" % (nxt, n - 1))
    finally:
        stop.set()
        while True:                       # drop queued work; wake blocked workers
            try:
                work.get_nowait()
            except queue.Empty:
                break
        for _ in threads:
            try:
                work.put_nowait(None)
            except queue.Full:
                break
        limit = JOIN_TIMEOUT_S if join_timeout is None else float(join_timeout)
        deadline = time.monotonic() + limit   # one deadline for every lane
        for q, (th, sess) in enumerate(zip(threads, sessions)):
            th.join(timeout=max(0.0, deadline - time.monotonic()))   # at most the run a worker is in
            if th.is_alive():
                # a worker stuck inside ic_run: leak its session (never destroyed
                # under a running call) and keep what it may still read alive,
                # rather than hang the caller's cleanup
                sys.stderr.write("iterative_cleaner: batch lane %d still inside ic_run after %.0f s; "
                                 "leaking its session\n" % (q, limit))
                _LEAKED.append((sess, getattr(sess, "h", None), list(held[q])))
                if hasattr(sess, "h"):
                    sess.h = None
                sess._ic_leaked = True
        feeder.join(timeout=5.0)          # may wait in `items`: the caller's stop ends that


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


def clean_batch(loader, shape, device=0, ring=None, max_iter=5, chanthresh=5.0, subintthresh=5.0,
                pulse_region=(0, 0, 1), baseline_duty=0.15, lanes=1, join_timeout=None):
    """Clean the archives produced by `loader` (an iterable of (cube, w0, shift)
    host arrays of one (nsub, nchan, nbin) shape; shift is reduced mod nbin).
    A loader thread copies them into a ring of page-locked slots; the GPU
    pipeline overlaps each upload with the previous cleaning, on `lanes`
    concurrent sessions.  Yields one ic_run dict per archive, in order."""
    nsub, nchan, nbin = (int(x) for x in shape)
    lanes = int(lanes)
    if lanes < 1:
        raise ValueError("lanes must be >= 1")
    if ring is None:
        ring = 3 * lanes + 1
    if ring < 3 * lanes:
        raise ValueError("ring must hold >= 3 slots per lane (loading, copying, cleaning)")
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
    sessions = []
    lanes_gen = None
    try:
        for _ in range(lanes):
            sessions.append(_native.GpuSession(nsub, nchan, nbin, max_iter, chanthresh, subintthresh,
                                               pulse_region, baseline_duty, device=device))
        lanes_gen = run_lanes(sessions, staged(), stop=stop, join_timeout=join_timeout)
        for k, out in enumerate(lanes_gen):
            free.put(order[k])          # archive k's slot is free once its result is yielded
            yield out
        if error:
            raise error[0]
    finally:
        stop.set()                      # loader and lanes stop taking archives
        for _ in range(ring):
            free.put(0)                 # a loader waiting for a slot wakes up and returns
        if lanes_gen is not None:
            lanes_gen.close()           # returns once no worker thread is inside ic_run
        th.join(timeout=60)
        for sess in sessions:
            sess.close()
        if any(getattr(sess, "_ic_leaked", False) for sess in sessions):
            _LEAKED.append(rg)          # a leaked lane's copies may still read the page-locked ring
        else:
            rg.close()
