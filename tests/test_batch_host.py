"""Host logic of the batch scheduler's concurrent lanes (batch.run_lanes), on
stand-in sessions: results in input order, every archive exactly once, the
upload-before-run discipline per session, and errors re-raised."""
import random
import threading
import time

import pytest


class FakeSession:
    """Records the ic_upload_async / ic_run protocol of one session."""

    def __init__(self, fail_on=None):
        self.queue = []        # uploaded, not yet run (FIFO, at most 2 deep)
        self.ran = []
        self.fail_on = fail_on
        self.lock = threading.Lock()

    def upload_async(self, tag, *_):
        with self.lock:
            assert len(self.queue) < 2, "more than two uploads in flight"
            self.queue.append(tag)

    def run(self, fetch=True):
        with self.lock:
            tag = self.queue.pop(0)
        time.sleep(random.random() * 0.003)
        if tag == self.fail_on:
            raise RuntimeError("boom %d" % tag)
        self.ran.append(tag)
        return {"tag": tag}


@pytest.mark.parametrize("lanes", [1, 2, 3, 5])
def test_run_lanes_order_and_coverage(lanes):
    from iterative_cleaner_amd import batch
    random.seed(lanes)
    sessions = [FakeSession() for _ in range(lanes)]
    items = [(k, None, None) for k in range(23)]
    got = [out["tag"] for out in batch.run_lanes(sessions, items)]
    assert got == list(range(23))
    assert sorted(t for s in sessions for t in s.ran) == list(range(23))
    assert all(not s.queue for s in sessions)
    if lanes > 1:
        assert sum(1 for s in sessions if s.ran) > 1   # the work was actually shared


def test_run_lanes_returns_when_the_last_lane_exits():
    """The consumer learns of each worker's exit from the worker itself: a
    call returns as soon as its last archive is done (round 3's consumer
    polled the workers every 0.5 s, a half-second stall per call that made
    several lanes look 7x slower than one)."""
    from iterative_cleaner_amd import batch
    random.seed(3)
    for lanes in (2, 4):
        sessions = [FakeSession() for _ in range(lanes)]
        t0 = time.perf_counter()
        for _ in range(5):
            got = [out["tag"] for out in batch.run_lanes(sessions, [(k, None, None) for k in range(8)])]
            assert got == list(range(8))
        assert time.perf_counter() - t0 < 1.0


def test_run_lanes_empty_and_error():
    from iterative_cleaner_amd import batch
    assert list(batch.run_lanes([FakeSession(), FakeSession()], [])) == []
    sessions = [FakeSession(fail_on=7), FakeSession(fail_on=7)]
    with pytest.raises(RuntimeError, match="boom 7"):
        list(batch.run_lanes(sessions, [(k, None, None) for k in range(12)]))


class SlowSession(FakeSession):
    """Counts runs in flight (a run must never be in flight after the lanes end)."""

    inflight = 0
    guard = threading.Lock()

    def run(self, fetch=True):
        with SlowSession.guard:
            SlowSession.inflight += 1
        try:
            time.sleep(0.02)
            return super().run(fetch)
        finally:
            with SlowSession.guard:
                SlowSession.inflight -= 1


def test_run_lanes_early_close_joins_workers():
    """The consumer stops after 3 results: closing the generator returns only
    once every worker has left ic_run, and nothing runs afterwards."""
    from iterative_cleaner_amd import batch
    sessions = [SlowSession() for _ in range(3)]
    items = [(k, None, None) for k in range(200)]
    gen = batch.run_lanes(sessions, items)
    got = [next(gen)["tag"] for _ in range(3)]
    t0 = time.time()
    gen.close()
    assert time.time() - t0 < 5.0
    assert SlowSession.inflight == 0
    ran = sum(len(s.ran) for s in sessions)
    time.sleep(0.1)
    assert sum(len(s.ran) for s in sessions) == ran < 200
    assert got == [0, 1, 2]


def test_run_lanes_error_stops_the_other_lanes():
    from iterative_cleaner_amd import batch
    sessions = [SlowSession(fail_on=5), SlowSession(fail_on=5), SlowSession(fail_on=5)]
    items = [(k, None, None) for k in range(300)]
    t0 = time.time()
    with pytest.raises(RuntimeError, match="boom 5"):
        for _ in batch.run_lanes(sessions, items):
            pass
    assert time.time() - t0 < 5.0
    assert SlowSession.inflight == 0
    assert sum(len(s.ran) for s in sessions) < 300



class StuckSession(FakeSession):
    """A run that never returns until released (a hung kernel), except for tag 0."""

    release = threading.Event()

    def __init__(self):
        super().__init__()
        self.h = object()   # stands in for the native handle

    def run(self, fetch=True):
        with self.lock:
            tag = self.queue[0]
        if tag != 0:
            StuckSession.release.wait()
        return super().run(fetch)


def test_run_lanes_stuck_lanes_share_one_deadline():
    """The consumer stops after the first result while the lanes are stuck
    inside ic_run: closing waits once for the shared deadline (not once per
    lane), leaks every stuck session with the arrays it was handed, and drops
    its handle so that nothing destroys it under the running call."""
    from iterative_cleaner_amd import batch
    StuckSession.release.clear()
    sessions = [StuckSession() for _ in range(3)]
    items = [(k, "array-%d" % k, None) for k in range(9)]
    n0 = len(batch._LEAKED)
    gen = batch.run_lanes(sessions, items, join_timeout=0.6)
    assert next(gen)["tag"] == 0
    t0 = time.time()
    gen.close()
    dt = time.time() - t0
    try:
        assert 0.5 < dt < 1.5, dt          # one shared 0.6-s deadline for three stuck lanes
        leaked = batch._LEAKED[n0:]
        # the lanes stuck in a run (the one that ran tag 0 may have stopped at
        # the close instead of entering its next run)
        assert 2 <= len(leaked) <= 3
        for sess, handle, arrays in leaked:
            assert sess._ic_leaked and sess.h is None and handle is not None
            assert arrays and all(a[1].startswith("array-") for a in arrays)
    finally:
        StuckSession.release.set()
