"""world_size-2 gloo runs of the multi-rank plumbing: the
archive-list sharding of the batch CLI and bench.py's max-over-ranks timing."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, items, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from iterative_cleaner_amd.dist import max_over_ranks, rank_world, shard
        r, w, local = rank_world()
        mine = shard(items, r, w)
        every = [None] * w
        dist.all_gather_object(every, mine)
        elapsed = max_over_ranks(1.0 + r)          # rank r "took" 1+r seconds
        q.put((r, local, every, elapsed))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_items", [0, 1, 5, 8])
def test_two_rank_shard_and_max(n_items):
    items = ["obs%02d.ar" % i for i in range(n_items)]
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, items, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, local, every, elapsed in res:
        assert local == r
        flat = [x for part in every for x in part]
        assert sorted(flat) == sorted(items) and len(flat) == len(items)   # disjoint cover
        assert every[0] == items[0::2] and every[1] == items[1::2]          # reference order kept
        assert elapsed == 2.0                                              # MAX over ranks


def test_single_process_defaults(monkeypatch):
    from iterative_cleaner_amd.dist import max_over_ranks, rank_world, shard
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    assert rank_world() == (0, 1, 0)
    assert shard([1, 2, 3], 0, 1) == [1, 2, 3]
    assert max_over_ranks(3.5) == 3.5
    with pytest.raises(ValueError):
        shard([1], 2, 2)
