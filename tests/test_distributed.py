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


# ------------------------------------------------------------ channel-shard transport
def _comm_worker(rank, world, port, q):
    import ctypes as C

    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from iterative_cleaner_amd.dist import TorchComm
        comm = TorchComm("cpu")
        ops = comm.ops()
        res = {}
        # all-gather through the C callback (device pointers = exchange buffers)
        send = comm.alloc(24)
        recv = comm.alloc(24 * world)
        send.view(torch.float64)[:] = torch.tensor([rank + 0.5, -rank, 1e300 * rank], dtype=torch.float64)
        assert ops.allgather(None, send.data_ptr(), recv.data_ptr(), 24, None) == 0
        res["gather"] = recv[:24 * world].view(torch.float64).tolist()
        # ragged all-to-all (rank r sends r+d+1 bytes of value 10r+d to rank d)
        sb = [rank + d + 1 for d in range(world)]
        rb = [p + rank + 1 for p in range(world)]
        s2 = comm.alloc(sum(sb))
        r2 = comm.alloc(sum(rb))
        off = 0
        for d in range(world):
            s2[off:off + sb[d]] = 10 * rank + d
            off += sb[d]
        SB = (C.c_size_t * world)(*sb)
        RB = (C.c_size_t * world)(*rb)
        assert ops.alltoallv(None, s2.data_ptr(), SB, r2.data_ptr(), RB, None) == 0
        res["a2a"] = r2[:sum(rb)].tolist()
        # counters all-reduce
        cnt = comm.alloc(16)
        cnt.view(torch.int32)[:] = torch.tensor([rank, 1, 0, 5 * rank], dtype=torch.int32)
        assert ops.allreduce_sum_i32(None, cnt.data_ptr(), 4, None) == 0
        res["sum"] = cnt[:16].view(torch.int32).tolist()
        # a pointer that is not an exchange buffer is an error code, not a crash
        junk = torch.zeros(8, dtype=torch.uint8)
        assert ops.allgather(None, junk.data_ptr(), recv.data_ptr(), 8, None) != 0
        assert comm.error and "not an exchange buffer" in comm.error
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_two_rank_torch_comm_gloo():
    """The ic_comm_ops transport (dist.TorchComm) a channel-sharded session
    calls: all-gather / ragged all-to-all / all-reduce through the ctypes
    callbacks, world size 2 over gloo on CPU."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in range(world):
        r = res[rank]
        assert r["gather"] == [0.5, 0.0, 0.0, 1.5, -1.0, 1e300]
        want = []
        for p in range(world):
            want += [10 * p + rank] * (p + rank + 1)
        assert r["a2a"] == want
        assert r["sum"] == [1, 2, 0, 5]


@pytest.mark.parametrize("nsub,nchan", [(3, 256), (9, 1100), (1024, 8192), (7, 777), (360, 3200)])
def test_cpp_shard_layout_matches_python(nsub, nchan):
    """ic_shard_layout (C++, host-only call) == shards.channel_shards/row_owners."""
    from iterative_cleaner_amd import _native
    from iterative_cleaner_amd.shards import channel_shards, row_owners
    for world in (1, 2, 4, 8, 16):
        try:
            want = (channel_shards(nchan, world), row_owners(nsub, world))
        except ValueError:
            with pytest.raises(_native.NativeError):
                _native.shard_layout(nsub, nchan, world)
            continue
        assert _native.shard_layout(nsub, nchan, world) == want
    with pytest.raises(_native.NativeError):
        _native.shard_layout(nsub, nchan, 3)


def _report_worker(rank, world, port, q):
    import sys

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import bench
        ktimes = {"k_fit_pass": {"ms": 10.0 + rank, "launches": 30}, "k_diag": {"ms": 5.0, "launches": 3},
                  "exchange": {"ms": 99.0, "launches": 7}}
        exch = {"alltoallv": {"ms": 0.5 * (rank + 1), "calls": 6, "bytes": 8_000_000},
                "allgather": {"ms": 0.25, "calls": 6, "bytes": 4_000_000}}
        q.put((rank, bench.per_rank_report(ktimes, exch, rank, world, "cpu", 12.0 + rank)))
    finally:
        dist.destroy_process_group()


def test_bench_per_rank_report_two_ranks():
    """bench.py's multi-GPU line carries every rank's compute time, exchange
    time per collective type and the world size its process group saw."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_report_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1]                      # the same gathered table on every rank
    table = res[0]
    assert [r["rank"] for r in table] == [0, 1]
    for r in table:
        assert r["world_size_seen"] == 2
        # the clean's wall time minus its exchanges; the kernels' summed durations
        # (which overlap when the diagnostics fork) apart
        assert r["wall_ms"] == 12.0 + r["rank"]
        assert r["compute_ms"] == 12.0 + r["rank"] - (0.5 * (r["rank"] + 1) + 0.25)
        assert r["kernel_ms"] == 15.0 + r["rank"]            # kernels only, not the exchange bucket
        assert r["exchange"]["alltoallv"] == {"ms": 0.5 * (r["rank"] + 1), "calls": 6, "MB": 8.0}
        assert r["exchange"]["allgather"]["calls"] == 6
        assert r["exchange"]["allreduce"] == {"ms": 0.0, "calls": 0, "MB": 0.0}
