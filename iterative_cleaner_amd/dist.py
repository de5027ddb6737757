"""Multi-GPU plumbing for the cleaning path.

C1/C2/C5 are "replicas only" and C4 is a batch of independent archives: one
process per GPU (torchrun), each cleaning its own archives, with no collective
on the data path.  The reference processes its archive list in one loop
(iterative_cleaner.py:59-62); ``shard`` splits that list across ranks.

C3 (one large archive) is channel-sharded: every rank runs a shard session
(_native.ShardSession) whose four per-iteration exchanges go through
``TorchComm`` — the ic_comm_ops transport of the C-ABI bound to
torch.distributed: RCCL over xGMI on the "nccl" backend, host-staged on
"gloo" (CPU tests, several ranks sharing one GPU).  Exchange buffers are torch
tensors owned here (PyTorch provides buffer ownership, streams and the
process group; the loop itself runs in libicgpu.so).
"""
from __future__ import annotations

import os
from typing import Sequence, TypeVar

T = TypeVar("T")


def rank_world() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment (1 process: 0, 1, 0)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad RANK/WORLD_SIZE: %d/%d" % (rank, world))
    return rank, world, local


def channel_sharding() -> bool:
    """True when the CLI should clean each archive as channel shards across the
    torchrun ranks (IC_CHANNEL_SHARDS=1 and WORLD_SIZE > 1).  The process group
    ("nccl": RCCL over xGMI; IC_SHARD_BACKEND=gloo for several ranks on one GPU)
    is created on first use."""
    if os.environ.get("IC_CHANNEL_SHARDS", "0") in ("", "0"):
        return False
    rank, world, local = rank_world()
    if world == 1:
        return False
    import torch
    import torch.distributed as dist
    if not dist.is_initialized():
        backend = os.environ.get("IC_SHARD_BACKEND", "nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=pg_timeout())
        else:
            dist.init_process_group(backend, timeout=pg_timeout())
    return True


def pg_timeout():
    """Process-group timeout of the channel-shard exchanges (IC_PG_TIMEOUT
    seconds, default 300): a peer that stops taking part makes the others'
    collectives fail after this long instead of blocking for ever."""
    import datetime
    return datetime.timedelta(seconds=float(os.environ.get("IC_PG_TIMEOUT", "300")))


def shard(items: Sequence[T], rank: int, world: int) -> list[T]:
    """Round-robin share of ``items`` for ``rank`` (disjoint, covers every item once,
    keeps the reference's processing order within a rank)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world: %d/%d" % (rank, world))
    return list(items[rank::world])


def max_over_ranks(value: float, device=None) -> float:
    """MAX all-reduce of one float (bench timing); identity without a process group."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    if dist.get_backend() == "gloo":
        device = "cpu"
    t = torch.tensor([float(value)], dtype=torch.float64, device=device or "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


class TorchComm:
    """ic_comm_ops over torch.distributed for one shard session.

    Collectives run in stream order on the session's HIP stream (wrapped as a
    torch ExternalStream): the RCCL kernels wait for the shard kernels that
    wrote the send buffers, and the kernels after them wait for the RCCL
    kernels.  On gloo the stream is synchronised and the buffers staged through
    host memory.  A failing collective is recorded in ``error`` and reported to
    the C++ side as a non-zero return code (the session then fails loudly).
    """

    def __init__(self, device, group=None, fail_at=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.device = torch.device(device)
        self.group = group
        self.backend = dist.get_backend(group)
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.bufs = {}
        self.error = None
        self._ops = None
        # fault injection (tests): the fail_at-th collective of this rank raises
        self.fail_at = fail_at
        self.calls = 0
        self.aborted = False
        # per-collective timing (bench.py's per-rank report): HIP events around
        # each collective on the session stream while `timing` is set
        self.timing = False
        self._events = []

    def _count(self):
        self.calls += 1
        if self.fail_at is not None and self.calls == self.fail_at:
            raise RuntimeError("injected transport failure at collective %d (rank %d)" % (self.calls, self.rank))

    def abort(self):
        """Called when this rank's session failed: tear the process group down so
        that peers blocked in a collective with this rank get an error (gloo:
        connection closed at once; RCCL: the communicator is aborted, or the
        peers' collectives fail at the process-group timeout)."""
        if self.aborted:
            return
        self.aborted = True
        dist = self.dist
        try:
            from torch.distributed import distributed_c10d as c10d
            if hasattr(c10d, "_abort_process_group"):
                c10d._abort_process_group(self.group)
                return
        except Exception:  # noqa: BLE001 - fall back to destroying the group
            pass
        try:
            dist.destroy_process_group(self.group)
        except Exception:  # noqa: BLE001
            pass

    # ------------------------------------------------------------ buffers
    def alloc(self, nbytes):
        t = self.torch.empty(max(int(nbytes), 8), dtype=self.torch.uint8, device=self.device)
        self.bufs[t.data_ptr()] = t
        return t

    def view(self, ptr, nbytes):
        """uint8 view of ``nbytes`` at device address ``ptr`` inside a buffer from alloc()."""
        for base_ptr, t in self.bufs.items():
            if base_ptr <= ptr and ptr + nbytes <= base_ptr + t.numel():
                off = ptr - base_ptr
                return t[off:off + nbytes]
        raise RuntimeError("address %#x (+%d) is not an exchange buffer" % (ptr, nbytes))

    # ------------------------------------------------------------ collectives on tensors
    def _stream_ctx(self, stream):
        import contextlib
        if stream and self.device.type == "cuda":
            return self.torch.cuda.stream(self.torch.cuda.ExternalStream(stream, device=self.device))
        return contextlib.nullcontext()

    def _staged(self):
        return self.backend == "gloo" and self.device.type == "cuda"

    def _timed(self, kind, nbytes, fn):
        """Run fn() (inside the stream context); with timing on, bracket it by
        events on the current (session) stream."""
        if not (self.timing and self.device.type == "cuda"):
            return fn()
        cuda = self.torch.cuda
        a, b = cuda.Event(enable_timing=True), cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        self._events.append((kind, int(nbytes), a, b))

    def exchange_report(self):
        """{collective: {"ms", "calls", "bytes"}} of the timed collectives since
        the last report (synchronises on their events)."""
        out = {}
        for kind, nbytes, a, b in self._events:
            b.synchronize()
            r = out.setdefault(kind, {"ms": 0.0, "calls": 0, "bytes": 0})
            r["ms"] += a.elapsed_time(b)
            r["calls"] += 1
            r["bytes"] += nbytes
        self._events = []
        return out

    def allgather(self, send, recv, stream=None):
        dist = self.dist
        self._count()

        def run():
            if self._staged():
                self.torch.cuda.current_stream(self.device).synchronize()
                s_c, r_c = send.cpu(), recv.new_empty(recv.shape, device="cpu")
                dist.all_gather(list(r_c.chunk(self.world)), s_c, group=self.group)
                recv.copy_(r_c)
            elif self.backend == "gloo":
                dist.all_gather(list(recv.chunk(self.world)), send, group=self.group)
            else:
                dist.all_gather_into_tensor(recv, send, group=self.group)
        with self._stream_ctx(stream):
            self._timed("allgather", recv.numel() * recv.element_size(), run)

    def alltoallv(self, send, send_sizes, recv, recv_sizes, stream=None):
        dist = self.dist
        self._count()

        def run():
            if self._staged():
                self.torch.cuda.current_stream(self.device).synchronize()
                s_c, r_c = send.cpu(), recv.new_empty(recv.shape, device="cpu")
                dist.all_to_all_single(r_c, s_c, list(recv_sizes), list(send_sizes), group=self.group)
                recv.copy_(r_c)
            else:
                dist.all_to_all_single(recv, send, list(recv_sizes), list(send_sizes), group=self.group)
        with self._stream_ctx(stream):
            self._timed("alltoallv", sum(send_sizes) * send.element_size(), run)

    def allreduce_sum(self, t, stream=None):
        dist = self.dist
        self._count()

        def run():
            if self._staged():
                self.torch.cuda.current_stream(self.device).synchronize()
                c = t.cpu()
                dist.all_reduce(c, group=self.group)
                t.copy_(c)
            else:
                dist.all_reduce(t, group=self.group)
        with self._stream_ctx(stream):
            self._timed("allreduce", t.numel() * t.element_size(), run)

    # ------------------------------------------------------------ C callbacks
    def ops(self):
        """The CommOps struct handed to ic_session_create_shard (callbacks kept alive here)."""
        from . import _native as nat
        if self._ops is not None:
            return self._ops

        def guard(fn):
            def run(*a):
                try:
                    fn(*a)
                    return 0
                except Exception as e:  # reported through the C++ error path
                    self.error = repr(e)
                    return -1
            return run

        def c_alloc(ctx, nbytes, out):
            out[0] = self.alloc(nbytes).data_ptr()

        def c_release(ctx, ptr):
            self.bufs.pop(ptr, None)

        def c_allgather(ctx, send, recv, nbytes, stream):
            self.allgather(self.view(send, nbytes), self.view(recv, nbytes * self.world), stream)

        def c_alltoallv(ctx, send, sb, recv, rb, stream):
            ss = [int(sb[r]) for r in range(self.world)]
            rs = [int(rb[r]) for r in range(self.world)]
            self.alltoallv(self.view(send, sum(ss)), ss, self.view(recv, sum(rs)), rs, stream)

        def c_allreduce(ctx, buf, n, stream):
            self.allreduce_sum(self.view(buf, 4 * n).view(self.torch.int32), stream)

        self._fns = (nat.ALLOC_FN(guard(c_alloc)), nat.RELEASE_FN(guard(c_release)),
                     nat.ALLGATHER_FN(guard(c_allgather)), nat.ALLTOALLV_FN(guard(c_alltoallv)),
                     nat.ALLREDUCE_FN(guard(c_allreduce)))
        self._ops = nat.CommOps(None, *self._fns)
        return self._ops


def share_rccl_id(group=None) -> bytes:
    """Rank 0's RCCL unique id (_native.rccl_unique_id) on every rank of the
    process group, for ShardSession(rccl_id=...): the one host exchange the
    native RCCL transport needs (torch.distributed object broadcast)."""
    import torch.distributed as dist

    from . import _native
    obj = [_native.rccl_unique_id() if dist.get_rank(group) == 0 else None]
    dist.broadcast_object_list(obj, src=0 if group is None else dist.get_global_rank(group, 0), group=group)
    return obj[0]
