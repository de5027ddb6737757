"""Channel-block sharding of one archive across ranks.

Rank r of a power-of-two ``world`` owns the channels of one node at depth
log2(world) of the canonical super-block tree (archive.sb_tree): the node is
reached from the root [0, nsb) by the bits of r, most significant first (0 =
left half [lo, mid), 1 = right half [mid, hi), mid = lo + (hi - lo) // 2).  Its
channel range is [lo * 256, min(hi * 256, nchan)).  Every template channel sum
of a shard is then one subtree of the single-device sum, and the top log2(world)
levels of the tree combine the shard roots in rank order, so a sharded run is
bit-identical to a single-device one.  The same rule is implemented in C++
(ic_session.hip, shard_channels); tests check they agree.

Subint rows (for the row medians of subint_scaler, iterative_cleaner.py:244-256)
are owned in balanced contiguous blocks: rank r owns rows
[r * nsub // world, (r + 1) * nsub // world).
"""
from __future__ import annotations

SUPER_BLOCK = 256


def _check_world(world: int) -> int:
    if world < 1 or world & (world - 1):
        raise ValueError("channel sharding needs a power-of-two world size, got %d" % world)
    return world.bit_length() - 1


def channel_shards(nchan: int, world: int) -> list[tuple[int, int]]:
    """[(c0, c1)] channel range of every rank (contiguous, in rank order)."""
    depth = _check_world(world)
    nsb = (nchan + SUPER_BLOCK - 1) // SUPER_BLOCK
    if nsb < world:
        raise ValueError("%d channels (%d super-blocks of %d) cannot be split over %d shards"
                         % (nchan, nsb, SUPER_BLOCK, world))
    out = []
    for r in range(world):
        lo, hi = 0, nsb
        for d in range(depth - 1, -1, -1):
            mid = lo + (hi - lo) // 2
            if (r >> d) & 1:
                lo = mid
            else:
                hi = mid
        out.append((lo * SUPER_BLOCK, min(hi * SUPER_BLOCK, nchan)))
    return out


def row_owners(nsub: int, world: int) -> list[tuple[int, int]]:
    """[(s0, s1)] subint rows whose medians rank r computes."""
    return [(r * nsub // world, (r + 1) * nsub // world) for r in range(world)]
