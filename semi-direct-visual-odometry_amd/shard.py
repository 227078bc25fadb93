"""Sharding of independent frame pairs over GPUs.

Pairs are self-contained (no shared state, the pose chain is per pair), so a batch of n pairs is cut into
contiguous blocks, pair i -> rank floor(i * world / n), one process per GPU, and no collective touches
the data path.  Results are per pair, so gathering the blocks in rank order reproduces the single-GPU
output bit for bit.
"""


def pair_block(n_pairs, rank, world):
    """(first, count) of the contiguous block of pairs owned by `rank` (pair i -> floor(i * world / n))."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    first = -(-rank * n_pairs // world)          # ceil(rank * n / world)
    last = -(-(rank + 1) * n_pairs // world)
    return first, last - first


def owner(pair, n_pairs, world):
    """Rank owning pair `pair`."""
    return pair * world // n_pairs


def gather_blocks(local, dist=None):
    """Concatenate every rank's per-pair result list in rank order (host-side, results only)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return list(local)
    parts = [None] * dist.get_world_size()
    dist.all_gather_object(parts, list(local))
    return [x for p in parts for x in p]
