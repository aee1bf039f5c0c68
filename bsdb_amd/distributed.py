"""Key sharding across GPUs of one node and the single histogram exchange.

SURVEY.md §8(e): the key set is split into contiguous shards by input order
(E2); each rank histograms its shard over all m buckets; ONE all-reduce(sum)
of the m counters over RCCL/xGMI (E3) gives every rank the global bucket
occupancy, and every rank then runs the same exclusive scan, so E[] is
identical everywhere.  The reference has no counterpart (single JVM,
GOV:385-402 accumulates edgeOffsetAndSeed sequentially).
"""
from __future__ import annotations

TILE = 8192  # pass-1 tile: shard boundaries stay tile aligned


def shard(n: int, rank: int, world: int):
    """[lo, hi) of rank `rank`: contiguous, tile aligned, covering [0, n)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    tiles = (n + TILE - 1) // TILE
    lo = min(n, tiles * rank // world * TILE)
    hi = min(n, tiles * (rank + 1) // world * TILE)
    return lo, hi


def global_histogram(local_hist, counts, group=None):
    """local_hist(counts) accumulates this rank's shard into `counts` (a torch
    tensor); the one collective sums it over the group.  Returns counts."""
    import torch.distributed as dist
    counts.zero_()
    local_hist(counts)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(counts, op=dist.ReduceOp.SUM, group=group)
    return counts
