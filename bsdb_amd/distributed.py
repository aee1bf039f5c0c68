"""Key sharding across the GPUs of one node, the single histogram exchange,
and the multi-GPU full build.

Histogram stage (E2/E3): the key set is split into contiguous shards by input
order; each rank histograms its shard over all m buckets; ONE all-reduce(sum)
of the m counters over RCCL/xGMI gives every rank the global bucket
occupancy and every rank runs the same exclusive scan, so E[] is identical
everywhere.  On GPUs that collective runs inside the C ABI
(``Context.histogram_finalize``); ``global_histogram`` is the same exchange
through ``torch.distributed`` (the gloo rehearsal on CPU).  The reference has
no counterpart (single JVM, GOV:385-402 accumulates edgeOffsetAndSeed
sequentially).

Full build (E4): bucket b belongs to rank floor(((b+1)*G - 1) / m), i.e. rank g
owns buckets [g*m/G, (g+1)*m/G) -- a contiguous sig0 range, since the bucket
is monotone in sig0 (CBHS:129-138) -- and buckets are independent
(GOV:405-448).  Each rank hashes its key shard, groups (sig0, sig1, addr) by
owner and ONE all-to-all delivers every key to its owner; each rank then
builds its range into zeroed full-size arrays (disjoint fields: the sum of
the ranks' arrays is the whole structure, assembled by one sum-reduce),
looks its own keys up and scatters their record addresses into its slice
[E[b_lo], E[b_hi]) of index.db, which it writes at that offset of the file.
"""
from __future__ import annotations

import os

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


def bucket_range(rank: int, m: int, world: int):
    """Buckets [lo, hi) owned by `rank` in the multi-GPU full build."""
    return rank * m // world, (rank + 1) * m // world


def owner_of_bucket(b: int, m: int, world: int) -> int:
    return ((b + 1) * world - 1) // m


class DeviceBuild:
    """The E4 per-rank steps on one GPU (the HIP product path)."""

    def __init__(self, ctx):
        self.ctx = ctx

    def zeros(self, count: int):
        import torch
        return torch.zeros(count, dtype=torch.int64, device=f"cuda:{self.ctx.device}")

    def partition(self, sig, addr, m: int, world: int):
        return self.ctx.partition_owners(sig, m, world, payload=addr)

    def build_range(self, sig, n_global, b_lo, b_hi, e_lo, width, E, values, sigbits):
        """The range build; the solve also returns every key's rank (F2)."""
        self._rank = self.zeros(sig.shape[0])
        self.ctx.gov_build_range(sig, n_global, b_lo, b_hi, e_lo, width, E, values, sigbits, rank=self._rank)

    def index_slice(self, sig, addr, n_global, E, values, width, sigbits, e_lo, n_local):
        """The big-endian index slots [e_lo, e_lo + n_local) of these records,
        placed by the ranks the solve returned (no lookup pass)."""
        out = self.zeros(n_local)
        self.ctx.index_scatter(self._rank, addr, e_lo, n_local, out)
        return out


def sharded_full_build(backend, sig_local, addr_local, n_global: int, width: int, group=None):
    """One rank's part of the multi-GPU full build (module docstring).

    sig_local: (n, 2) int64 signatures of this rank's key shard, addr_local:
    (n,) int64 record addresses.  Returns a dict: E, values, sigbits (the whole
    structure on rank 0 after the sum-reduce; this rank's fields elsewhere),
    index (this rank's big-endian index.db slots), e_lo, n_local, b_lo, b_hi."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    m = n_global // 1500 + 1
    host_coll = dist.get_backend(group) == "gloo"
    dev = sig_local.device

    def coll(t):  # gloo reduces host tensors, RCCL device tensors
        return t.cpu() if host_coll else t

    sig_g, addr_g, counts = backend.partition(sig_local, addr_local, m, world)
    send_n = coll(torch.tensor(counts, dtype=torch.int64, device=dev))
    recv_n = torch.empty_like(send_n)
    dist.all_to_all_single(recv_n, send_n, group=group)
    recv_counts = [int(x) for x in recv_n.tolist()]
    n_local = sum(recv_counts)
    # the one data exchange: (sig0, sig1, addr) triples to their owners
    payload = coll(torch.cat([sig_g.reshape(-1, 2), addr_g.reshape(-1, 1)], dim=1).reshape(-1).contiguous())
    recv = torch.empty(3 * n_local, dtype=torch.int64, device=payload.device)
    dist.all_to_all_single(recv, payload, [3 * c for c in recv_counts], [3 * c for c in counts], group=group)
    recv = recv.to(dev).reshape(-1, 3)
    sig_r, addr_r = recv[:, :2].contiguous(), recv[:, 2].contiguous()
    # keys before this rank's range: an exclusive prefix of the per-rank totals
    all_n = [torch.zeros(1, dtype=torch.int64, device=payload.device) for _ in range(world)]
    dist.all_gather(all_n, coll(torch.tensor([n_local], dtype=torch.int64, device=dev)), group=group)
    e_lo = sum(int(t.item()) for t in all_n[:rank])
    b_lo, b_hi = bucket_range(rank, m, world)
    E = backend.zeros(m + 1)
    values = backend.zeros(_values_words(n_global))
    sigbits = backend.zeros((n_global * width + 63) // 64 + 1 if width else 1)
    if b_lo < b_hi:
        backend.build_range(sig_r, n_global, b_lo, b_hi, e_lo, width, E, values, sigbits if width else None)
        # this rank's index slice; its lookups need E[b_hi]'s offset, which the
        # next range owns (kept zero for the sum)
        if b_hi < m:
            E[b_hi] = e_lo + n_local
        index = backend.index_slice(sig_r, addr_r, n_global, E, values, width, sigbits if width else None, e_lo,
                                    n_local)
        if b_hi < m:
            E[b_hi] = 0
    else:
        # more ranks than buckets: an empty range receives no keys (the owner
        # map sends none here) but still joins the collectives below
        if n_local:
            raise RuntimeError(f"rank {rank} owns no buckets but received {n_local} keys")
        index = backend.zeros(0)
    # assemble the structure on rank 0: fields are disjoint bits, sum == or.
    # Only rank 0's copy is defined after a reduce, so only rank 0 copies a
    # host-side result back; every other rank keeps its own fields.
    for t in (E, values, sigbits):
        c = coll(t)
        dist.reduce(c, dst=0, op=dist.ReduceOp.SUM, group=group)
        if c is not t and rank == 0:
            t.copy_(c)
    return {"E": E, "values": values, "sigbits": sigbits if width else None, "index": index, "e_lo": e_lo,
            "n_local": n_local, "b_lo": b_lo, "b_hi": b_hi}


def _values_words(n: int) -> int:
    return (2 * (1 + ((n * 281) >> 8)) + 63) // 64  # GOV:357,483-485


def write_index_slice(path: str, e_lo: int, index_be, n_total: int, create: bool):
    """Each rank writes its big-endian slots at byte 8*e_lo of index.db; rank 0
    creates the file at its final size first (create=True, before a barrier)."""
    if create:
        with open(path, "wb") as f:
            f.truncate(8 * n_total)
        return
    data = index_be.cpu().numpy().tobytes() if hasattr(index_be, "cpu") else bytes(index_be)
    fd = os.open(path, os.O_WRONLY)
    try:
        off = 0
        while off < len(data):  # writes of <= 128 MiB (W:166-179)
            off += os.pwrite(fd, data[off: off + (128 << 20)], 8 * e_lo + off)
    finally:
        os.close(fd)
