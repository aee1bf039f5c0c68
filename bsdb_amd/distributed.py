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
builds its range into WINDOWS of the structure -- E[b_lo..b_hi], the value
words of its vertices, the checksum words of its ranks (range_windows) --
so a rank holds and moves O(n/G) words, places its own keys' record
addresses (the solve returns their ranks) into its slice [E[b_lo], E[b_hi])
of index.db, which it writes at that offset of the file, and sends its
windows to rank 0, which ORs them into the whole structure (a word on a range
boundary holds bits of both neighbours; every other word comes from one rank).
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


def range_windows(n_global: int, width: int, e_lo: int, n_local: int):
    """(values_w0, values_words, sig_w0, sig_words): the value words and the
    checksum words a range build over the keys [e_lo, e_lo + n_local) writes
    -- words [vo(e_lo) >> 5, (vo(e_hi) + 31) >> 5) of the 2-bit values (32 a
    word; vo = vertexOffset, GOV:315-317) and [w e_lo >> 6, (w e_hi + 63) >> 6)
    of the w-bit checksums.  Equals bsdb_gov_range_windows."""
    vo = lambda x: (x * 281) >> 8
    e_hi = e_lo + n_local
    v0 = vo(e_lo) >> 5
    s0 = (e_lo * width) >> 6 if width else 0
    return v0, ((vo(e_hi) + 31) >> 5) - v0, s0, (((e_hi * width) + 63) >> 6) - s0 if width else 0


class DeviceBuild:
    """The E4 per-rank steps on one GPU (the HIP product path)."""

    def __init__(self, ctx):
        self.ctx = ctx

    def zeros(self, count: int):
        import torch
        return torch.zeros(count, dtype=torch.int64, device=f"cuda:{self.ctx.device}")

    def partition(self, sig, addr, m: int, world: int):
        return self.ctx.partition_owners(sig, m, world, payload=addr)

    def build_window(self, sig, n_global, b_lo, b_hi, e_lo, width, E_win, values_win, values_w0, sig_win, sig_w0):
        """The range build into windows; the solve also returns every key's rank (F2)."""
        self._rank = self.zeros(sig.shape[0])
        self.ctx.gov_build_window(sig, n_global, b_lo, b_hi, e_lo, width, E_win, values_win, values_w0, sig_win,
                                  sig_w0, rank=self._rank)

    def index_slice(self, addr, e_lo, n_local):
        """The big-endian index slots [e_lo, e_lo + n_local) of these records,
        placed by the ranks the solve returned (no lookup pass)."""
        out = self.zeros(n_local)
        self.ctx.index_scatter(self._rank, addr, e_lo, n_local, out)
        return out


def sharded_full_build(backend, sig_local, addr_local, n_global: int, width: int, group=None, assemble: bool = True):
    """One rank's part of the multi-GPU full build (module docstring).

    sig_local: (n, 2) int64 signatures of this rank's key shard, addr_local:
    (n,) int64 record addresses (both may be released by the caller after the
    call starts: the exchange keeps its own copies).  Returns a dict: E,
    values, sigbits (rank 0, assemble=True: the whole structure; otherwise
    this rank's windows, at E_b0 = b_lo / values_w0 / sig_w0), index (this
    rank's big-endian index.db slots), e_lo, n_local, b_lo, b_hi, and
    bytes_sent (this rank's exchange + assembly payload)."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    m = n_global // 1500 + 1
    host_coll = dist.get_backend(group) == "gloo"
    dev = sig_local.device

    def coll(t):  # gloo moves host tensors, RCCL device tensors
        return t.cpu() if host_coll else t

    sig_g, addr_g, counts = backend.partition(sig_local, addr_local, m, world)
    send_n = coll(torch.tensor(counts, dtype=torch.int64, device=dev))
    recv_n = torch.empty_like(send_n)
    dist.all_to_all_single(recv_n, send_n, group=group)
    recv_counts = [int(x) for x in recv_n.tolist()]
    n_local = sum(recv_counts)
    # the one data exchange: (sig0, sig1, addr) triples to their owners
    payload = coll(torch.cat([sig_g.reshape(-1, 2), addr_g.reshape(-1, 1)], dim=1).reshape(-1).contiguous())
    del sig_g, addr_g
    recv = torch.empty(3 * n_local, dtype=torch.int64, device=payload.device)
    dist.all_to_all_single(recv, payload, [3 * c for c in recv_counts], [3 * c for c in counts], group=group)
    bytes_sent = 8 * (payload.numel() - 3 * counts[rank])
    del payload
    recv = recv.to(dev).reshape(-1, 3)
    sig_r, addr_r = recv[:, :2].contiguous(), recv[:, 2].contiguous()
    del recv
    # keys before each rank's range: an exclusive prefix of the per-rank totals
    all_n = [torch.zeros(1, dtype=torch.int64, device=send_n.device) for _ in range(world)]
    dist.all_gather(all_n, coll(torch.tensor([n_local], dtype=torch.int64, device=dev)), group=group)
    n_of = [int(t.item()) for t in all_n]
    e_of = [sum(n_of[:g]) for g in range(world)]
    e_lo = e_of[rank]
    b_lo, b_hi = bucket_range(rank, m, world)
    v0, vn, s0, sn = range_windows(n_global, width, e_lo, n_local)
    E_w = backend.zeros(b_hi - b_lo + 1)
    values_w = backend.zeros(max(vn, 1))
    sig_w = backend.zeros(max(sn, 1)) if width else None
    if b_lo < b_hi:
        backend.build_window(sig_r, n_global, b_lo, b_hi, e_lo, width, E_w, values_w, v0, sig_w, s0)
        index = backend.index_slice(addr_r, e_lo, n_local)
    else:
        # more ranks than buckets: an empty range receives no keys (the owner
        # map sends none here) but still joins the collectives below
        if n_local:
            raise RuntimeError(f"rank {rank} owns no buckets but received {n_local} keys")
        index = backend.zeros(0)
    del sig_r, addr_r
    out = {"index": index, "e_lo": e_lo, "n_local": n_local, "b_lo": b_lo, "b_hi": b_hi}
    if not assemble:
        out.update(E=E_w, values=values_w, sigbits=sig_w, E_b0=b_lo, values_w0=v0, sig_w0=s0, bytes_sent=bytes_sent)
        return out
    # assembly on rank 0: every other rank sends its three windows (point to
    # point, O(n/G) words each); rank 0 places them, OR-ing shared words
    wins = [(*bucket_range(g, m, world), *range_windows(n_global, width, e_of[g], n_of[g])) for g in range(world)]
    if rank == 0:
        E = backend.zeros(m + 1)
        values = backend.zeros(_values_words(n_global))
        sigbits = backend.zeros((n_global * width + 63) // 64 + 1) if width else None
        for g in range(world):
            gb_lo, gb_hi, gv0, gvn, gs0, gsn = wins[g]
            if gb_lo >= gb_hi:
                continue
            if g == 0:
                e_g, v_g, s_g = E_w, values_w, sig_w
            else:
                e_g = coll(backend.zeros(gb_hi - gb_lo + 1))
                v_g = coll(backend.zeros(max(gvn, 1)))
                s_g = coll(backend.zeros(max(gsn, 1))) if width else None
                for t in (e_g, v_g) + ((s_g,) if width else ()):
                    dist.recv(t, src=g, group=group)
                e_g, v_g = e_g.to(dev), v_g.to(dev)
                s_g = s_g.to(dev) if width else None
            E[gb_lo:gb_hi] = e_g[: gb_hi - gb_lo]
            if gb_hi == m:
                E[m] = e_g[gb_hi - gb_lo]
            values[gv0: gv0 + gvn].bitwise_or_(v_g[:gvn])
            if width:
                sigbits[gs0: gs0 + gsn].bitwise_or_(s_g[:gsn])
        out.update(E=E, values=values, sigbits=sigbits)
    else:
        if b_lo < b_hi:
            for t in (E_w, values_w) + ((sig_w,) if width else ()):
                dist.send(coll(t), dst=0, group=group)
                bytes_sent += 8 * t.numel()
        out.update(E=E_w, values=values_w, sigbits=sig_w, E_b0=b_lo, values_w0=v0, sig_w0=s0)
    out["bytes_sent"] = bytes_sent
    return out


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
