"""N>1 path on CPU: world_size-2 (and 3) gloo groups run the exact sharding +
single all-reduce that bench.py runs over RCCL, with the oracle standing in
for the per-rank kernel; the result must equal the single-process histogram."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from bsdb_amd.distributed import TILE, global_histogram, range_windows, shard


def test_shard_cover():
    for n in (0, 1, TILE - 1, TILE, 10 * TILE + 3, 13_193_787_549):
        for world in (1, 2, 3, 8):
            spans = [shard(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c and a <= b
            assert all(lo % TILE == 0 for lo, _ in spans)


def test_bucket_owner_ranges():
    """E4 ownership: rank g owns [g*m/G, (g+1)*m/G) -- the ranges tile [0, m)
    and owner_of_bucket (the kernels' ((b+1)*G-1)/m, gov_kernels.hip owner_of)
    names the rank whose range holds b, also with more ranks than buckets."""
    from bsdb_amd.distributed import bucket_range, owner_of_bucket
    for m in (1, 2, 3, 7, 667, 66_667, 8_795_859):
        for G in (1, 2, 3, 5, 8, 64):
            ranges = [bucket_range(g, m, G) for g in range(G)]
            assert ranges[0][0] == 0 and ranges[-1][1] == m
            assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
            probe = sorted({0, m - 1, m // 2, m // 3, max(0, m - 2)} | {r[0] for r in ranges if r[0] < m})
            for b in probe:
                g = owner_of_bucket(b, m, G)
                lo, hi = ranges[g]
                assert lo <= b < hi, (m, G, b, g)


def _worker(rank, world, port, n, m, q, use_gpu=False):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import oracle as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard(n, rank, world)

    if use_gpu:  # the HIP histogram of this rank's shard (every rank on cuda:0), reduced on the host
        from bsdb_amd import Context
        ctx = Context(0)

        def local(counts):
            keys = ctx.gen_keys13(lo, hi - lo)
            counts += ctx.histogram_fixed(keys, 13, m, n=hi - lo).cpu()
    else:
        def local(counts):
            keys = O.gen_keys13(lo, hi - lo)
            counts += torch.from_numpy(O.histogram_fixed(keys, 13, m).astype(np.int32))

    c = global_histogram(local, torch.zeros(m, dtype=torch.int32))
    E = O.edge_offsets(c.numpy().view(np.uint32))
    q.put((rank, c.numpy().copy(), E))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_sharded_histogram(world):
    _sharded_histogram(world, 300_001, 5_000, use_gpu=False)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_gloo_sharded_histogram_hip_ranks(world):
    """E2/E3 with the product kernels: each rank histograms its shard with
    the HIP path (all ranks on this box's one GPU), ONE all-reduce (gloo on
    the host here; RCCL in bench.py / the C ABI), every rank the same E."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _sharded_histogram(world, 2_000_003, 8_795_859, use_gpu=True)


def _sharded_histogram(world, n, m, use_gpu):
    port = 29500 + world * 7 + os.getpid() % 500 + (60 if use_gpu else 0)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, n, m, q, use_gpu)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    import oracle as O
    ref = O.histogram_fixed(O.gen_keys13(0, n), 13, m)
    refE = O.edge_offsets(ref)
    for _, c, E in res:
        np.testing.assert_array_equal(c.view(np.uint32), ref)
        np.testing.assert_array_equal(E, refE)


# ---- E4: the multi-GPU full build (bucket-range owners, one all-to-all) ----
class OracleBuild:
    """CPU stand-in for bsdb_amd.distributed.DeviceBuild (test infrastructure):
    the oracle's range build, lookups and the index scatter on host tensors."""

    def __init__(self, O):
        self.O = O

    def zeros(self, count):
        return torch.zeros(count, dtype=torch.int64)

    def partition(self, sig, addr, m, world):
        s = sig.numpy().view(np.uint64).reshape(-1, 2)
        b = self.O.buckets(s, m).astype(np.int64)
        own = ((b + 1) * world - 1) // m
        order = np.argsort(own, kind="stable")
        counts = [int((own == g).sum()) for g in range(world)]
        return sig[torch.from_numpy(order)], addr[torch.from_numpy(order)], counts

    def build_window(self, sig, n_global, b_lo, b_hi, e_lo, width, E_win, values_win, values_w0, sig_win, sig_w0):
        """The oracle's range build into full-size arrays (small test sets),
        cut to the windows DeviceBuild fills; the full arrays stay for the
        lookups of index_slice."""
        m = n_global // 1500 + 1
        E = np.zeros(m + 1, np.uint64)
        vals = np.zeros((2 * (1 + ((n_global * 281) >> 8)) + 63) // 64, np.uint64)
        sb = np.zeros((n_global * width + 63) // 64 + 1 if width else 1, np.uint64)
        s = sig.numpy().view(np.uint64)
        assert self.O.gov_build_range(s, n_global, b_lo, b_hi, e_lo, width, E, vals, sb, 2) == 0
        # nothing outside the range's windows was written
        v0, vn, s0, sn = range_windows(n_global, width, e_lo, s.size // 2)
        assert not vals[:v0].any() and not vals[v0 + vn:].any()
        if width:
            assert not sb[:s0].any() and not sb[s0 + sn:].any()
        E_win.numpy().view(np.uint64)[: b_hi - b_lo + 1] = E[b_lo: b_hi + 1]
        values_win.numpy().view(np.uint64)[:vn] = vals[v0: v0 + vn]
        if width:
            sig_win.numpy().view(np.uint64)[:sn] = sb[s0: s0 + sn]
        E[b_hi] = e_lo + s.size // 2  # (the lookups of index_slice need the range's end)
        self._full = (s, n_global, E, vals, width, sb if width else None)

    def index_slice(self, addr, e_lo, n_local):
        s, n_global, E, vals, width, sb = self._full
        r = self.O.lookup_batch(s, n_global, E, vals, width, sb, True)
        assert r.min() >= e_lo and r.max() < e_lo + n_local
        idx = np.zeros(n_local, ">u8")
        idx[r - e_lo] = addr.numpy().view(np.uint64)
        return torch.from_numpy(idx.view(np.int64).copy())


def _e4_worker(rank, world, port, n, width, path, q, use_gpu, pg="gloo"):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import oracle as O
    from bsdb_amd.distributed import DeviceBuild, sharded_full_build, write_index_slice
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if pg == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard(n, rank, world)
    keys = O.gen_keys13(lo, hi - lo)
    addr = torch.arange(lo, hi, dtype=torch.int64) * 48 + 4096
    if use_gpu:
        from bsdb_amd import Context
        ctx = Context(0)
        backend = DeviceBuild(ctx)
        sig = ctx.hash_fixed(torch.from_numpy(keys).cuda(), 13)
        addr = addr.cuda()
    else:
        backend = OracleBuild(O)
        sig = torch.from_numpy(O.hash_fixed(keys, 13).view(np.int64).copy())
    res = sharded_full_build(backend, sig, addr, n, width)
    if rank == 0:
        write_index_slice(path, 0, None, n, create=True)
    dist.barrier()
    write_index_slice(path, res["e_lo"], res["index"], n, create=False)
    dist.barrier()
    out = {k: (v.cpu().numpy().copy() if hasattr(v, "cpu") else v) for k, v in res.items() if k != "index"}
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def run_e4(world, n, width, tmp_path, use_gpu, pg="gloo"):
    path = str(tmp_path / f"index_{world}.db")
    port = 29700 + world * 11 + os.getpid() % 400 + (50 if use_gpu else 0) + (25 if pg == "nccl" else 0)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_e4_worker, args=(r, world, port, n, width, path, q, use_gpu, pg)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    import oracle as O
    sig = O.hash_fixed(O.gen_keys13(0, n), 13)
    rc, E, vals, sb, _ = O.gov_build_mt(sig, width, 4)
    assert rc == 0
    r0 = res[0]
    np.testing.assert_array_equal(r0["E"].view(np.uint64), E)
    np.testing.assert_array_equal(r0["values"].view(np.uint64), vals)
    if width:
        np.testing.assert_array_equal(r0["sigbits"].view(np.uint64)[: sb.size], sb)
    # ranks' slices tile [0, n) in rank order; index.db == the whole-build restatement
    assert sum(res[g]["n_local"] for g in range(world)) == n
    assert [res[g]["e_lo"] for g in range(world)] == list(np.cumsum([0] + [res[g]["n_local"] for g in range(world)])[:-1])
    ranks = O.lookup_batch(sig, n, E, vals, width, sb if width else None, True)
    exp = np.zeros(n, ">u8")
    exp[ranks] = np.arange(n, dtype=np.uint64) * 48 + 4096
    assert open(path, "rb").read() == exp.tobytes()
    # every other rank keeps its windows: E[b_lo..b_hi), its value and checksum
    # words (a boundary word holds only this rank's bits of it)
    for g in range(1, world):
        lo, hi = res[g]["b_lo"], res[g]["b_hi"]
        if lo >= hi:
            continue
        assert res[g]["E_b0"] == lo
        np.testing.assert_array_equal(res[g]["E"].view(np.uint64)[: hi - lo], E[lo:hi])
        v0, vn, s0, sn = range_windows(n, width, res[g]["e_lo"], res[g]["n_local"])
        assert res[g]["values_w0"] == v0
        w = res[g]["values"].view(np.uint64)[:vn]
        np.testing.assert_array_equal(w[1:-1], vals[v0 + 1: v0 + vn - 1])
        assert not (w & ~vals[v0: v0 + vn]).any()
        # bytes this rank moved: its exchange payload plus its windows, O(n / G)
        assert res[g]["bytes_sent"] <= 24 * (n // world + 8192) + 8 * (hi - lo + 1 + vn + sn) + 64


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_multi_gpu_full_build_oracle_standins(world, tmp_path):
    """E4 on CPU: ranks exchange (sig0, sig1, addr) by bucket-range owner with
    one all-to-all, build their ranges, sum-reduce the structure and write
    their index.db slices; equal to the single-process build."""
    run_e4(world, 240_007, 4, tmp_path, use_gpu=False)


def test_gloo_multi_gpu_full_build_more_ranks_than_buckets(tmp_path):
    """world 3 over 2 000 keys (m = 2 buckets): rank 0 owns no bucket, receives
    no keys, skips the range build and still joins every collective."""
    run_e4(3, 2_000, 4, tmp_path, use_gpu=False)


@pytest.mark.gpu
def test_gloo_multi_gpu_full_build_hip_ranks(tmp_path):
    """The same with the HIP kernels per rank (two ranks on this one GPU,
    gloo for the collectives): the rehearsal of the 8-GPU RCCL run."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    run_e4(2, 600_001, 4, tmp_path, use_gpu=True)


@pytest.mark.gpu
def test_nccl_full_build_device_tensors(tmp_path):
    """E4's RCCL code path (device tensors straight into all_to_all_single,
    all_gather and the int64 sum-reduce) on a one-rank NCCL group: RCCL
    refuses two ranks on one GPU, so this is as far as a one-GPU box goes."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    run_e4(1, 400_003, 4, tmp_path, use_gpu=True, pg="nccl")


def test_range_windows_equal_the_abi():
    """distributed.range_windows == bsdb_gov_range_windows (host arithmetic, no
    device), and consecutive ranges' windows tile the structure's words with
    at most one shared word at each boundary."""
    from bsdb_amd.native import range_windows as abi_windows
    for n, width, cuts in [(1_000_000, 4, [0, 1, 333_333, 999_999, 1_000_000]),
                           (13_193_787_549, 4, [0, 1_649_223_443, 6_596_893_774, 13_193_787_549]),
                           (4_000_000_000, 16, [0, 500_000_001, 4_000_000_000]), (2_000, 0, [0, 700, 2_000])]:
        vw = (2 * (1 + ((n * 281) >> 8)) + 63) // 64
        sw = (n * width + 63) // 64
        prev = None
        for a, b in zip(cuts, cuts[1:]):
            w = range_windows(n, width, a, b - a)
            assert w == abi_windows(n, width, a, b - a)
            assert w[0] + w[1] <= vw and w[2] + w[3] <= max(sw, 1)
            if prev is not None:
                assert prev[0] + prev[1] - 1 <= w[0] <= prev[0] + prev[1]
                if width:
                    assert prev[2] + prev[3] - 1 <= w[2] <= prev[2] + prev[3]
            prev = w
