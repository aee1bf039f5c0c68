"""N>1 path on CPU: world_size-2 (and 3) gloo groups run the exact sharding +
single all-reduce that bench.py runs over RCCL, with the oracle standing in
for the per-rank kernel; the result must equal the single-process histogram."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from bsdb_amd.distributed import TILE, global_histogram, shard


def test_shard_cover():
    for n in (0, 1, TILE - 1, TILE, 10 * TILE + 3, 13_193_787_549):
        for world in (1, 2, 3, 8):
            spans = [shard(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c and a <= b
            assert all(lo % TILE == 0 for lo, _ in spans)


def _worker(rank, world, port, n, m, q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import oracle as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard(n, rank, world)

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
    n = 300_001
    m = 5_000
    port = 29500 + world * 7 + os.getpid() % 500
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, n, m, q)) for r in range(world)]
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
