"""Full device-resident index build (BASELINE configs 2/3): keys in HBM ->
signatures (A3) -> GOV build (A5/A6/A8/A11) -> ranks (A12) -> index scatter
(A13, one pass covering all ranks), each stage timed with HIP events.

    python tools/full_build.py [--n KEYS] [--width 4] [--approx]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bsdb_amd import Context  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--width", type=int, default=4)
    ap.add_argument("--approx", action="store_true")
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    n, w = args.n, args.width
    ctx = Context(0)
    keys = ctx.gen_keys13(0, n)
    sig = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    rank = torch.empty(n, dtype=torch.int64, device="cuda")
    addr = torch.arange(n, dtype=torch.int64, device="cuda") * 48      # synthetic kv.db record addresses
    index = torch.empty(n, dtype=torch.int64, device="cuda")
    v8 = vlen = index_a = None
    if args.approx:
        v8 = torch.arange(n, dtype=torch.int64, device="cuda")
        vlen = torch.full((n,), 32, dtype=torch.uint8, device="cuda")
        index_a = torch.empty(n * 8, dtype=torch.uint8, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
    res = {"n": n, "width": w, "approx": args.approx}
    for rep in range(args.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev[0].record()
        ctx.hash_fixed(keys[: 13 * n], 13, out=sig)
        ev[1].record()
        E, values, sigbits = ctx.gov_build(sig, w)
        ev[2].record()
        ctx.lookup(sig, n, E, values, w, sigbits, check=True, out=rank)
        ev[3].record()
        ctx.index_scatter(rank, addr, 0, n, index, v8, vlen, index_a)
        ev[4].record()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        st = [ev[i].elapsed_time(ev[i + 1]) for i in range(4)]
        res[f"rep{rep}"] = {"hash_ms": st[0], "gov_build_ms": st[1], "lookup_ms": st[2], "scatter_ms": st[3],
                            "total_ms": sum(st), "wall_s": wall, "keys_per_s": n / wall}
        print(json.dumps(res[f"rep{rep}"]), file=sys.stderr, flush=True)
        assert torch.equal(torch.sort(rank).values, torch.arange(n, device="cuda")), "ranks not a bijection"
    print(json.dumps(res))


if __name__ == "__main__":
    main()
