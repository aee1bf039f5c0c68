"""Histogram throughput of fixed-length keys of several lengths, device-resident
(random bytes), default front end vs the one-tile-per-workgroup kernels.
    python tools/fixed_len_bench.py [--n KEYS] [--lens 8,16,20,32]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bsdb_amd import Context  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=400_000_000)
    ap.add_argument("--lens", type=str, default="8,12,16,20,32")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    ctx = Context(0)
    out = {}
    for L in (int(x) for x in args.lens.split(",")):
        n = args.n
        m = n // 1500 + 1
        keys = torch.randint(0, 256, (n * L + 16,), dtype=torch.uint8, device="cuda")
        counts = torch.zeros(m, dtype=torch.int32, device="cuda")
        row = {}
        for fe, name in ((0, "default"), (1, "staged")):
            ctx.set_frontend(fe)
            ms = timed(lambda: ctx.histogram_fixed(keys, L, m, counts=counts, n=n), args.reps)
            row[name + "_Gkeys_per_s"] = n / ms / 1e6
        ctx.set_frontend(0)
        out[L] = row
        print(json.dumps({L: row}), file=sys.stderr, flush=True)
        del keys
    print(json.dumps(out))


if __name__ == "__main__":
    main()
