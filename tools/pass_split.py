"""Pass-1 / pass-2 times of the two-pass histogram at C4 size (HIP events
around each pass, the context's live profile), for the grid knobs read at
context open (BSDB_D13_GRID).  Measurement tool.

    BSDB_D13_GRID=224 python tools/pass_split.py [--n KEYS] [--reps R]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bsdb_amd import Context  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=13_193_787_549)
    ap.add_argument("--reps", type=int, default=4)
    args = ap.parse_args()
    n, m = args.n, args.n // 1500 + 1
    ctx = Context(0)
    keys = ctx.gen_keys13(0, n)
    counts = torch.zeros(m, dtype=torch.int32, device="cuda")
    ctx.histogram_fixed(keys, 13, m, counts=counts, n=n)
    torch.cuda.synchronize()
    ctx.set_profiling(True)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(args.reps):
        counts.zero_()
        ctx.histogram_fixed(keys, 13, m, counts=counts, n=n)
    b.record()
    torch.cuda.synchronize()
    ctx.set_profiling(False)
    p1, p2 = ctx.profile_read(0), ctx.profile_read(1)
    print(json.dumps({"grid": os.environ.get("BSDB_D13_GRID", "all"), "n": n,
                      "ms_per_call": a.elapsed_time(b) / args.reps,
                      "pass1_ms": p1[0] / args.reps, "pass2_ms": p2[0] / args.reps,
                      "sum_ok": int(counts.to(torch.int64).sum().item()) == n}), flush=True)


if __name__ == "__main__":
    main()
