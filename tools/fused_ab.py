"""A/B of the headline histogram: two-pass (mode 1) vs single pass (mode 3,
k_hist13_fused) on the same device-resident 13-byte keys (measurement tool,
not product code).

    python tools/fused_ab.py [--n KEYS] [--reps R]
Checks the two count arrays are identical, then times each mode (HIP events,
best and median of R calls) and prints one JSON line."""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bsdb_amd import Context  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=13_193_787_549)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--modes", type=str, default="1,3")
    args = ap.parse_args()
    n = args.n
    m = n // 1500 + 1
    ctx = Context(0)
    keys = ctx.gen_keys13(0, n)
    res = {"n": n, "m": m}
    ref = None
    for mode in [int(x) for x in args.modes.split(",")]:
        ctx.set_histogram_mode(mode)
        counts = torch.zeros(m, dtype=torch.int32, device="cuda")
        ctx.histogram_fixed(keys, 13, m, counts=counts, n=n)
        torch.cuda.synchronize()
        total = int(counts.to(torch.int64).sum().item())
        if ref is None:
            ref = counts.clone()
            same = True
        else:
            same = bool(torch.equal(ref, counts))
        times = []
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            counts.zero_()
            a.record()
            ctx.histogram_fixed(keys, 13, m, counts=counts, n=n)
            b.record()
            torch.cuda.synchronize()
            times.append(a.elapsed_time(b))
        same_again = bool(torch.equal(ref, counts))
        res[f"mode{mode}"] = {"sum_ok": total == n, "equal_to_first": same and same_again,
                              "ms_best": min(times), "ms_median": statistics.median(times),
                              "Gkeys_best": n / min(times) / 1e6, "fallbacks": ctx.fallback_count()}
        del counts
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
