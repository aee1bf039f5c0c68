"""A/B of the two-pass histogram with pass 2 of chunk i beside pass 1 of
chunk i + 1 (BSDB_PIPE=1) against the serial chunk loop, on the same
device-resident 13-byte keys (measurement tool).  Knobs are read at context
open, so each configuration gets a fresh context.

    python tools/pipe_ab.py [--n KEYS] [--reps R] [--configs "0,1:8:32,1:16:32"]
A config is PIPE[:CHUNKS[:P2CUS]].  Prints one JSON line per config: ms
(best / median of R calls, HIP events), whether the counts equal the first
config's."""
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
    ap.add_argument("--configs", type=str, default="0,1:8:32,0,1:8:32")
    args = ap.parse_args()
    n, m = args.n, args.n // 1500 + 1
    keys, ref = None, None
    for cfg in args.configs.split(","):
        parts = cfg.split(":")
        os.environ["BSDB_PIPE"] = parts[0]
        os.environ["BSDB_PIPE_CHUNKS"] = parts[1] if len(parts) > 1 else "0"
        os.environ["BSDB_PIPE_P2CUS"] = parts[2] if len(parts) > 2 else "0"
        ctx = Context(0)
        if keys is None:
            keys = ctx.gen_keys13(0, n)
        counts = torch.zeros(m, dtype=torch.int32, device="cuda")
        ctx.histogram_fixed(keys, 13, m, counts=counts, n=n)
        torch.cuda.synchronize()
        if ref is None:
            ref = counts.clone()
        equal = bool(torch.equal(ref, counts))
        times = []
        ctx.set_profiling(True)
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            counts.zero_()
            a.record()
            ctx.histogram_fixed(keys, 13, m, counts=counts, n=n)
            b.record()
            torch.cuda.synchronize()
            times.append(a.elapsed_time(b))
        ctx.set_profiling(False)
        p1, p2 = ctx.profile_read(0), ctx.profile_read(1)
        equal = equal and bool(torch.equal(ref, counts))
        print(json.dumps({"config": cfg, "n": n, "ms_best": min(times), "ms_median": statistics.median(times),
                          "Gkeys_best": n / min(times) / 1e6, "equal": equal,
                          "sum_ok": int(counts.to(torch.int64).sum().item()) == n,
                          "pass1_ms_per_call": p1[0] / args.reps, "pass1_launches_per_call": p1[1] / args.reps,
                          "pass2_ms_per_call": p2[0] / args.reps, "fallbacks": ctx.fallback_count()}), flush=True)
        del counts
        ctx.close()


if __name__ == "__main__":
    main()
