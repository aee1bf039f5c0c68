"""Kernel-variant microbenchmark (device-resident keys, HIP-event timing).

    python tools/kbench.py [--n KEYS] [--reps R]
Times: signature kernel (hash only, 16 B/key written), histogram via direct
atomics, histogram via the partitioned two-pass path (pass 1 / pass 2 split
from the context's live event profile), for 13-byte keys."""
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
    ap.add_argument("--n", type=int, default=1_000_000_000)
    ap.add_argument("--m", type=int, default=0, help="buckets (default n/1500+1)")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--chunks", type=str, default="0")
    ap.add_argument("--frontends", type=str, default="0")
    args = ap.parse_args()
    n = args.n
    m = args.m or n // 1500 + 1
    ctx = Context(0)
    keys = ctx.gen_keys13(0, n)
    counts = torch.zeros(m, dtype=torch.int32, device="cuda")
    res = {"n": n, "m": m}
    sig_n = min(n, 2_000_000_000)
    sig = torch.empty((sig_n, 2), dtype=torch.int64, device="cuda")
    for fe in [int(f) for f in args.frontends.split(",")]:
        ctx.set_frontend(fe)
        ms = timed(lambda: ctx.hash_fixed(keys[: 13 * sig_n], 13, out=sig), args.reps)
        res[f"hash_sig_fe{fe}_Gkeys"] = sig_n / ms / 1e6
    ctx.set_frontend(0)
    del sig
    ctx.set_histogram_mode(2)
    ms = timed(lambda: ctx.histogram_fixed(keys, 13, m, counts=counts, n=n), args.reps)
    res["atomic_ms"] = ms
    res["atomic_Gkeys"] = n / ms / 1e6
    ctx.set_histogram_mode(0)
    for fe, ch in [(int(f), int(x)) for f in args.frontends.split(",") for x in args.chunks.split(",")]:
        ctx.set_chunk_keys(ch)
        ctx.set_frontend(fe)
        ms = timed(lambda: ctx.histogram_fixed(keys, 13, m, counts=counts, n=n), 1)
        ctx.set_profiling(True)
        ms = timed(lambda: ctx.histogram_fixed(keys, 13, m, counts=counts, n=n), args.reps)
        ctx.set_profiling(False)
        p1 = ctx.profile_read(0)
        p2 = ctx.profile_read(1)
        res[f"part_fe{fe}_chunk{ch}"] = {"ms": ms, "Gkeys": n / ms / 1e6,
                                  "pass1_ms": p1[0] / (args.reps + 1), "pass2_ms": p2[0] / (args.reps + 1),
                                  "launches_per_call": p1[1] / (args.reps + 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
