"""Config C5 (var-len 8-64 B Zipf keys) histogram throughput, device-resident.

    python tools/varlen_bench.py [--n KEYS] [--reps R]
Algorithmic bytes/key = mean key length + 8 (u64 offsets)."""
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
    ap.add_argument("--n", type=int, default=500_000_000)
    ap.add_argument("--total", type=int, default=4_000_000_000, help="key-set size that sets m")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--fe", type=int, default=None, help="time only this front end (0 binned, 1 staged, 2 direct)")
    args = ap.parse_args()
    n = args.n
    m = args.total // 1500 + 1
    ctx = Context(0)
    blob, off = ctx.gen_keys_var(0, n)
    torch.cuda.synchronize()
    total_bytes = int(off[-1])
    mean_len = total_bytes / n
    res = {"n": n, "m": m, "mean_len": mean_len, "bytes_per_key": mean_len + 8}
    counts = torch.zeros(m, dtype=torch.int32, device="cuda")
    for fe, name in ((0, "binned"), (1, "staged"), (2, "direct")):
        if args.fe is not None and fe != args.fe:
            continue
        ctx.set_frontend(fe)
        ms = timed(lambda: ctx.histogram_var(blob, off, m, counts=counts), args.reps)
        res[f"{name}_ms"] = ms
        res[f"{name}_Gkeys_per_s"] = n / ms / 1e6
        res[f"{name}_GBps"] = n * (mean_len + 8) / ms / 1e6
        print(json.dumps(res), file=sys.stderr, flush=True)
    ctx.set_frontend(0)
    counts.zero_()
    ctx.histogram_var(blob, off, m, counts=counts)
    if os.environ.get("BSDB_D13_VARIANT", "0") == "0":  # profiling variants give invalid counts
        assert int(counts.sum(dtype=torch.int64)) == n
    print(json.dumps(res))


if __name__ == "__main__":
    main()
