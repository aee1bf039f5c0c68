"""Profiling variants of the single-pass histogram (k_hist13_fused) at one
key count: BSDB_FU_VARIANT / BSDB_FU_LAG are read per context open, so each
variant runs in a fresh context of this process (measurement tool).

    python tools/fused_variants.py --n N --runs "0:4,1:4,2:4,4:4,0:6,0:8" [--stamps]
Prints one JSON line per run: ms (best of reps), and with --stamps the
per-wave phase cycles of variant 8 (wait, write-out, hash, consume, drain +
barrier) summed over every wave, as fractions."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bsdb_amd import Context  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4_000_000_000)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--runs", type=str, default="0:4,1:4,2:4,4:4,8:4")
    ap.add_argument("--two-pass", action="store_true", help="also time mode 1 (the two-pass path) first")
    args = ap.parse_args()
    n, m = args.n, args.n // 1500 + 1
    keys = None
    if args.two_pass:
        ctx = Context(0)
        keys = ctx.gen_keys13(0, n)
        ctx.set_histogram_mode(1)
        counts = torch.zeros(m, dtype=torch.int32, device="cuda")
        times = []
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            counts.zero_()
            a.record()
            ctx.histogram_fixed(keys, 13, m, counts=counts, n=n)
            b.record()
            torch.cuda.synchronize()
            times.append(a.elapsed_time(b))
        print(json.dumps({"mode": "two-pass", "n": n, "ms_best": min(times), "Gkeys": n / min(times) / 1e6}), flush=True)
        ctx.close()
    for run in args.runs.split(","):
        var, lag = (int(x) for x in run.split(":"))
        os.environ["BSDB_FU_VARIANT"] = str(var)
        os.environ["BSDB_FU_LAG"] = str(lag)
        ctx = Context(0)
        if keys is None:
            keys = ctx.gen_keys13(0, n)
        ctx.set_histogram_mode(3)
        counts = torch.zeros(max(m, 256 * 16 * 8), dtype=torch.int32, device="cuda")
        times = []
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            counts.zero_()
            a.record()
            ctx.histogram_fixed(keys, 13, m, counts=counts, n=n)
            b.record()
            torch.cuda.synchronize()
            times.append(a.elapsed_time(b))
        out = {"variant": var, "lag": lag, "n": n, "ms_best": min(times), "Gkeys": n / min(times) / 1e6}
        if var == 0:
            out["sum_ok"] = int(counts[:m].to(torch.int64).sum().item()) == n
        if var == 8:
            st = counts[: 256 * 16 * 8].view(256 * 16, 8).to(torch.int64).cpu()
            tot = st[:, :5].sum(dim=0).tolist()
            allc = sum(tot)
            out["phase_frac"] = dict(zip(["wait", "write_out", "hash", "consume", "drain_barrier"],
                                         [round(t / allc, 4) for t in tot]))
            out["iters_per_wave"] = int(st[:, 5].float().mean().item())
            out["spin_frac"] = round(float(st[:, 6].sum().item()) / allc, 4)
            out["store_drain_frac"] = round(float(st[:, 7].sum().item()) / allc, 4)
            out["wait_max_wg_frac"] = round(float(st[:, 0].max().item()) / (allc / st.shape[0]), 4)
        print(json.dumps(out), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
