#!/usr/bin/env python3
"""The bench's end-to-end legs alone (BSDB_BUILDER_PROFILE=1 prints their
phases): C4 from host memory through the streaming builder into index.db,
and C2 / C3 from kv.db files.
python tools/e2e_legs.py [--c4] [--kv] [--parts P] [--kv-n N] [--approx]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c4", action="store_true")
    ap.add_argument("--kv", action="store_true")
    ap.add_argument("--n", type=int, default=13_193_787_549)
    ap.add_argument("--reps", type=int, default=1, help="kv leg repetitions in this process")
    ap.add_argument("--parts", type=int, default=8, help="kv.db partitions (0 = 2 x usable CPUs)")
    ap.add_argument("--kv-n", type=int, default=100_000_000)
    ap.add_argument("--approx", action="store_true", help="index.approximate = true (C3)")
    ap.add_argument("--threads", type=int, default=0, help="kv scan threads (0 = the library's default)")
    args = ap.parse_args()
    import bench
    from bsdb_amd import Context
    ctx = Context(0)
    out = {}
    for _ in range(args.reps if args.kv else 0):
        parts = args.parts or 2 * bench.usable_cpus()
        out["e2e_kv_to_disk"] = bench.e2e_kv_to_disk(ctx, args.kv_n, 4, parts, args.approx, args.threads)
        print(json.dumps(out["e2e_kv_to_disk"]), flush=True)
    if args.c4:
        out["e2e_c4_host_passes"] = bench.e2e_c4_host_passes(ctx, args.n, 4)
        print(json.dumps(out["e2e_c4_host_passes"]), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
