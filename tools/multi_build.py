"""E4 in one process (bsdb_multi_mph_build_index_fixed) against the one-device
F2 call (bsdb_mph_build_index_fixed): host keys -> MPHF fields on the host +
index.db on disk, wall time per call.  On one GPU, G contexts share the card
(the exchange is a copy within it), so this measures the protocol's overhead,
not scaling.

    python tools/multi_build.py [--n KEYS] [--width 4] [--gpus-listed 1,2]"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bsdb_amd import Context  # noqa: E402
from bsdb_amd.native import Multi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--width", type=int, default=4)
    ap.add_argument("--listed", type=str, default="1,2", help="device contexts of the multi build (all on GPU 0)")
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    n, w = args.n, args.width
    ctx = Context(0)
    keys = ctx.gen_keys13(0, n).cpu().numpy()                  # synthetic keys (D2), host memory
    addr = (np.arange(n, dtype=np.uint64) * np.uint64(48))   # synthetic kv.db record addresses
    d = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    res = {"n": n, "width": w}
    best = None
    for _ in range(args.reps):
        t = time.perf_counter()
        m = ctx.mph_build_index_fixed(keys, 13, w, addr, os.path.join(d, "one.db"))
        dt = time.perf_counter() - t
        ref = m.export()
        m.close()
        best = dt if best is None else min(best, dt)
    res["one_device_f2"] = {"s": best, "keys_per_s": n / best}
    ctx.close()
    for G in [int(x) for x in args.listed.split(",")]:
        with Multi(G, [0] * G) as mc:
            best = None
            for _ in range(args.reps):
                t = time.perf_counter()
                got = mc.mph_build_index_fixed(keys, 13, w, addr, os.path.join(d, f"multi{G}.db"))
                dt = time.perf_counter() - t
                best = dt if best is None else min(best, dt)
        same = all(np.array_equal(a, b) for a, b in zip(got, ref))
        same_file = open(os.path.join(d, "one.db"), "rb").read() == open(os.path.join(d, f"multi{G}.db"), "rb").read()
        res[f"multi_{G}_contexts"] = {"s": best, "keys_per_s": n / best, "fields_equal": same, "index_equal": same_file}
        print(json.dumps(res), file=sys.stderr, flush=True)
    for f in os.listdir(d):
        os.remove(os.path.join(d, f))
    os.rmdir(d)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
