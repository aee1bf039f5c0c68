"""End-to-end (PCIe-inclusive) rate of the host-buffer entry points: keys
start in host memory, counts / signatures end in host memory.

    python tools/e2e_host.py [--n KEYS]
Keys are generated on the device (D2 recipe) and copied to a host buffer
before timing; both a pageable and a pinned host buffer are timed."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bsdb_amd import Context  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2_000_000_000)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    n = args.n
    m = n // 1500 + 1
    ctx = Context(0)
    pinned = torch.empty(13 * n, dtype=torch.uint8, pin_memory=True)
    step = 500_000_000
    for k0 in range(0, n, step):
        k = min(step, n - k0)
        pinned[13 * k0: 13 * (k0 + k)].copy_(ctx.gen_keys13(k0, k)[: 13 * k])
    torch.cuda.synchronize()
    pageable = np.empty(13 * n, np.uint8)
    pageable[:] = pinned.numpy()
    res = {"n": n, "m": m}
    for name, buf in (("pinned", pinned.numpy()), ("pageable", pageable)):
        best = None
        for _ in range(args.reps):
            counts = np.zeros(m, np.uint32)
            t = time.perf_counter()
            ctx.histogram_fixed_host(buf, 13, m, counts_np=counts)
            dt = time.perf_counter() - t
            best = dt if best is None else min(best, dt)
            assert int(counts.sum(dtype=np.uint64)) == n
        res[f"histogram_{name}_keys_per_s"] = n / best
        res[f"histogram_{name}_GBps"] = 13 * n / best / 1e9
        print(json.dumps(res), file=sys.stderr, flush=True)
    hn = min(n, 500_000_000)
    t = time.perf_counter()
    sig = ctx.hash_fixed_host(pinned.numpy()[: 13 * hn], 13)
    dt = time.perf_counter() - t
    res["hash_pinned_in_pageable_out_keys_per_s"] = hn / dt
    del sig
    print(json.dumps(res))


if __name__ == "__main__":
    main()
