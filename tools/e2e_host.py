"""End-to-end (PCIe-inclusive) rate of the host-buffer entry points: keys
start in host memory, counts / signatures end in host memory.

    python tools/e2e_host.py [--n KEYS]
    python tools/e2e_host.py --full KEYS [--approx] [--dir D] [--ps BYTES | --fused]
Keys are generated on the device (D2 recipe) and copied to a host buffer
before timing; both a pageable and a pinned host buffer are timed.

--full: "keys in host memory -> hash.dump + index.db on disk" through the
host ABI only (bsdb_mph_build_fixed, bsdb_mph_dump, bsdb_index_* with the
reference's pass loop at -ps 1024 MiB, or --ps 0: device-sized passes); times the MPHF build, the dump and
the index write separately."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bsdb_amd import Context  # noqa: E402


def full(ctx, n, approx, d, ps, fused=False):
    keys = np.empty(13 * n, np.uint8)
    step = 500_000_000
    for k0 in range(0, n, step):
        k = min(step, n - k0)
        keys[13 * k0: 13 * (k0 + k)] = ctx.gen_keys13(k0, k)[: 13 * k].cpu().numpy()
    i = np.arange(n, dtype=np.uint64)
    addr = np.uint64(0x1000) + np.uint64(48) * i
    value8 = i * np.uint64(0x9E3779B97F4A7C15) if approx else None
    vlen = np.full(n, 8, np.uint8) if approx else None
    os.makedirs(d, exist_ok=True)
    ip, ap_, hp = (os.path.join(d, f) for f in ("index.db", "index_a.db", "hash.dump"))
    if fused:  # F2: one call, index from the solve's ranks
        t0 = time.perf_counter()
        mph = ctx.mph_build_index_fixed(keys, 13, 4, addr, ip, ap_, approx, value8, vlen)
        t1 = time.perf_counter()
        mph.dump(hp)
        t2 = time.perf_counter()
        res = {"n": n, "approximate": approx, "fused_index": True, "mph_build_and_index_s": t1 - t0,
               "dump_s": t2 - t1, "total_s": t2 - t0, "keys_per_s": n / (t2 - t0),
               "index_db_bytes": os.path.getsize(ip), "index_a_db_bytes": os.path.getsize(ap_)}
        mph.close()
        for f in (ip, ap_, hp):
            os.remove(f)
        print(json.dumps(res), flush=True)
        return
    t0 = time.perf_counter()
    mph = ctx.mph_build_fixed(keys, 13, 4)
    t1 = time.perf_counter()
    mph.dump(hp)
    t2 = time.perf_counter()
    B = 50_000_000

    def feed(w):
        for lo in range(0, n, B):
            hi = min(n, lo + B)
            w.put_fixed(keys[13 * lo: 13 * hi], 13, addr[lo:hi], value8[lo:hi] if approx else None,
                        vlen[lo:hi] if approx else None)
    passes = mph.write_index(ip, ap_, approx, ps, feed)
    t3 = time.perf_counter()
    res = {"n": n, "approximate": approx, "pass_cache_bytes": ps, "passes": passes, "mph_build_s": t1 - t0, "dump_s": t2 - t1,
           "index_s": t3 - t2, "total_s": t3 - t0, "keys_per_s": n / (t3 - t0),
           "index_db_bytes": os.path.getsize(ip), "index_a_db_bytes": os.path.getsize(ap_)}
    mph.close()
    for f in (ip, ap_, hp):
        os.remove(f)
    print(json.dumps(res), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2_000_000_000)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--full", type=int, default=0)
    ap.add_argument("--approx", action="store_true")
    ap.add_argument("--dir", default="/tmp/bsdb_e2e")
    ap.add_argument("--fused", action="store_true", help="F2: bsdb_mph_build_index_fixed")
    ap.add_argument("--ps", type=int, default=1 << 30, help="pass cache bytes (0 = device-sized)")
    args = ap.parse_args()
    if args.full:
        ctx = Context(0)
        full(ctx, args.full, args.approx, args.dir, args.ps, args.fused)
        return
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
