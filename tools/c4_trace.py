#!/usr/bin/env python3
"""C4 exact full build on one GPU (bsdb_dev_mph_build_index_passes_fixed), run
once, for a kernel trace: under `rocprofv3 --kernel-trace` the per-pass
k_gov_solve / k_gov_solve_big start and end times come out of the trace CSV
(tools/trace_passes.py).  n defaults to the README count."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=13_193_787_549)
    ap.add_argument("--width", type=int, default=4)
    ap.add_argument("--passes", type=int, default=0)
    ap.add_argument("--host-index", action="store_true", help="index slots to host memory (as the bench)")
    args = ap.parse_args()
    import numpy as np
    import torch
    from bsdb_amd import Context
    ctx = Context(0)
    n = args.n
    keys = torch.empty(13 * n + 16, dtype=torch.uint8, device="cuda")
    ctx.gen_keys13(0, n, out=keys)
    torch.cuda.synchronize()
    index = np.empty(n, np.uint64) if args.host_index else None
    t0 = time.perf_counter()
    E, vals, sb, used = ctx.mph_build_index_passes(keys, 13, n, args.width, args.passes, addr_base=0x1000,
                                                   addr_stride=48, index=index)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ok = int(E[-1].item()) & ((1 << 56) - 1) == n
    print(f'{{"n": {n}, "passes": {used}, "s": {dt:.3f}, "keys_per_s": {n / dt:.4g}, "E[m]==n": {str(ok).lower()}}}',
          flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
