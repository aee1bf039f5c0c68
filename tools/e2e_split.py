"""Where the end-to-end C2 time goes (measurement tool): the F2 host build
(bsdb_mph_build_index_fixed) into a directory, then the dump, timed apart;
the same with the files under /dev/shm (memory) to separate the file system.

    python tools/e2e_split.py [--n KEYS]"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bsdb_amd import Context  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    args = ap.parse_args()
    n = args.n
    ctx = Context(0)
    keys = ctx.gen_keys13(0, n)[: 13 * n].cpu().numpy()
    addr = np.uint64(0x1000) + np.uint64(48) * np.arange(n, dtype=np.uint64)
    for where in ("/tmp", "/dev/shm", "/tmp", "/dev/shm"):
        d = tempfile.mkdtemp(prefix="bsdb_split_", dir=where)
        try:
            t0 = time.perf_counter()
            mph = ctx.mph_build_index_fixed(keys, 13, 4, addr, os.path.join(d, "index.db"), os.path.join(d, "index_a.db"))
            t1 = time.perf_counter()
            mph.dump(os.path.join(d, "hash.dump"))
            t2 = time.perf_counter()
            mph.close()
        finally:
            shutil.rmtree(d, ignore_errors=True)
        print(json.dumps({"dir": where, "n": n, "build_index_ms": (t1 - t0) * 1e3, "dump_ms": (t2 - t1) * 1e3,
                          "keys_per_s": n / (t2 - t0)}), flush=True)


if __name__ == "__main__":
    main()
