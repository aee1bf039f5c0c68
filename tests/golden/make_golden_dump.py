"""Generates tests/golden/dump_v1.npz: a GOV.dump-format MPHF file (A15) and
the REFERENCE's own reading of it.

The dump is the raw layout of GOVMinimalPerfectHashFunctionModified.dump
(src/main/java/it/unimi/dsi/sux4j/mph/GOVMinimalPerfectHashFunctionModified.java:592-619):
native-endian u64 n, multiplier (= 2m), globalSeed (= 0), len(E), E[],
len(array), array[].  Its contents are a GOV build of the NativeTest key set
"0".."29999" (NativeTest.java:119-122) by the CPU oracle.  The expected
outputs are what the reference's own C does with that file:
load_mph (src/main/c/mph.c:28-43) reads it from a file descriptor and
mph_get_byte_array (mph.c:86-96) returns every key's unchecked rank.

The fixture is data only (the file bytes, the keys and the reference's
answers); the GPU test loads the same bytes through bsdb_mph_load and must
return the same ranks, so A15 is pinned even where oracle/_ref is absent.

Run (needs /root/reference and `make -C oracle`):
    python tests/golden/make_golden_dump.py
"""
from __future__ import annotations

import os
import struct
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dump_v1.npz")
N = 30_000


def dump_bytes(n: int, E: np.ndarray, values: np.ndarray) -> bytes:
    m = E.size - 1
    head = struct.pack("<4Q", n, 2 * m, 0, m + 1)
    return head + E.astype("<u8").tobytes() + struct.pack("<Q", values.size) + values.astype("<u8").tobytes()


def main():
    R = O.ref_lib()
    if R is None:
        raise SystemExit("oracle/_ref/libbsdbref.so missing: run `make -C oracle` with /root/reference present")
    keys = [str(i).encode() for i in range(N)]
    off = np.zeros(N + 1, np.uint64)
    off[1:] = np.cumsum([len(k) for k in keys])
    blob = np.frombuffer(b"".join(keys), np.uint8).copy()
    sig = O.hash_var(blob, off)
    rc, E, values, _ = O.gov_build(sig, 0)
    assert rc == 0
    data = dump_bytes(N, E, values)
    with tempfile.NamedTemporaryFile(suffix=".dump", delete=False) as f:
        f.write(data)
        path = f.name
    try:
        fd = os.open(path, os.O_RDONLY)
        try:
            rm = R.load_mph(fd)
        finally:
            os.close(fd)
        res = np.array([R.mph_get_byte_array(rm, k, len(k)) for k in keys], np.int64)
    finally:
        os.unlink(path)
    assert np.array_equal(np.sort(res), np.arange(N)), "the reference reads a minimal perfect hash"
    np.savez_compressed(OUT, dump=np.frombuffer(data, np.uint8), blob=blob, off=off, ref_rank=res)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
