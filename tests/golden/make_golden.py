"""Generates tests/golden/golden_v1.npz from the REFERENCE's own C code.

The expected outputs here come from /root/reference/src/main/c/spooky.c and
mph.c, compiled unmodified by oracle/Makefile into oracle/_ref/libbsdbref.so.
Those two files are the reference's bit-exact spec of the hash path: the
reference's own NativeTest.testLoadHash (src/test/java/tech/bsdb/io/
NativeTest.java:115-135) asserts that sux4j's Java getLong equals this C
mph_get_byte_array on 1 M keys.  Inputs are generated deterministically below;
the fixture stores inputs and outputs (data only, no reference source).

Run (needs /root/reference and `make -C oracle`):
    python tests/golden/make_golden.py
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden_v1.npz")
SEEDS = np.array([0, 0x0123456789ABCDEF, (1 << 63) + 5, 0x3F << 56], dtype=np.uint64)


def ref_spooky(R, key: bytes, seed: int):
    out = (C.c_uint64 * 4)()
    buf = C.create_string_buffer(key, len(key) + 1)
    R.spooky_short(buf, len(key), seed, out)
    return list(out)


def ref_rehash(R, s0, s1, seed):
    sig = (C.c_uint64 * 2)(s0, s1)
    out = (C.c_uint64 * 4)()
    R.spooky_short_rehash(sig, seed, out)
    return list(out)


def ascii_keys(lo, hi):
    return [str(i).encode() for i in range(lo, hi)]


def pack_var(keys):
    off = np.zeros(len(keys) + 1, np.uint64)
    off[1:] = np.cumsum([len(k) for k in keys])
    return np.frombuffer(b"".join(keys), np.uint8).copy(), off


def basetest_keys(n, rng):
    """BaseTest.genKey(len, index) style (src/test/java/tech/bsdb/BaseTest.java:16-24):
    8-byte big-endian index, then a random tail; lengths 8..64, Zipf(1.1)."""
    lens = np.arange(8, 65)
    p = 1.0 / np.arange(1, lens.size + 1) ** 1.1
    p /= p.sum()
    L = rng.choice(lens, size=n, p=p)
    return [int(i).to_bytes(8, "big") + rng.integers(0, 256, int(l) - 8, dtype=np.uint8).tobytes()
            for i, l in zip(range(n), L)]


def histogram(R, keys, m):
    counts = np.zeros(m, np.uint32)
    for k in keys:
        s0 = ref_spooky(R, k, 0)[0]
        counts[O.bucket(s0, m)] += 1
    return counts


def main():
    R = O.ref_lib()
    if R is None:
        raise SystemExit("oracle/_ref/libbsdbref.so missing: run `make -C oracle` with /root/reference present")
    R.mph_get_byte_array.argtypes = [C.POINTER(O.RefMph), C.c_char_p, C.c_uint64]
    rng = np.random.default_rng(0xB5DB)
    g = {}

    # 1. spooky_short, every length 0..200 (all tail/16-byte/32-byte-block paths), 4 seeds
    msg = ((np.arange(256) * 131 + 7) & 255).astype(np.uint8).tobytes()
    g["len_msg"] = np.frombuffer(msg, np.uint8)
    g["len_seeds"] = SEEDS
    g["len_sig"] = np.array([[ref_spooky(R, msg[:L], int(s)) for L in range(201)] for s in SEEDS], np.uint64)

    # 2. NativeTest keys "0".."999999" (NativeTest.java:119-122): full histogram at
    #    m = 1e6/1500+1 = 667 and a strided sample of signatures.
    keys = ascii_keys(0, 1_000_000)
    m = 1_000_000 // 1500 + 1
    sig0 = np.array([ref_spooky(R, k, 0)[:2] for k in keys], np.uint64)
    g["native_sample_idx"] = np.arange(0, 1_000_000, 97, dtype=np.int64)
    g["native_sample_sig"] = sig0[g["native_sample_idx"]]
    counts = np.zeros(m, np.uint32)
    np.add.at(counts, np.array([O.bucket(int(s), m) for s in sig0[:, 0]]), 1)
    g["native_counts"] = counts
    g["native_xor_sig0"] = np.bitwise_xor.reduce(sig0[:, 0])
    g["native_xor_sig1"] = np.bitwise_xor.reduce(sig0[:, 1])

    # 3. BSDBWriterTest keys "1".."8290050" would be 8.3 M ctypes calls; keep the
    #    first 200 000 (BSDBWriterTest.java:162-164 getKey) with a full histogram.
    wkeys = ascii_keys(1, 200_001)
    wm = len(wkeys) // 1500 + 1
    g["writer_counts"] = histogram(R, wkeys, wm)

    # 4. 13-byte synthetic keys: signatures of the first
    #    8192 and the histogram of the first 1 M at m = 667.
    k13 = O.gen_keys13(0, 1_000_000).reshape(-1, 13)
    g["k13_sig"] = np.array([ref_spooky(R, k13[i].tobytes(), 0)[:2] for i in range(8192)], np.uint64)
    g["k13_counts"] = histogram(R, [k13[i].tobytes() for i in range(1_000_000)], m)
    g["k13_head"] = k13[:16].copy()   # the generator's own first keys, pinned

    # 5. variable-length BaseTest-style keys 8..64 B
    vk = basetest_keys(4000, rng)
    g["var_blob"], g["var_off"] = pack_var(vk)
    g["var_sig"] = np.array([ref_spooky(R, k, 0)[:2] for k in vk], np.uint64)

    # 6. rehash (spooky_short_rehash, the equation generator's first step)
    rs = rng.integers(0, 2**63, size=(512, 2), dtype=np.uint64) * np.uint64(2) + np.uint64(1)
    rseed = (rng.integers(0, 256, size=512, dtype=np.uint64) << np.uint64(56))
    g["rehash_in"] = rs
    g["rehash_seed"] = rseed
    g["rehash_out"] = np.array([ref_rehash(R, int(a), int(b), int(s)) for (a, b), s in zip(rs, rseed)], np.uint64)

    # 7. A12 lookup arithmetic through the reference's mph_get_byte_array on an
    #    mph with real edge offsets (the keys' own histogram), random local seeds
    #    and random 2-bit values: pins bucket, vertexOffset, signatureToEquation,
    #    the 2-bit reads and countNonzeroPairs (mph.c:63-96, GOV:557-580).
    for name, lk in (("lk_ascii", ascii_keys(0, 30_000)),
                     ("lk_k13", [k13[i].tobytes() for i in range(30_000)])):
        n = len(lk)
        lm = n // 1500 + 1
        cnt = histogram(R, lk, lm)
        E = np.zeros(lm + 1, np.uint64)
        E[1:] = np.cumsum(cnt.astype(np.uint64))
        E[:-1] |= rng.integers(0, 256, size=lm, dtype=np.uint64) << np.uint64(56)
        words = int(O.lib().bo_values_words(n))
        arr = rng.integers(0, 2**63, size=words, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, size=words, dtype=np.uint64)
        mp = O.RefMph(n, 2 * lm, 0, lm + 1, E.ctypes.data_as(C.POINTER(C.c_uint64)), words,
                      arr.ctypes.data_as(C.POINTER(C.c_uint64)))
        res = np.array([R.mph_get_byte_array(C.byref(mp), k, len(k)) for k in lk], np.int64)
        blob, off = pack_var(lk)
        g[name + "_blob"], g[name + "_off"] = blob, off
        g[name + "_E"], g[name + "_array"], g[name + "_res"] = E, arr, res

    np.savez_compressed(OUT, **g)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
