"""ctypes view of the CPU oracle (``liboracle.so``) and of the reference's own C
(``_ref/libbsdbref.so``).

TEST INFRASTRUCTURE ONLY: imported by ``tests/``, ``__graft_entry__.smoke()``
and the ``cpu_baseline`` leg of ``bench.py`` -- never by the product path in
``bsdb_amd/``.  The restatement follows the reference file:line cited in
``bsdb_oracle.c``; the reference library is the reference's own
``src/main/c/spooky.c`` + ``mph.c`` compiled by ``oracle/Makefile``.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_u64p = C.POINTER(C.c_uint64)
_u32p = C.POINTER(C.c_uint32)
_u8p = C.POINTER(C.c_uint8)


def _p(a: np.ndarray, t):
    return a.ctypes.data_as(t)


class BoMph(C.Structure):
    _fields_ = [("n", C.c_uint64), ("multiplier", C.c_uint64), ("global_seed", C.c_uint64),
                ("num_buckets", C.c_uint64), ("E", _u64p), ("array", _u64p),
                ("sig_width", C.c_uint32), ("signatures", _u64p)]


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"oracle not built: run `make -C {HERE}`")
        L = C.CDLL(path)
        L.bo_spooky_short.argtypes = [_u8p, C.c_uint64, C.c_uint64, _u64p]
        L.bo_spooky_rehash.argtypes = [_u64p, C.c_uint64, _u64p]
        L.bo_num_buckets.argtypes = [C.c_uint64]; L.bo_num_buckets.restype = C.c_uint64
        L.bo_bucket.argtypes = [C.c_uint64, C.c_uint64]; L.bo_bucket.restype = C.c_uint32
        L.bo_vertex_offset.argtypes = [C.c_uint64]; L.bo_vertex_offset.restype = C.c_uint64
        L.bo_signature_to_equation.argtypes = [_u64p, C.c_uint64, C.c_uint32, _u32p]
        L.bo_count_nonzero_pairs.argtypes = [C.c_uint64, C.c_uint64, _u64p]
        L.bo_count_nonzero_pairs.restype = C.c_uint64
        L.bo_hash_fixed.argtypes = [_u8p, C.c_uint32, C.c_uint64, C.c_uint64, _u64p]
        L.bo_hash_var.argtypes = [_u8p, _u64p, C.c_uint64, C.c_uint64, _u64p]
        L.bo_histogram_fixed.argtypes = [_u8p, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64, _u32p]
        L.bo_histogram_var.argtypes = [_u8p, _u64p, C.c_uint64, C.c_uint64, C.c_uint64, _u32p]
        L.bo_edge_offsets.argtypes = [_u32p, C.c_uint64, _u64p]
        L.bo_splitmix64.argtypes = [C.c_uint64]; L.bo_splitmix64.restype = C.c_uint64
        L.bo_gen_keys13.argtypes = [C.c_uint64, C.c_uint64, _u8p]
        L.bo_gen_keys13_mt.argtypes = [C.c_uint64, C.c_uint64, _u8p, C.c_int]
        L.bo_histogram_gen13_mt.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, _u32p, C.c_int]
        L.bo_histogram_gen13_mt.restype = C.c_double
        L.bo_histogram_fixed_mt.argtypes = [_u8p, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64, _u32p, C.c_int]
        L.bo_histogram_fixed_mt.restype = C.c_double
        L.bo_lookup_nocheck.argtypes = [C.POINTER(BoMph), _u64p]; L.bo_lookup_nocheck.restype = C.c_int64
        L.bo_lookup.argtypes = [C.POINTER(BoMph), _u64p]; L.bo_lookup.restype = C.c_int64
        L.bo_bitlist_get.argtypes = [_u64p, C.c_uint64, C.c_uint32]; L.bo_bitlist_get.restype = C.c_uint64
        L.bo_values_words.argtypes = [C.c_uint64]; L.bo_values_words.restype = C.c_uint64
        if hasattr(L, "bo_gov_build"):
            L.bo_gov_build.argtypes = [_u64p, C.c_uint64, C.c_uint32, _u64p, _u64p, C.c_uint64, _u64p, C.c_uint64]
            L.bo_gov_build.restype = C.c_int
        if hasattr(L, "bo_lookup_batch"):
            L.bo_lookup_batch.argtypes = [C.POINTER(BoMph), _u64p, C.c_uint64, C.c_int, C.POINTER(C.c_int64)]
        L.bo_bucket_batch.argtypes = [_u64p, C.c_uint64, C.c_uint64, _u32p]
        L.bo_gov_build_range_mt.argtypes = [_u64p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                                            C.c_uint32, _u64p, _u64p, _u64p, C.c_int]
        L.bo_gov_build_range_mt.restype = C.c_int
        L.bo_gov_build_mt.argtypes = [_u64p, C.c_uint64, C.c_uint32, _u64p, _u64p, C.c_uint64, _u64p, C.c_uint64,
                                      C.c_int, C.POINTER(C.c_double)]
        L.bo_gov_build_mt.restype = C.c_int
        L.bo_lookup_batch_mt.argtypes = [C.POINTER(BoMph), _u64p, C.c_uint64, C.c_int, C.POINTER(C.c_int64), C.c_int]
        L.bo_hash_fixed_mt.argtypes = [_u8p, C.c_uint32, C.c_uint64, C.c_uint64, _u64p, C.c_int]
        L.bo_varkey_len.argtypes = [C.c_uint64]; L.bo_varkey_len.restype = C.c_uint32
        L.bo_solve_stats.argtypes = [_u64p, C.c_int]
        L.bo_gen_keys_var.argtypes = [C.c_uint64, C.c_uint64, _u64p, _u8p]
        L.bo_histogram_genvar_mt.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, _u32p, C.c_int]
        L.bo_histogram_genvar_mt.restype = C.c_double
        _lib = L
    return _lib


# ---------------------------------------------------------------- helpers
def spooky_short(key: bytes, seed: int = 0) -> tuple:
    out = np.zeros(4, np.uint64)
    buf = np.frombuffer(bytes(key) + b"\0", np.uint8)
    lib().bo_spooky_short(_p(buf, _u8p), len(key), seed, _p(out, _u64p))
    return tuple(int(x) for x in out)


def spooky_rehash(sig0: int, sig1: int, seed: int) -> tuple:
    s = np.array([sig0, sig1], np.uint64)
    out = np.zeros(4, np.uint64)
    lib().bo_spooky_rehash(_p(s, _u64p), seed, _p(out, _u64p))
    return tuple(int(x) for x in out)


def num_buckets(n: int) -> int:
    return int(lib().bo_num_buckets(n))


def bucket(sig0: int, m: int) -> int:
    return int(lib().bo_bucket(sig0, m))


def signature_to_equation(sig0: int, sig1: int, seed_bits: int, nv: int) -> tuple:
    s = np.array([sig0, sig1], np.uint64)
    e = np.zeros(3, np.uint32)
    lib().bo_signature_to_equation(_p(s, _u64p), seed_bits, nv, _p(e, _u32p))
    return tuple(int(x) for x in e)


def hash_fixed(keys: np.ndarray, key_len: int, seed: int = 0) -> np.ndarray:
    keys = np.ascontiguousarray(keys, np.uint8).reshape(-1)
    n = keys.size // key_len if key_len else 0
    sig = np.zeros(2 * max(n, 1), np.uint64)
    lib().bo_hash_fixed(_p(keys, _u8p), key_len, n, seed, _p(sig, _u64p))
    return sig[: 2 * n].reshape(n, 2)


def hash_var(blob: np.ndarray, offsets: np.ndarray, seed: int = 0) -> np.ndarray:
    blob = np.ascontiguousarray(blob, np.uint8)
    if blob.size == 0:
        blob = np.zeros(1, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    n = offsets.size - 1
    sig = np.zeros(2 * max(n, 1), np.uint64)
    lib().bo_hash_var(_p(blob, _u8p), _p(offsets, _u64p), n, seed, _p(sig, _u64p))
    return sig[: 2 * n].reshape(n, 2)


def histogram_fixed(keys: np.ndarray, key_len: int, m: int, seed: int = 0) -> np.ndarray:
    keys = np.ascontiguousarray(keys, np.uint8).reshape(-1)
    n = keys.size // key_len
    counts = np.zeros(m, np.uint32)
    lib().bo_histogram_fixed(_p(keys, _u8p), key_len, n, seed, m, _p(counts, _u32p))
    return counts


def histogram_var(blob: np.ndarray, offsets: np.ndarray, m: int, seed: int = 0) -> np.ndarray:
    blob = np.ascontiguousarray(blob, np.uint8)
    if blob.size == 0:
        blob = np.zeros(1, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    counts = np.zeros(m, np.uint32)
    lib().bo_histogram_var(_p(blob, _u8p), _p(offsets, _u64p), offsets.size - 1, seed, m, _p(counts, _u32p))
    return counts


def edge_offsets(counts: np.ndarray) -> np.ndarray:
    counts = np.ascontiguousarray(counts, np.uint32)
    E = np.zeros(counts.size + 1, np.uint64)
    lib().bo_edge_offsets(_p(counts, _u32p), counts.size, _p(E, _u64p))
    return E


def gen_keys13(first: int, n: int) -> np.ndarray:
    out = np.zeros(13 * max(n, 1), np.uint8)
    lib().bo_gen_keys13(first, n, _p(out, _u8p))
    return out[: 13 * n]


def gen_keys13_mt(first: int, n: int, threads: int) -> np.ndarray:
    out = np.empty(13 * max(n, 1), np.uint8)
    lib().bo_gen_keys13_mt(first, n, _p(out, _u8p), threads)
    return out[: 13 * n]


def histogram_gen13_mt(first: int, n: int, m: int, threads: int, seed: int = 0):
    counts = np.zeros(m, np.uint32)
    dt = lib().bo_histogram_gen13_mt(first, n, seed, m, _p(counts, _u32p), threads)
    return counts, dt


def histogram_fixed_mt(keys: np.ndarray, key_len: int, m: int, threads: int, seed: int = 0):
    keys = np.ascontiguousarray(keys, np.uint8).reshape(-1)
    counts = np.zeros(m, np.uint32)
    dt = lib().bo_histogram_fixed_mt(_p(keys, _u8p), key_len, keys.size // key_len, seed, m,
                                     _p(counts, _u32p), threads)
    return counts, dt


def count_nonzero_pairs(start: int, end: int, array: np.ndarray) -> int:
    array = np.ascontiguousarray(array, np.uint64)
    return int(lib().bo_count_nonzero_pairs(start, end, _p(array, _u64p)))


# ----------------------------------------------- reference library (_ref)
_ref = None


class RefMph(C.Structure):
    """Layout of ``mph`` in the reference's src/main/c/mph.h:29-37."""
    _fields_ = [("size", C.c_uint64), ("multiplier", C.c_uint64), ("global_seed", C.c_uint64),
                ("edge_offset_and_seed_length", C.c_uint64), ("edge_offset_and_seed", _u64p),
                ("array_length", C.c_uint64), ("array", _u64p)]


def ref_lib():
    """The reference's own spooky.c + mph.c, or None when not built here."""
    global _ref
    if _ref is None:
        path = os.path.join(HERE, "_ref", "libbsdbref.so")
        if not os.path.exists(path):
            return None
        L = C.CDLL(path)
        L.spooky_short.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64, _u64p]
        L.spooky_short_rehash.argtypes = [_u64p, C.c_uint64, _u64p]
        L.mph_get_byte_array.argtypes = [C.POINTER(RefMph), C.c_char_p, C.c_uint64]
        L.mph_get_byte_array.restype = C.c_int64
        L.load_mph.argtypes = [C.c_int]
        L.load_mph.restype = C.POINTER(RefMph)
        _ref = L
    return _ref


def gov_build(sig: np.ndarray, width: int):
    """CPU GOV build (own deterministic solver; see bsdb_oracle.c).  Returns
    (rc, E, values, sigbits)."""
    sig = np.ascontiguousarray(sig, np.uint64).reshape(-1, 2)
    n = sig.shape[0]
    m = num_buckets(n)
    E = np.zeros(m + 1, np.uint64)
    vw = int(lib().bo_values_words(n))
    values = np.zeros(vw, np.uint64)
    sw = (n * width + 63) // 64 + 1
    sigbits = np.zeros(sw, np.uint64)
    rc = lib().bo_gov_build(_p(sig, _u64p), n, width, _p(E, _u64p), _p(values, _u64p), vw, _p(sigbits, _u64p), sw)
    return rc, E, values, sigbits


def solve_stats(reset: bool = True) -> dict:
    """The oracle solver's counters (bo_solve_stats), optionally reset."""
    out = np.zeros(5, np.uint64)
    lib().bo_solve_stats(_p(out, _u64p), 1 if reset else 0)
    return dict(zip(("attempts", "unorientable", "inconsistent", "degenerate", "singular_solved"),
                    (int(x) for x in out)))


def lookup_batch(sig: np.ndarray, n: int, E: np.ndarray, values: np.ndarray, width: int = 0, sigbits=None,
                 check: bool = True) -> np.ndarray:
    sig = np.ascontiguousarray(sig, np.uint64).reshape(-1, 2)
    m = E.size - 1
    sb = sigbits if sigbits is not None else np.zeros(1, np.uint64)
    mp = BoMph(n, 2 * m, 0, m, _p(E, _u64p), _p(values, _u64p), width, _p(sb, _u64p))
    out = np.zeros(max(sig.shape[0], 1), np.int64)
    lib().bo_lookup_batch(C.byref(mp), _p(sig, _u64p), sig.shape[0], 1 if check else 0,
                          out.ctypes.data_as(C.POINTER(C.c_int64)))
    return out[: sig.shape[0]]


# ------------------------------------------------- threaded forms, C5 keys
def cpu_threads() -> int:
    """CPUs this process may actually use: the affinity mask, capped by a
    cgroup CPU quota when one is set (the GPU box's os.cpu_count() shows the
    whole machine, its quota is lower)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def gov_build_mt(sig: np.ndarray, width: int, threads: int):
    """bo_gov_build over bucket ranges on `threads` threads: (rc, E, values,
    sigbits, seconds), identical to gov_build."""
    sig = np.ascontiguousarray(sig, np.uint64).reshape(-1, 2)
    n = sig.shape[0]
    m = num_buckets(n)
    E = np.zeros(m + 1, np.uint64)
    vw = int(lib().bo_values_words(n))
    values = np.zeros(vw, np.uint64)
    sw = (n * width + 63) // 64 + 1
    sigbits = np.zeros(sw, np.uint64)
    dt = C.c_double()
    rc = lib().bo_gov_build_mt(_p(sig, _u64p), n, width, _p(E, _u64p), _p(values, _u64p), vw, _p(sigbits, _u64p), sw,
                               threads, C.byref(dt))
    return rc, E, values, sigbits, dt.value


def lookup_batch_mt(sig: np.ndarray, n: int, E: np.ndarray, values: np.ndarray, width: int = 0, sigbits=None,
                    check: bool = True, threads: int = 1) -> np.ndarray:
    sig = np.ascontiguousarray(sig, np.uint64).reshape(-1, 2)
    m = E.size - 1
    sb = sigbits if sigbits is not None else np.zeros(1, np.uint64)
    mp = BoMph(n, 2 * m, 0, m, _p(E, _u64p), _p(values, _u64p), width, _p(sb, _u64p))
    out = np.zeros(max(sig.shape[0], 1), np.int64)
    lib().bo_lookup_batch_mt(C.byref(mp), _p(sig, _u64p), sig.shape[0], 1 if check else 0,
                             out.ctypes.data_as(C.POINTER(C.c_int64)), threads)
    return out[: sig.shape[0]]


def hash_fixed_mt(keys: np.ndarray, key_len: int, threads: int, seed: int = 0) -> np.ndarray:
    keys = np.ascontiguousarray(keys, np.uint8).reshape(-1)
    n = keys.size // key_len
    sig = np.zeros(2 * max(n, 1), np.uint64)
    lib().bo_hash_fixed_mt(_p(keys, _u8p), key_len, n, seed, _p(sig, _u64p), threads)
    return sig[: 2 * n].reshape(n, 2)


def gen_keys_var(first: int, n: int):
    """Config C5 keys [first, first+n): (blob u8, offsets u64[n+1])."""
    off = np.zeros(n + 1, np.uint64)
    lib().bo_gen_keys_var(first, n, _p(off, _u64p), None)
    blob = np.zeros(max(int(off[-1]), 1), np.uint8)
    lib().bo_gen_keys_var(first, n, _p(off, _u64p), _p(blob, _u8p))
    return blob[: int(off[-1])], off


def varkey_len(i: int) -> int:
    return int(lib().bo_varkey_len(i))


def histogram_genvar_mt(first: int, n: int, m: int, threads: int, seed: int = 0):
    counts = np.zeros(m, np.uint32)
    dt = lib().bo_histogram_genvar_mt(first, n, seed, m, _p(counts, _u32p), threads)
    return counts, dt


def splitmix64_np(x: np.ndarray) -> np.ndarray:
    """bo_splitmix64 over a u64 array (wrapping arithmetic)."""
    with np.errstate(over="ignore"):
        z = np.asarray(x, np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def buckets(sig: np.ndarray, m: int) -> np.ndarray:
    sig = np.ascontiguousarray(sig, np.uint64).reshape(-1, 2)
    out = np.zeros(max(sig.shape[0], 1), np.uint32)
    lib().bo_bucket_batch(_p(sig, _u64p), sig.shape[0], m, _p(out, _u32p))
    return out[: sig.shape[0]]


def gov_build_range(sig: np.ndarray, n_global: int, b_lo: int, b_hi: int, e_lo: int, width: int,
                    E: np.ndarray, values: np.ndarray, sigbits: np.ndarray, threads: int = 1) -> int:
    """bo_gov_build_range_mt into caller-zeroed full-size u64 arrays (in place)."""
    sig = np.ascontiguousarray(sig, np.uint64).reshape(-1, 2)
    for a in (E, values, sigbits):
        assert a.dtype == np.uint64 and a.flags.c_contiguous
    return lib().bo_gov_build_range_mt(_p(sig, _u64p), sig.shape[0], n_global, b_lo, b_hi, e_lo, width,
                                       _p(E, _u64p), _p(values, _u64p), _p(sigbits, _u64p), threads)
