"""ctypes binding of ``include/bsdb_mi355x.h`` (``libbsdb_mi355x.so``).

This is the product path: every call lands in a hand-written gfx950 kernel.
There is no CPU fallback -- if the library is missing or a call fails, a
:class:`BsdbError` is raised (mirroring the reference's JNI convention of
negative return codes turned into exceptions, ``src/main/c/native.c:29-34``).

Device buffers are ``torch`` tensors (torch is plumbing here: HBM allocation,
streams, ``torch.distributed``); the C ABI itself takes plain pointers.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libbsdb_mi355x.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "bsdb_mi355x.h")

BSDB_OK = 0
ERRORS = {-22: "EINVAL", -12: "ENOMEM", -5: "EIO", -19: "ENODEV", -17: "EDUP", -34: "ESEEDS", -7: "E2BIG"}

# (name, restype, argtypes) -- kept in the order of include/bsdb_mi355x.h
_vp, _u64, _u32, _i = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int
SIGNATURES = [
    ("bsdb_abi_version", _i, []),
    ("bsdb_strerror", C.c_char_p, [_i]),
    ("bsdb_open", _i, [_i, C.POINTER(_vp)]),
    ("bsdb_close", _i, [_vp]),
    ("bsdb_num_buckets", _u64, [_u64]),
    ("bsdb_dev_hash_fixed", _i, [_vp, _vp, _u32, _u64, _u64, _vp, _vp]),
    ("bsdb_dev_hash_var", _i, [_vp, _vp, _u64, _vp, _u64, _u64, _vp, _vp]),
    ("bsdb_dev_histogram_fixed", _i, [_vp, _vp, _u32, _u64, _u64, _u64, _vp, _vp]),
    ("bsdb_dev_histogram_var", _i, [_vp, _vp, _u64, _vp, _u64, _u64, _u64, _vp, _vp]),
    ("bsdb_dev_edge_offsets", _i, [_vp, _vp, _u64, _vp, _vp]),
    ("bsdb_dev_lookup", _i, [_vp, _vp, _u64, _u64, _u64, _vp, _vp, _u32, _vp, _i, _vp, _vp]),
    ("bsdb_dev_sign", _i, [_vp, _vp, _u64, _u64, _vp, _vp, _u32, _vp, _vp]),
    ("bsdb_dev_index_scatter", _i, [_vp, _vp, _vp, _u64, _u64, _u64, _vp, _vp, _vp, _vp, _vp]),
    ("bsdb_values_words", _u64, [_u64]),
    ("bsdb_dev_gov_build", _i, [_vp, _vp, _u64, _u32, _vp, _vp, _vp, _vp]),
    ("bsdb_set_histogram_mode", _i, [_vp, _i]),
    ("bsdb_set_frontend", _i, [_vp, _i]),
    ("bsdb_set_chunk_keys", _i, [_vp, _u64]),
    ("bsdb_fallback_count", _i, [_vp, C.POINTER(_u64)]),
    ("bsdb_set_profiling", _i, [_vp, _i]),
    ("bsdb_profile_read", _i, [_vp, _i, C.POINTER(C.c_double), C.POINTER(_u64), C.POINTER(_u64)]),
    ("bsdb_histogram_fixed", _i, [_vp, _vp, _u32, _u64, _u64, _u64, _vp]),
    ("bsdb_hash_fixed", _i, [_vp, _vp, _u32, _u64, _u64, _vp]),
    ("bsdb_histogram_var", _i, [_vp, _vp, _vp, _u64, _u64, _u64, _vp]),
    ("bsdb_hash_var", _i, [_vp, _vp, _vp, _u64, _u64, _vp]),
    ("bsdb_dev_gen_keys13", _i, [_vp, _u64, _u64, _vp, _vp]),
    ("bsdb_dev_gen_keys_var", _i, [_vp, _u64, _u64, _vp, _vp, _u64, _vp]),
]

HIST_AUTO, HIST_PARTITIONED, HIST_ATOMIC = 0, 1, 2


class BsdbError(RuntimeError):
    def __init__(self, fn: str, code: int):
        super().__init__(f"{fn} failed: {code} ({ERRORS.get(code, '?')})")
        self.code = code


_lib: Optional[C.CDLL] = None


def lib() -> C.CDLL:
    """Loads the gfx950 library; raises if it was not built (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `python -c 'import __graft_entry__ as g; g.build()'` "
                               "or `make -C bsdb_amd/csrc` (hipcc --offload-arch=gfx950)")
        # torch's bundled HIP runtime shares the soname libamdhip64.so.7: import
        # torch first so this library binds to the same runtime instance.
        import torch  # noqa: F401
        L = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _check(fn: str, rc: int):
    if rc != BSDB_OK:
        raise BsdbError(fn, rc)


def num_buckets(n: int) -> int:
    return int(lib().bsdb_num_buckets(n))


def _ptr(t) -> int:
    return t.data_ptr()


def _stream(stream) -> Optional[int]:
    import torch
    if stream is None:
        return torch.cuda.current_stream().cuda_stream
    return stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)


class Context:
    """One ``bsdb_ctx`` on one HIP device.  All ``*_dev`` methods take torch
    tensors resident on that device and enqueue on the current torch stream."""

    def __init__(self, device: int = 0):
        self._h = C.c_void_p()
        _check("bsdb_open", lib().bsdb_open(device, C.byref(self._h)))
        self.device = device

    def close(self):
        if self._h:
            _check("bsdb_close", lib().bsdb_close(self._h))
            self._h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- configuration
    def set_histogram_mode(self, mode: int):
        _check("bsdb_set_histogram_mode", lib().bsdb_set_histogram_mode(self._h, mode))

    def set_frontend(self, frontend: int):
        _check("bsdb_set_frontend", lib().bsdb_set_frontend(self._h, frontend))

    def set_chunk_keys(self, n: int):
        _check("bsdb_set_chunk_keys", lib().bsdb_set_chunk_keys(self._h, n))

    def fallback_count(self) -> int:
        """Chunks recounted by the overflow fallback since open (synchronises)."""
        v = C.c_uint64()
        _check("bsdb_fallback_count", lib().bsdb_fallback_count(self._h, C.byref(v)))
        return v.value

    # ---- live per-kernel timing (HIP events on the launch stream)
    PASS1, PASS2, SCAN = 0, 1, 2

    def set_profiling(self, on: bool):
        _check("bsdb_set_profiling", lib().bsdb_set_profiling(self._h, 1 if on else 0))

    def profile_read(self, kind: int):
        t, nl, nk = C.c_double(), C.c_uint64(), C.c_uint64()
        _check("bsdb_profile_read", lib().bsdb_profile_read(self._h, kind, C.byref(t), C.byref(nl), C.byref(nk)))
        return t.value, nl.value, nk.value

    # ---- A3: signatures
    def hash_fixed(self, keys, key_len: int, seed: int = 0, out=None, stream=None):
        import torch
        n = keys.numel() // key_len if key_len else 0
        if out is None:
            out = torch.empty((n, 2), dtype=torch.int64, device=keys.device)
        _check("bsdb_dev_hash_fixed", lib().bsdb_dev_hash_fixed(
            self._h, _ptr(keys), key_len, n, seed & (2**64 - 1), _ptr(out), _stream(stream)))
        return out

    def hash_var(self, blob, offsets, seed: int = 0, out=None, stream=None):
        import torch
        n = offsets.numel() - 1
        if out is None:
            out = torch.empty((n, 2), dtype=torch.int64, device=offsets.device)
        _check("bsdb_dev_hash_var", lib().bsdb_dev_hash_var(
            self._h, _ptr(blob), blob.numel(), _ptr(offsets), n, seed & (2**64 - 1), _ptr(out), _stream(stream)))
        return out

    # ---- A3+A4+A6: bucket-occupancy histogram (accumulating)
    def histogram_fixed(self, keys, key_len: int, m: int, counts=None, seed: int = 0, n: Optional[int] = None,
                        stream=None):
        import torch
        if n is None:
            n = keys.numel() // key_len
        if counts is None:
            counts = torch.zeros(m, dtype=torch.int32, device=keys.device)
        _check("bsdb_dev_histogram_fixed", lib().bsdb_dev_histogram_fixed(
            self._h, _ptr(keys), key_len, n, seed & (2**64 - 1), m, _ptr(counts), _stream(stream)))
        return counts

    def histogram_var(self, blob, offsets, m: int, counts=None, seed: int = 0, stream=None):
        import torch
        if counts is None:
            counts = torch.zeros(m, dtype=torch.int32, device=offsets.device)
        _check("bsdb_dev_histogram_var", lib().bsdb_dev_histogram_var(
            self._h, _ptr(blob), blob.numel(), _ptr(offsets), offsets.numel() - 1, seed & (2**64 - 1), m,
            _ptr(counts), _stream(stream)))
        return counts

    def edge_offsets(self, counts, out=None, stream=None):
        import torch
        m = counts.numel()
        if out is None:
            out = torch.empty(m + 1, dtype=torch.int64, device=counts.device)
        _check("bsdb_dev_edge_offsets", lib().bsdb_dev_edge_offsets(
            self._h, _ptr(counts), m, _ptr(out), _stream(stream)))
        return out

    # ---- A5/A6/A8/A11: GOV build on the device
    def gov_build(self, sig, width: int, stream=None):
        import torch
        n = sig.shape[0]
        m = n // 1500 + 1
        E = torch.empty(m + 1, dtype=torch.int64, device=sig.device)
        values = torch.empty(int(lib().bsdb_values_words(n)), dtype=torch.int64, device=sig.device)
        sigbits = torch.empty((n * width + 63) // 64 + 1, dtype=torch.int64, device=sig.device) if width else None
        _check("bsdb_dev_gov_build", lib().bsdb_dev_gov_build(
            self._h, _ptr(sig), n, width, _ptr(E), _ptr(values), _ptr(sigbits) if sigbits is not None else None,
            _stream(stream)))
        return E, values, sigbits

    # ---- A11-A13: MPHF evaluation over (E, values[, checksum bits])
    def lookup(self, sig, n: int, E, values, width: int = 0, sigbits=None, check: bool = True, out=None,
               stream=None):
        import torch
        nq = sig.shape[0]
        if out is None:
            out = torch.empty(nq, dtype=torch.int64, device=sig.device)
        _check("bsdb_dev_lookup", lib().bsdb_dev_lookup(
            self._h, _ptr(sig), nq, n, E.numel() - 1, _ptr(E), _ptr(values), width,
            _ptr(sigbits) if sigbits is not None else None, 1 if check else 0, _ptr(out), _stream(stream)))
        return out

    def sign(self, sig, E, values, width: int, out=None, stream=None):
        import torch
        n = sig.shape[0]
        if out is None:
            out = torch.zeros((n * width + 63) // 64 + 1, dtype=torch.int64, device=sig.device)
        _check("bsdb_dev_sign", lib().bsdb_dev_sign(
            self._h, _ptr(sig), n, E.numel() - 1, _ptr(E), _ptr(values), width, _ptr(out), _stream(stream)))
        return out

    def index_scatter(self, rank, addr, start: int, length: int, index, value8=None, value_len=None, index_a=None,
                      stream=None):
        _check("bsdb_dev_index_scatter", lib().bsdb_dev_index_scatter(
            self._h, _ptr(rank), _ptr(addr), rank.numel(), start, length, _ptr(index),
            _ptr(value8) if value8 is not None else None, _ptr(value_len) if value_len is not None else None,
            _ptr(index_a) if index_a is not None else None, _stream(stream)))

    def gen_keys_var(self, first: int, n: int, stream=None):
        """Config C5 var-len keys on the device: (blob u8, offsets int64[n+1])."""
        import torch
        off = torch.empty(n + 1, dtype=torch.int64, device=f"cuda:{self.device}")
        _check("bsdb_dev_gen_keys_var", lib().bsdb_dev_gen_keys_var(self._h, first, n, _ptr(off), None, 0,
                                                                    _stream(stream)))
        total = int(off[-1])
        blob = torch.empty(total + 16, dtype=torch.uint8, device=f"cuda:{self.device}")
        _check("bsdb_dev_gen_keys_var", lib().bsdb_dev_gen_keys_var(self._h, first, n, _ptr(off), _ptr(blob),
                                                                    total + 16, _stream(stream)))
        return blob, off

    def gen_keys13(self, first: int, n: int, out=None, stream=None):
        import torch
        if out is None:
            out = torch.empty(13 * n + 16, dtype=torch.uint8, device=f"cuda:{self.device}")
        _check("bsdb_dev_gen_keys13", lib().bsdb_dev_gen_keys13(self._h, first, n, _ptr(out), _stream(stream)))
        return out

    # ---- host-buffer API (numpy in, numpy out; includes H2D/D2H)
    def histogram_fixed_host(self, keys_np, key_len: int, m: int, counts_np=None, seed: int = 0):
        import numpy as np
        keys_np = np.ascontiguousarray(keys_np, np.uint8)
        if counts_np is None:
            counts_np = np.zeros(m, np.uint32)
        n = keys_np.size // key_len
        _check("bsdb_histogram_fixed", lib().bsdb_histogram_fixed(
            self._h, keys_np.ctypes.data, key_len, n, seed & (2**64 - 1), m, counts_np.ctypes.data))
        return counts_np

    def hash_fixed_host(self, keys_np, key_len: int, seed: int = 0):
        import numpy as np
        keys_np = np.ascontiguousarray(keys_np, np.uint8)
        n = keys_np.size // key_len
        out = np.zeros((max(n, 1), 2), np.uint64)
        _check("bsdb_hash_fixed", lib().bsdb_hash_fixed(
            self._h, keys_np.ctypes.data, key_len, n, seed & (2**64 - 1), out.ctypes.data))
        return out[:n]

    @staticmethod
    def _var_host_args(blob_np, off_np):
        import numpy as np
        blob_np = np.ascontiguousarray(blob_np, np.uint8)
        off_np = np.ascontiguousarray(off_np, np.uint64)
        if off_np.ndim != 1 or off_np.size < 1:
            raise ValueError("offsets must be a 1-D array of n+1 entries")
        if off_np.size > 1 and (int(off_np[-1]) > blob_np.size or np.any(off_np[1:] < off_np[:-1])):
            raise ValueError("offsets must be non-decreasing and within the blob")
        return blob_np, off_np, off_np.size - 1

    def histogram_var_host(self, blob_np, off_np, m: int, counts_np=None, seed: int = 0):
        """Host-buffer var-len histogram (bsdb_histogram_var): key i is
        blob[off[i]:off[i+1]]; counts accumulate into counts_np (u32[m])."""
        import numpy as np
        blob_np, off_np, n = self._var_host_args(blob_np, off_np)
        if counts_np is None:
            counts_np = np.zeros(m, np.uint32)
        _check("bsdb_histogram_var", lib().bsdb_histogram_var(
            self._h, blob_np.ctypes.data, off_np.ctypes.data, n, seed & (2**64 - 1), m, counts_np.ctypes.data))
        return counts_np

    def hash_var_host(self, blob_np, off_np, seed: int = 0):
        """Host-buffer var-len signatures (bsdb_hash_var), (n, 2) u64."""
        import numpy as np
        blob_np, off_np, n = self._var_host_args(blob_np, off_np)
        out = np.zeros((max(n, 1), 2), np.uint64)
        _check("bsdb_hash_var", lib().bsdb_hash_var(
            self._h, blob_np.ctypes.data, off_np.ctypes.data, n, seed & (2**64 - 1), out.ctypes.data))
        return out[:n]
