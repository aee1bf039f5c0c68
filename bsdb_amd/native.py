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
# BSDB_LIB: an alternative in-tree build of the same library (tools/ variant
# experiments); the default is the product build
LIB_PATH = os.environ.get("BSDB_LIB") or os.path.join(HERE, "libbsdb_mi355x.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "bsdb_mi355x.h")

BSDB_OK = 0
ERRORS = {-22: "EINVAL", -12: "ENOMEM", -5: "EIO", -19: "ENODEV", -17: "EDUP", -34: "ESEEDS", -7: "E2BIG",
          -70: "ECOMM", -9: "EFILE", -74: "EVERIFY"}
COMM_ID_BYTES = 128

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
    ("bsdb_dev_gov_build_ranks", _i, [_vp, _vp, _u64, _u32, _vp, _vp, _vp, _vp, _vp]),
    ("bsdb_dev_gov_build_range", _i, [_vp, _vp, _u64, _u64, _u64, _u64, _u64, _u32, _vp, _vp, _vp, _vp, _vp]),
    ("bsdb_gov_range_windows", _i, [_u64, _u32, _u64, _u64, _vp]),
    ("bsdb_dev_gov_build_window", _i, [_vp, _vp, _u64, _u64, _u64, _u64, _u64, _u32, _vp, _vp, _u64, _u64, _vp, _u64,
                                       _u64, _vp, _vp]),
    ("bsdb_dev_mph_build_index_passes_fixed", _i, [_vp, _vp, _u32, _u64, _u32, _u32, _vp, _u64, _u64, _vp, _vp,
                                                   _vp, _vp, _vp, C.POINTER(_u32), _vp]),
    ("bsdb_dev_mph_build_index_passes_var", _i, [_vp, _vp, _u64, _vp, _u64, _u32, _u32, _vp, _u64, _u64, _vp, _vp,
                                                 _vp, _vp, _vp, C.POINTER(_u32), _vp]),
    ("bsdb_dev_partition_owners", _i, [_vp, _vp, _vp, _u64, _u64, _i, _vp, _vp, _vp, _vp]),
    ("bsdb_release_workspace", _i, [_vp]),
    ("bsdb_set_verify", _i, [_vp, _i]),
    ("bsdb_set_histogram_mode", _i, [_vp, _i]),
    ("bsdb_set_frontend", _i, [_vp, _i]),
    ("bsdb_set_chunk_keys", _i, [_vp, _u64]),
    ("bsdb_set_pipeline", _i, [_vp, _i, _u64, _u32]),
    ("bsdb_fallback_count", _i, [_vp, C.POINTER(_u64)]),
    ("bsdb_fused_status", _i, [_vp, C.POINTER(_u64), C.POINTER(_u64)]),
    ("bsdb_set_profiling", _i, [_vp, _i]),
    ("bsdb_profile_read", _i, [_vp, _i, C.POINTER(C.c_double), C.POINTER(_u64), C.POINTER(_u64)]),
    ("bsdb_histogram_fixed", _i, [_vp, _vp, _u32, _u64, _u64, _u64, _vp]),
    ("bsdb_hash_fixed", _i, [_vp, _vp, _u32, _u64, _u64, _vp]),
    ("bsdb_histogram_var", _i, [_vp, _vp, _vp, _u64, _u64, _u64, _vp]),
    ("bsdb_hash_var", _i, [_vp, _vp, _vp, _u64, _u64, _vp]),
    ("bsdb_dev_gen_keys13", _i, [_vp, _u64, _u64, _vp, _vp]),
    ("bsdb_dev_gen_keys_var", _i, [_vp, _u64, _u64, _vp, _vp, _u64, _vp]),
    ("bsdb_comm_available", _i, []),
    ("bsdb_comm_unique_id", _i, [_vp]),
    ("bsdb_comm_init", _i, [_vp, _i, _i, _vp]),
    ("bsdb_dev_histogram_finalize", _i, [_vp, _vp, _u64, _u64, _vp, _vp]),
    ("bsdb_dev_allreduce_u64", _i, [_vp, _vp, _u64, _vp]),
    ("bsdb_multi_open", _i, [_i, _vp, C.POINTER(_vp)]),
    ("bsdb_multi_close", _i, [_vp]),
    ("bsdb_multi_size", _i, [_vp]),
    ("bsdb_multi_ctx", _i, [_vp, _i, C.POINTER(_vp)]),
    ("bsdb_multi_histogram_fixed", _i, [_vp, _vp, _u32, _u64, _u64, _vp]),
    ("bsdb_multi_histogram_var", _i, [_vp, _vp, _vp, _u64, _u64, _vp]),
    ("bsdb_multi_mph_build_index_fixed", _i, [_vp, _vp, _u32, _u64, _u32, _vp, _vp, _vp, _i, C.c_char_p, C.c_char_p,
                                              _vp, _vp, _vp]),
    ("bsdb_multi_mph_build_index_var", _i, [_vp, _vp, _vp, _u64, _u32, _vp, _vp, _vp, _i, C.c_char_p, C.c_char_p,
                                            _vp, _vp, _vp]),
    ("bsdb_mph_build_fixed", _i, [_vp, _vp, _u32, _u64, _u32, C.POINTER(_vp)]),
    ("bsdb_mph_build_var", _i, [_vp, _vp, _vp, _u64, _u32, C.POINTER(_vp)]),
    ("bsdb_mph_build_index_fixed", _i, [_vp, _vp, _u32, _u64, _u32, _vp, _vp, _vp, _i, C.c_char_p, C.c_char_p,
                                        C.POINTER(_vp)]),
    ("bsdb_mph_build_index_var", _i, [_vp, _vp, _vp, _u64, _u32, _vp, _vp, _vp, _i, C.c_char_p, C.c_char_p,
                                      C.POINTER(_vp)]),
    ("bsdb_mph_info", _i, [_vp, C.POINTER(_u64), C.POINTER(_u64), C.POINTER(_u32), C.POINTER(_u64), C.POINTER(_u64)]),
    ("bsdb_mph_sizes", _i, [_u64, _u32, C.POINTER(_u64), C.POINTER(_u64), C.POINTER(_u64), C.POINTER(_u64)]),
    ("bsdb_mph_export", _i, [_vp, _vp, _vp, _vp]),
    ("bsdb_mph_import", _i, [_vp, _u64, _u32, _vp, _vp, _vp, C.POINTER(_vp)]),
    ("bsdb_mph_dump", _i, [_vp, C.c_char_p]),
    ("bsdb_mph_load", _i, [_vp, C.c_char_p, C.POINTER(_vp)]),
    ("bsdb_mph_lookup_fixed", _i, [_vp, _vp, _u32, _u64, _i, _vp]),
    ("bsdb_mph_lookup_var", _i, [_vp, _vp, _vp, _u64, _i, _vp]),
    ("bsdb_mph_free", _i, [_vp]),
    ("bsdb_mph_build_index_passes_fixed", _i, [_vp, _vp, _u32, _u64, _u32, _vp, _u64, _u64, _vp, _vp, _i, _u32,
                                               C.c_char_p, C.c_char_p, C.POINTER(_vp), C.POINTER(_u32)]),
    ("bsdb_mph_build_index_passes_var", _i, [_vp, _vp, _vp, _u64, _u32, _vp, _u64, _u64, _vp, _vp, _i, _u32,
                                             C.c_char_p, C.c_char_p, C.POINTER(_vp), C.POINTER(_u32)]),
    ("bsdb_builder_open", _i, [_vp, _u32, _u64, _u64, _i, _u64, _u64, C.POINTER(_vp)]),
    ("bsdb_builder_add_fixed", _i, [_vp, _vp, _u32, _u64, _vp, _vp, _vp]),
    ("bsdb_builder_add_var", _i, [_vp, _vp, _vp, _u64, _vp, _vp, _vp]),
    ("bsdb_builder_count", _i, [_vp, C.POINTER(_u64)]),
    ("bsdb_builder_finish", _i, [_vp, _u32, _u32, C.c_char_p, C.c_char_p, C.POINTER(_vp), C.POINTER(_u32)]),
    ("bsdb_builder_free", _i, [_vp]),
    ("bsdb_index_open", _i, [_vp, _i, _u64, C.c_char_p, C.c_char_p, C.POINTER(_vp), C.POINTER(_u64)]),
    ("bsdb_index_begin_pass", _i, [_vp, _u64]),
    ("bsdb_index_put_var", _i, [_vp, _vp, _vp, _u64, _vp, _vp, _vp]),
    ("bsdb_index_put_fixed", _i, [_vp, _vp, _u32, _u64, _vp, _vp, _vp]),
    ("bsdb_index_end_pass", _i, [_vp]),
    ("bsdb_index_close", _i, [_vp]),
    ("bsdb_kv_scan", _i, [C.c_char_p, _i, _i, _u32, _i, C.POINTER(_vp)]),
    ("bsdb_kv_records_info", _i, [_vp, C.POINTER(_u64), C.POINTER(_u64), C.POINTER(_u32)]),
    ("bsdb_kv_records_arrays", _i, [_vp, C.POINTER(_vp), C.POINTER(_vp), C.POINTER(_vp), C.POINTER(_vp),
                                    C.POINTER(_vp)]),
    ("bsdb_kv_records_free", _i, [_vp]),
    ("bsdb_kv_build_index", _i, [_vp, C.c_char_p, _i, _i, _u32, _i, _u32, _i, C.c_char_p, C.c_char_p,
                                 C.POINTER(_vp)]),
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


def mph_sizes(n: int, width: int) -> dict:
    """bsdb_mph_sizes: the field sizes of an MPHF on n keys (no device needed)."""
    m, vw, vb, sw = C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_uint64()
    _check("bsdb_mph_sizes", lib().bsdb_mph_sizes(n, width, C.byref(m), C.byref(vw), C.byref(vb), C.byref(sw)))
    return {"num_buckets": m.value, "values_words": vw.value, "value_bits": vb.value, "sig_words": sw.value}


def range_windows(n_global: int, width: int, e_lo: int, n_local: int):
    """bsdb_gov_range_windows: (values_w0, values_words, sig_w0, sig_words), the
    words the keys [e_lo, e_lo + n_local) of a range build write (host only)."""
    out = (C.c_uint64 * 4)()
    _check("bsdb_gov_range_windows", lib().bsdb_gov_range_windows(n_global, width, e_lo, n_local, out))
    return tuple(int(x) for x in out)


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

    def set_pipeline(self, mode: int, chunks: int = 0, p2_cus: int = 0):
        """Pass 2 of chunk i beside pass 1 of chunk i + 1 (13-byte keys): -1 default, 0 off, 1 on."""
        _check("bsdb_set_pipeline", lib().bsdb_set_pipeline(self._h, mode, chunks, p2_cus))

    def set_chunk_keys(self, n: int):
        _check("bsdb_set_chunk_keys", lib().bsdb_set_chunk_keys(self._h, n))

    def fallback_count(self) -> int:
        """Chunks recounted by the overflow fallback since open (synchronises)."""
        v = C.c_uint64()
        _check("bsdb_fallback_count", lib().bsdb_fallback_count(self._h, C.byref(v)))
        return v.value

    def fused_status(self):
        """(single-pass launches since open, launches that timed out) -- synchronises."""
        a, b = C.c_uint64(), C.c_uint64()
        _check("bsdb_fused_status", lib().bsdb_fused_status(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

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
        m = num_buckets(n)
        E = torch.empty(m + 1, dtype=torch.int64, device=sig.device)
        values = torch.empty(int(lib().bsdb_values_words(n)), dtype=torch.int64, device=sig.device)
        sigbits = torch.empty((n * width + 63) // 64 + 1, dtype=torch.int64, device=sig.device) if width else None
        _check("bsdb_dev_gov_build", lib().bsdb_dev_gov_build(
            self._h, _ptr(sig), n, width, _ptr(E), _ptr(values), _ptr(sigbits) if sigbits is not None else None,
            _stream(stream)))
        return E, values, sigbits

    def gov_build_ranks(self, sig, width: int, stream=None):
        """F2: (E, values, sigbits, rank) -- rank[i] = getLong of sig[i], from the solve."""
        import torch
        n = sig.shape[0]
        m = num_buckets(n)
        E = torch.empty(m + 1, dtype=torch.int64, device=sig.device)
        values = torch.empty(int(lib().bsdb_values_words(n)), dtype=torch.int64, device=sig.device)
        sigbits = torch.empty((n * width + 63) // 64 + 1, dtype=torch.int64, device=sig.device) if width else None
        rank = torch.empty(max(n, 1), dtype=torch.int64, device=sig.device)[:n]
        _check("bsdb_dev_gov_build_ranks", lib().bsdb_dev_gov_build_ranks(
            self._h, _ptr(sig), n, width, _ptr(E), _ptr(values), _ptr(sigbits) if sigbits is not None else None,
            _ptr(rank), _stream(stream)))
        return E, values, sigbits, rank

    def gov_build_range(self, sig, n_global: int, b_lo: int, b_hi: int, e_lo: int, width: int, E, values, sigbits=None,
                        rank=None, stream=None):
        """E4: one rank's bucket range [b_lo, b_hi) into FULL-size zeroed arrays
        (rank: optional, the global rank of each local signature)."""
        _check("bsdb_dev_gov_build_range", lib().bsdb_dev_gov_build_range(
            self._h, _ptr(sig), sig.shape[0], n_global, b_lo, b_hi, e_lo, width, _ptr(E), _ptr(values),
            _ptr(sigbits) if sigbits is not None else None, _ptr(rank) if rank is not None else None, _stream(stream)))

    def gov_build_window(self, sig, n_global: int, b_lo: int, b_hi: int, e_lo: int, width: int, E_win, values_win,
                         values_w0: int, sigbits_win=None, sig_w0: int = 0, rank=None, stream=None):
        """E4 with O(n/G) memory: the range build into zeroed windows of the
        structure (E[b_lo..b_hi], value words from values_w0, checksum words
        from sig_w0; range_windows gives the words the range writes)."""
        assert E_win.numel() >= b_hi - b_lo + 1
        _check("bsdb_dev_gov_build_window", lib().bsdb_dev_gov_build_window(
            self._h, _ptr(sig), sig.shape[0], n_global, b_lo, b_hi, e_lo, width, _ptr(E_win), _ptr(values_win),
            values_w0, values_win.numel(), _ptr(sigbits_win) if sigbits_win is not None else None, sig_w0,
            sigbits_win.numel() if sigbits_win is not None else 0, _ptr(rank) if rank is not None else None,
            _stream(stream)))

    def mph_build_index_passes(self, keys, key_len: int, n: int, width: int, passes: int = 0, offsets=None,
                               addr=None, addr_base: int = 0, addr_stride: int = 0, index=None, stream=None):
        """The whole build from keys resident on the device by sequential
        bucket-range passes (fixed key_len, or a var-len blob with offsets).
        index: None (structure only), a device int64 tensor of n slots, or a
        host numpy uint64/int64 array of n slots (each pass's slice copied out
        while the next solves).  addr: device int64 tensor of n addresses, else
        addr_base + addr_stride * i.  Returns (E, values, sigbits, passes_used)."""
        import torch
        import numpy as np
        dev = keys.device
        m = num_buckets(n)
        E = torch.empty(m + 1, dtype=torch.int64, device=dev)
        values = torch.empty(int(lib().bsdb_values_words(n)), dtype=torch.int64, device=dev)
        sigbits = torch.empty((n * width + 63) // 64 + 1, dtype=torch.int64, device=dev) if width else None
        d_index = h_index = None
        if index is not None:
            if isinstance(index, np.ndarray):
                assert index.dtype.itemsize == 8 and index.size >= n and index.flags.c_contiguous
                h_index = index.ctypes.data
            else:
                assert index.dtype == torch.int64 and index.numel() >= n and index.device == dev
                d_index = _ptr(index)
        used = C.c_uint32()
        sb = _ptr(sigbits) if sigbits is not None else None
        ad = _ptr(addr) if addr is not None else None
        if offsets is None:
            _check("bsdb_dev_mph_build_index_passes_fixed", lib().bsdb_dev_mph_build_index_passes_fixed(
                self._h, _ptr(keys), key_len, n, width, passes, ad, addr_base, addr_stride, _ptr(E), _ptr(values), sb,
                d_index, h_index, C.byref(used), _stream(stream)))
        else:
            _check("bsdb_dev_mph_build_index_passes_var", lib().bsdb_dev_mph_build_index_passes_var(
                self._h, _ptr(keys), keys.numel(), _ptr(offsets), n, width, passes, ad, addr_base, addr_stride,
                _ptr(E), _ptr(values), sb, d_index, h_index, C.byref(used), _stream(stream)))
        return E, values, sigbits, used.value

    def partition_owners(self, sig, m: int, nranks: int, payload=None, stream=None):
        """Signatures (and one int64 payload per key) grouped by owning rank
        (bucket ranges); returns (sig_out, payload_out or None, counts)."""
        import torch
        import numpy as np
        n = sig.shape[0]
        out = torch.empty((max(n, 1), 2), dtype=torch.int64, device=sig.device)[:n]
        pout = torch.empty(max(n, 1), dtype=torch.int64, device=sig.device)[:n] if payload is not None else None
        counts = np.zeros(nranks, np.uint64)
        _check("bsdb_dev_partition_owners", lib().bsdb_dev_partition_owners(
            self._h, _ptr(sig), _ptr(payload) if payload is not None else None, n, m, nranks, _ptr(out),
            _ptr(pout) if pout is not None else None, counts.ctypes.data, _stream(stream)))
        return out, pout, [int(x) for x in counts]

    def release_workspace(self):
        _check("bsdb_release_workspace", lib().bsdb_release_workspace(self._h))

    def set_verify(self, on: bool):
        _check("bsdb_set_verify", lib().bsdb_set_verify(self._h, 1 if on else 0))

    # ---- B4: the histogram collective (RCCL) inside the library
    @staticmethod
    def comm_available() -> bool:
        return bool(lib().bsdb_comm_available())

    @staticmethod
    def comm_unique_id() -> bytes:
        buf = C.create_string_buffer(COMM_ID_BYTES)
        _check("bsdb_comm_unique_id", lib().bsdb_comm_unique_id(buf))
        return buf.raw

    def comm_init(self, nranks: int, rank: int, uid: bytes):
        buf = C.create_string_buffer(bytes(uid), COMM_ID_BYTES)
        _check("bsdb_comm_init", lib().bsdb_comm_init(self._h, nranks, rank, buf))

    def histogram_finalize(self, counts, n_total: int, out=None, stream=None):
        """All-reduce of the local counts over RCCL + scan -> E (every rank)."""
        import torch
        m = counts.numel()
        if out is None:
            out = torch.empty(m + 1, dtype=torch.int64, device=counts.device)
        _check("bsdb_dev_histogram_finalize", lib().bsdb_dev_histogram_finalize(
            self._h, _ptr(counts), m, n_total, _ptr(out), _stream(stream)))
        return out

    def allreduce_u64(self, buf, stream=None):
        _check("bsdb_dev_allreduce_u64", lib().bsdb_dev_allreduce_u64(self._h, _ptr(buf), buf.numel(), _stream(stream)))

    # ---- A14/A15/F4: a device-resident MPHF built from host keys
    def mph_build_fixed(self, keys_np, key_len: int, width: int) -> "Mph":
        import numpy as np
        keys_np = np.ascontiguousarray(keys_np, np.uint8)
        h = C.c_void_p()
        _check("bsdb_mph_build_fixed", lib().bsdb_mph_build_fixed(
            self._h, keys_np.ctypes.data, key_len, keys_np.size // key_len, width, C.byref(h)))
        return Mph(h, self)

    @staticmethod
    def _records_args(n, addr_np, value8_np, vlen_np, approximate):
        import numpy as np
        addr_np = np.ascontiguousarray(addr_np, np.uint64)
        if addr_np.size != n:
            raise ValueError("one address per key")
        v8 = vl = None
        if approximate:
            if value8_np is None or vlen_np is None:
                raise ValueError("approximate mode needs value8 and vlen")
            v8 = np.ascontiguousarray(value8_np, np.uint64)
            vl = np.ascontiguousarray(vlen_np, np.uint8)
            if v8.size != n or vl.size != n:
                raise ValueError("one value8/vlen per key")
        return addr_np, v8, vl

    def mph_build_index_fixed(self, keys_np, key_len: int, width: int, addr_np, index_path: str,
                              index_a_path: Optional[str] = None, approximate: bool = False, value8_np=None,
                              vlen_np=None) -> "Mph":
        """F2: MPHF + index.db (+ index_a.db) in one call from the solve's
        ranks (bsdb_mph_build_index_fixed), no rescan of the records."""
        import numpy as np
        keys_np = np.ascontiguousarray(keys_np, np.uint8)
        n = keys_np.size // key_len
        addr_np, v8, vl = self._records_args(n, addr_np, value8_np, vlen_np, approximate)
        h = C.c_void_p()
        _check("bsdb_mph_build_index_fixed", lib().bsdb_mph_build_index_fixed(
            self._h, keys_np.ctypes.data, key_len, n, width, addr_np.ctypes.data,
            v8.ctypes.data if v8 is not None else None, vl.ctypes.data if vl is not None else None,
            1 if approximate else 0, index_path.encode(), index_a_path.encode() if index_a_path else None,
            C.byref(h)))
        return Mph(h, self)

    def mph_build_index_passes_host(self, keys_np, key_len: int, width: int, index_path: str,
                                    index_a_path: Optional[str] = None, addr_np=None, addr_base: int = 0,
                                    addr_stride: int = 0, approximate: bool = False, value8_np=None, vlen_np=None,
                                    passes: int = 0, offsets_np=None):
        """F2 in bounded device memory from host records
        (bsdb_mph_build_index_passes_{fixed,var}): keys uploaded once, built by
        bucket-range passes, each pass's slots written at their file offset.
        key_len 0 with offsets_np: variable-length keys.  addr_np None:
        addresses addr_base + addr_stride * i.  Returns (Mph, passes_used)."""
        import numpy as np
        if offsets_np is not None:
            blob, off, n = self._var_host_args(keys_np, offsets_np)
        else:
            blob = np.ascontiguousarray(keys_np, np.uint8)
            n = blob.size // key_len
        if addr_np is not None:
            a, v8, vl = self._records_args(n, addr_np, value8_np, vlen_np, approximate)
        else:
            a = None
            _, v8, vl = self._records_args(n, np.zeros(n, np.uint64), value8_np, vlen_np, approximate)
        h = C.c_void_p()
        used = C.c_uint32()
        ip, ap = index_path.encode(), index_a_path.encode() if index_a_path else None
        if offsets_np is not None:
            _check("bsdb_mph_build_index_passes_var", lib().bsdb_mph_build_index_passes_var(
                self._h, blob.ctypes.data, off.ctypes.data, n, width, _np_ptr(a), addr_base, addr_stride, _np_ptr(v8),
                _np_ptr(vl), 1 if approximate else 0, passes, ip, ap, C.byref(h), C.byref(used)))
        else:
            _check("bsdb_mph_build_index_passes_fixed", lib().bsdb_mph_build_index_passes_fixed(
                self._h, blob.ctypes.data, key_len, n, width, _np_ptr(a), addr_base, addr_stride, _np_ptr(v8),
                _np_ptr(vl), 1 if approximate else 0, passes, ip, ap, C.byref(h), C.byref(used)))
        return Mph(h, self), used.value

    def builder(self, key_len: int = 0, key_capacity: int = 0, blob_capacity: int = 0, approximate: bool = False,
                addr_base: int = 0, addr_stride: int = 0) -> "Builder":
        """A streaming builder (bsdb_builder_*): keys added in batches into
        HBM, then one bucket-range-pass build into the index files."""
        return Builder(self, key_len, key_capacity, blob_capacity, approximate, addr_base, addr_stride)

    def kv_build_index(self, kv_base: str, partitions: int, width: int, index_path: str,
                       index_a_path: Optional[str] = None, approximate: bool = False, fmt: int = 0,
                       block_size: int = 4096, threads: int = 0) -> "Mph":
        """W:91-155 from the data files: native kv.db scan + the one-call build."""
        h = C.c_void_p()
        _check("bsdb_kv_build_index", lib().bsdb_kv_build_index(
            self._h, kv_base.encode(), partitions, fmt, block_size, threads, width, 1 if approximate else 0,
            index_path.encode(), index_a_path.encode() if index_a_path else None, C.byref(h)))
        return Mph(h, self)

    def mph_build_index_var(self, blob_np, off_np, width: int, addr_np, index_path: str,
                            index_a_path: Optional[str] = None, approximate: bool = False, value8_np=None,
                            vlen_np=None) -> "Mph":
        blob_np, off_np, n = self._var_host_args(blob_np, off_np)
        addr_np, v8, vl = self._records_args(n, addr_np, value8_np, vlen_np, approximate)
        h = C.c_void_p()
        _check("bsdb_mph_build_index_var", lib().bsdb_mph_build_index_var(
            self._h, blob_np.ctypes.data, off_np.ctypes.data, n, width, addr_np.ctypes.data,
            v8.ctypes.data if v8 is not None else None, vl.ctypes.data if vl is not None else None,
            1 if approximate else 0, index_path.encode(), index_a_path.encode() if index_a_path else None,
            C.byref(h)))
        return Mph(h, self)

    def mph_build_var(self, blob_np, off_np, width: int) -> "Mph":
        blob_np, off_np, n = self._var_host_args(blob_np, off_np)
        h = C.c_void_p()
        _check("bsdb_mph_build_var", lib().bsdb_mph_build_var(
            self._h, blob_np.ctypes.data, off_np.ctypes.data, n, width, C.byref(h)))
        return Mph(h, self)

    def mph_import(self, n: int, width: int, E, values, sigbits=None) -> "Mph":
        import numpy as np
        E = np.ascontiguousarray(E, np.uint64)
        values = np.ascontiguousarray(values, np.uint64)
        sb = np.ascontiguousarray(sigbits, np.uint64) if sigbits is not None else None
        h = C.c_void_p()
        _check("bsdb_mph_import", lib().bsdb_mph_import(
            self._h, n, width, E.ctypes.data, values.ctypes.data, sb.ctypes.data if sb is not None else None,
            C.byref(h)))
        return Mph(h, self)

    def mph_load(self, path: str) -> "Mph":
        h = C.c_void_p()
        _check("bsdb_mph_load", lib().bsdb_mph_load(self._h, path.encode(), C.byref(h)))
        return Mph(h, self)

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
        """13*n key bytes (a view of a 16-B-padded allocation when `out` is
        None, so keys.numel() // 13 == n)."""
        import torch
        if out is None:
            out = torch.empty(13 * n + 16, dtype=torch.uint8, device=f"cuda:{self.device}")[: 13 * n]
        elif out.numel() < 13 * n:
            raise ValueError("out holds fewer than 13*n bytes")
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


class Mph:
    """A GOV MPHF resident on one device (``bsdb_mph``)."""

    def __init__(self, h, ctx: Context):
        self._h = h
        self.ctx = ctx  # keeps the context alive

    def close(self):
        if self._h:
            _check("bsdb_mph_free", lib().bsdb_mph_free(self._h))
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

    def info(self):
        n, m, vw, sw = C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_uint64()
        w = C.c_uint32()
        _check("bsdb_mph_info", lib().bsdb_mph_info(self._h, C.byref(n), C.byref(m), C.byref(w), C.byref(vw),
                                                    C.byref(sw)))
        return {"n": n.value, "num_buckets": m.value, "width": w.value, "values_words": vw.value,
                "sig_words": sw.value}

    def export(self):
        """(E u64[m+1], values u64[], sigbits u64[] or None) -- the fields of
        GOVMinimalPerfectHashFunctionModified (GOV:284-313)."""
        import numpy as np
        i = self.info()
        E = np.zeros(i["num_buckets"] + 1, np.uint64)
        vals = np.zeros(i["values_words"], np.uint64)
        sb = np.zeros(i["sig_words"], np.uint64) if i["width"] else None
        _check("bsdb_mph_export", lib().bsdb_mph_export(self._h, E.ctypes.data, vals.ctypes.data,
                                                        sb.ctypes.data if sb is not None else None))
        return E, vals, sb

    def dump(self, path: str):
        _check("bsdb_mph_dump", lib().bsdb_mph_dump(self._h, path.encode()))

    def lookup_fixed(self, keys_np, key_len: int, check: bool = True):
        import numpy as np
        keys_np = np.ascontiguousarray(keys_np, np.uint8)
        n = keys_np.size // key_len
        out = np.zeros(max(n, 1), np.int64)
        _check("bsdb_mph_lookup_fixed", lib().bsdb_mph_lookup_fixed(
            self._h, keys_np.ctypes.data, key_len, n, 1 if check else 0, out.ctypes.data))
        return out[:n]

    def lookup_var(self, blob_np, off_np, check: bool = True):
        import numpy as np
        blob_np, off_np, n = Context._var_host_args(blob_np, off_np)
        out = np.zeros(max(n, 1), np.int64)
        _check("bsdb_mph_lookup_var", lib().bsdb_mph_lookup_var(
            self._h, blob_np.ctypes.data, off_np.ctypes.data, n, 1 if check else 0, out.ctypes.data))
        return out[:n]

    def write_index(self, index_path: str, index_a_path: Optional[str], approximate: bool, pass_cache_bytes: int,
                    feed):
        """BSDBWriter.buildIndex (W:107-155): for every pass, ``feed(put)``
        must call ``put(keys..., addr, value8, vlen)`` for every record (the
        kv.db scan).  Returns the number of passes."""
        return IndexWriter(self, index_path, index_a_path, approximate, pass_cache_bytes).run(feed)


class Builder:
    """``bsdb_builder``: BSDBWriter.put's key stream into one device's HBM,
    then the whole build by bucket-range passes (``finish``)."""

    def __init__(self, ctx: Context, key_len: int, key_capacity: int, blob_capacity: int, approximate: bool,
                 addr_base: int, addr_stride: int):
        self.ctx = ctx
        self.approx = approximate
        self._h = C.c_void_p()
        _check("bsdb_builder_open", lib().bsdb_builder_open(ctx._h, key_len, key_capacity, blob_capacity,
                                                            1 if approximate else 0, addr_base, addr_stride,
                                                            C.byref(self._h)))

    def close(self):
        if self._h:
            _check("bsdb_builder_free", lib().bsdb_builder_free(self._h))
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

    def count(self) -> int:
        n = C.c_uint64()
        _check("bsdb_builder_count", lib().bsdb_builder_count(self._h, C.byref(n)))
        return n.value

    def add_fixed(self, keys_np, key_len: int, addr_np=None, value8_np=None, vlen_np=None):
        import numpy as np
        keys_np = np.ascontiguousarray(keys_np, np.uint8)
        n = keys_np.size // key_len
        a = np.ascontiguousarray(addr_np, np.uint64) if addr_np is not None else None
        v8 = np.ascontiguousarray(value8_np, np.uint64) if value8_np is not None else None
        vl = np.ascontiguousarray(vlen_np, np.uint8) if vlen_np is not None else None
        _check("bsdb_builder_add_fixed", lib().bsdb_builder_add_fixed(
            self._h, keys_np.ctypes.data, key_len, n, _np_ptr(a), _np_ptr(v8), _np_ptr(vl)))

    def add_var(self, blob_np, off_np, addr_np=None, value8_np=None, vlen_np=None):
        import numpy as np
        blob_np, off_np, n = Context._var_host_args(blob_np, off_np)
        a = np.ascontiguousarray(addr_np, np.uint64) if addr_np is not None else None
        v8 = np.ascontiguousarray(value8_np, np.uint64) if value8_np is not None else None
        vl = np.ascontiguousarray(vlen_np, np.uint8) if vlen_np is not None else None
        _check("bsdb_builder_add_var", lib().bsdb_builder_add_var(
            self._h, blob_np.ctypes.data, off_np.ctypes.data, n, _np_ptr(a), _np_ptr(v8), _np_ptr(vl)))

    def finish(self, width: int, index_path: Optional[str] = None, index_a_path: Optional[str] = None,
               passes: int = 0):
        """Builds everything added; returns (Mph, passes_used)."""
        h = C.c_void_p()
        used = C.c_uint32()
        _check("bsdb_builder_finish", lib().bsdb_builder_finish(
            self._h, width, passes, index_path.encode() if index_path else None,
            index_a_path.encode() if index_a_path else None, C.byref(h), C.byref(used)))
        return Mph(h, self.ctx), used.value


class IndexWriter:
    """``bsdb_index``: index.db / index_a.db of BSDBWriter.buildIndex."""

    def __init__(self, mph: Mph, index_path: str, index_a_path: Optional[str], approximate: bool,
                 pass_cache_bytes: int):
        self.mph = mph
        self.approx = approximate
        self._h = C.c_void_p()
        p = C.c_uint64()
        _check("bsdb_index_open", lib().bsdb_index_open(
            mph._h, 1 if approximate else 0, pass_cache_bytes, index_path.encode(),
            index_a_path.encode() if index_a_path else None, C.byref(self._h), C.byref(p)))
        self.passes = p.value

    def begin_pass(self, i: int):
        _check("bsdb_index_begin_pass", lib().bsdb_index_begin_pass(self._h, i))

    def end_pass(self):
        _check("bsdb_index_end_pass", lib().bsdb_index_end_pass(self._h))

    def put_fixed(self, keys_np, key_len: int, addr_np, value8_np=None, vlen_np=None):
        import numpy as np
        keys_np = np.ascontiguousarray(keys_np, np.uint8)
        addr_np = np.ascontiguousarray(addr_np, np.uint64)
        v8 = np.ascontiguousarray(value8_np, np.uint64) if value8_np is not None else None
        vl = np.ascontiguousarray(vlen_np, np.uint8) if vlen_np is not None else None
        _check("bsdb_index_put_fixed", lib().bsdb_index_put_fixed(
            self._h, keys_np.ctypes.data, key_len, addr_np.size, addr_np.ctypes.data,
            v8.ctypes.data if v8 is not None else None, vl.ctypes.data if vl is not None else None))

    def put_var(self, blob_np, off_np, addr_np, value8_np=None, vlen_np=None):
        import numpy as np
        blob_np, off_np, n = Context._var_host_args(blob_np, off_np)
        addr_np = np.ascontiguousarray(addr_np, np.uint64)
        v8 = np.ascontiguousarray(value8_np, np.uint64) if value8_np is not None else None
        vl = np.ascontiguousarray(vlen_np, np.uint8) if vlen_np is not None else None
        _check("bsdb_index_put_var", lib().bsdb_index_put_var(
            self._h, blob_np.ctypes.data, off_np.ctypes.data, n, addr_np.ctypes.data,
            v8.ctypes.data if v8 is not None else None, vl.ctypes.data if vl is not None else None))

    def close(self):
        if self._h:
            rc = lib().bsdb_index_close(self._h)
            self._h = C.c_void_p()
            _check("bsdb_index_close", rc)

    def run(self, feed):
        try:
            for i in range(self.passes):
                self.begin_pass(i)
                feed(self)
                self.end_pass()
        finally:
            self.close()
        return self.passes


class Multi:
    """``bsdb_multi``: every listed device of this process + one RCCL communicator."""

    def __init__(self, ndev: int, devices=None):
        self._h = C.c_void_p()
        arr = (C.c_int * ndev)(*devices) if devices is not None else None
        _check("bsdb_multi_open", lib().bsdb_multi_open(ndev, arr, C.byref(self._h)))

    def close(self):
        if self._h:
            _check("bsdb_multi_close", lib().bsdb_multi_close(self._h))
            self._h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def size(self) -> int:
        return int(lib().bsdb_multi_size(self._h))

    def histogram_fixed(self, keys_np, key_len: int, seed: int = 0):
        """E[0..m] of host keys sharded over the devices (one all-reduce)."""
        import numpy as np
        keys_np = np.ascontiguousarray(keys_np, np.uint8)
        n = keys_np.size // key_len
        E = np.zeros(num_buckets(n) + 1, np.uint64)
        _check("bsdb_multi_histogram_fixed", lib().bsdb_multi_histogram_fixed(
            self._h, keys_np.ctypes.data, key_len, n, seed & (2**64 - 1), E.ctypes.data))
        return E

    def histogram_var(self, blob_np, off_np, seed: int = 0):
        import numpy as np
        blob_np, off_np, n = Context._var_host_args(blob_np, off_np)
        E = np.zeros(num_buckets(n) + 1, np.uint64)
        _check("bsdb_multi_histogram_var", lib().bsdb_multi_histogram_var(
            self._h, blob_np.ctypes.data, off_np.ctypes.data, n, seed & (2**64 - 1), E.ctypes.data))
        return E

    def _build_outputs(self, n: int, width: int):
        import numpy as np
        E = np.zeros(num_buckets(n) + 1, np.uint64)
        vals = np.zeros(int(lib().bsdb_values_words(n)), np.uint64)
        sb = np.zeros((n * width + 63) // 64 + 1, np.uint64) if width else None
        return E, vals, sb

    def mph_build_index_fixed(self, keys_np, key_len: int, width: int, addr_np=None, index_path: Optional[str] = None,
                              index_a_path: Optional[str] = None, approximate: bool = False, value8_np=None,
                              vlen_np=None):
        """E4 over this process's devices (bsdb_multi_mph_build_index_fixed):
        the structure's fields (E, values, sigbits) as host arrays -- the same
        as Mph.export() of a one-device build -- and, with index_path, the
        index files written by every device at its slice's offset."""
        import numpy as np
        keys_np = np.ascontiguousarray(keys_np, np.uint8)
        n = keys_np.size // key_len
        addr_np, v8, vl = (Context._records_args(n, addr_np, value8_np, vlen_np, approximate) if index_path
                           else (None, None, None))
        E, vals, sb = self._build_outputs(n, width)
        _check("bsdb_multi_mph_build_index_fixed", lib().bsdb_multi_mph_build_index_fixed(
            self._h, keys_np.ctypes.data, key_len, n, width, _np_ptr(addr_np), _np_ptr(v8), _np_ptr(vl),
            1 if approximate else 0, index_path.encode() if index_path else None,
            index_a_path.encode() if index_a_path else None, E.ctypes.data, vals.ctypes.data, _np_ptr(sb)))
        return E, vals, sb

    def mph_build_index_var(self, blob_np, off_np, width: int, addr_np=None, index_path: Optional[str] = None,
                            index_a_path: Optional[str] = None, approximate: bool = False, value8_np=None,
                            vlen_np=None):
        blob_np, off_np, n = Context._var_host_args(blob_np, off_np)
        addr_np, v8, vl = (Context._records_args(n, addr_np, value8_np, vlen_np, approximate) if index_path
                           else (None, None, None))
        E, vals, sb = self._build_outputs(n, width)
        _check("bsdb_multi_mph_build_index_var", lib().bsdb_multi_mph_build_index_var(
            self._h, blob_np.ctypes.data, off_np.ctypes.data, n, width, _np_ptr(addr_np), _np_ptr(v8), _np_ptr(vl),
            1 if approximate else 0, index_path.encode() if index_path else None,
            index_a_path.encode() if index_a_path else None, E.ctypes.data, vals.ctypes.data, _np_ptr(sb)))
        return E, vals, sb


def kv_scan(kv_base: str, partitions: int, fmt: int = 0, block_size: int = 4096, threads: int = 0) -> dict:
    """The native kv.db scan (bsdb_kv_scan): dict of numpy copies -- blob,
    offsets, addr, value8, vlen, fixed_len.  Host only (no device needed)."""
    import numpy as np
    h = C.c_void_p()
    _check("bsdb_kv_scan", lib().bsdb_kv_scan(kv_base.encode(), partitions, fmt, block_size, threads, C.byref(h)))
    try:
        n, nb, fl = C.c_uint64(), C.c_uint64(), C.c_uint32()
        _check("bsdb_kv_records_info", lib().bsdb_kv_records_info(h, C.byref(n), C.byref(nb), C.byref(fl)))
        ptrs = [C.c_void_p() for _ in range(5)]
        _check("bsdb_kv_records_arrays", lib().bsdb_kv_records_arrays(h, *[C.byref(q) for q in ptrs]))

        def arr(q, count, dt):
            if count == 0 or not q.value:
                return np.zeros(0, dt)
            return np.ctypeslib.as_array(C.cast(q, C.POINTER(np.ctypeslib.as_ctypes_type(dt))),
                                         shape=(count,)).copy()
        N = n.value
        return {"blob": arr(ptrs[0], nb.value, np.uint8), "offsets": arr(ptrs[1], N + 1, np.uint64),
                "addr": arr(ptrs[2], N, np.uint64), "value8": arr(ptrs[3], N, np.uint64),
                "vlen": arr(ptrs[4], N, np.uint8), "fixed_len": fl.value}
    finally:
        lib().bsdb_kv_records_free(h)


def _np_ptr(a):
    return a.ctypes.data if a is not None else None
