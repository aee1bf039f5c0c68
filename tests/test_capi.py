"""The C ABI library builds, loads without a GPU and exports exactly what
include/bsdb_mi355x.h declares (no compute calls here)."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "bsdb_amd", "libbsdb_mi355x.so")
HDR = os.path.join(ROOT, "include", "bsdb_mi355x.h")


def declared():
    txt = open(HDR).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(bsdb_\w+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} not built: run __graft_entry__.build()")
    return C.CDLL(LIB)


def test_every_declared_symbol_exported(lib):
    names = declared()
    assert len(names) >= 14
    for n in names:
        assert hasattr(lib, n), n


def test_only_bsdb_symbols_exported():
    out = os.popen(f"nm -D --defined-only {LIB}").read().split("\n")
    syms = [l.split()[-1] for l in out if " T " in l]
    assert syms and all(s.startswith("bsdb_") for s in syms), syms


def test_python_binding_covers_header():
    import bsdb_amd.native as N
    assert sorted(n for n, _, _ in N.SIGNATURES) == declared()


def test_host_only_calls(lib):
    lib.bsdb_num_buckets.restype = C.c_uint64
    lib.bsdb_num_buckets.argtypes = [C.c_uint64]
    assert lib.bsdb_num_buckets(13_193_787_549) == 8_795_859
    assert lib.bsdb_num_buckets(0) == 1
    assert lib.bsdb_abi_version() == 1
    lib.bsdb_strerror.restype = C.c_char_p
    assert lib.bsdb_strerror(-17) == b"duplicate key signature"
    lib.bsdb_open.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    assert lib.bsdb_open(0, None) == -22
