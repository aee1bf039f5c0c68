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
    assert lib.bsdb_abi_version() == 6
    hdr = open(os.path.join(ROOT, "include", "bsdb_mi355x.h")).read()
    assert f"#define BSDB_ABI_VERSION {lib.bsdb_abi_version()}" in hdr

    lib.bsdb_strerror.restype = C.c_char_p
    assert lib.bsdb_strerror(-17) == b"duplicate key signature"
    lib.bsdb_open.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    assert lib.bsdb_open(0, None) == -22


@pytest.mark.parametrize("n", [0, 1, 1_499, 1_500, 1_000_000, 13_193_787_549])
@pytest.mark.parametrize("width", [0, 4, 16, 64])
def test_mph_sizes_equal_gov_field_arithmetic(n, width):
    """the sizes a JVM allocates for the export (and that
    bsdb_mph_info reports for a built MPHF) are GOV's own field arithmetic:
    numBuckets = n/1500 + 1 (GOV:350) with edgeOffsetAndSeed of numBuckets + 1
    longs (GOV:355); the 2-bit value vector holds one value per vertex,
    vertexOffset(n) = n*C_TIMES_256 >> 8 with C_TIMES_256 = floor(1.10*256) =
    281 (GOV:160-162,315-317), plus the trailing 0 of values.add(0) (GOV:484);
    the checksums are n width-bit entries (GOV:493-494)."""
    from bsdb_amd.native import mph_sizes
    s = mph_sizes(n, width)
    C_TIMES_256 = int(1.10 * 256)
    assert C_TIMES_256 == 281
    buckets = n // 1500 + 1
    vertices = n * C_TIMES_256 >> 8
    value_bits = 2 * (vertices + 1)
    assert s["num_buckets"] == buckets
    assert s["value_bits"] == value_bits
    assert s["values_words"] == -(-value_bits // 64)
    assert s["sig_words"] == (0 if width == 0 else -(-(n * width) // 64) + 1)  # (+1: a zero word of slack)
    if n == 13_193_787_549:
        assert buckets == 8_795_859


def test_mph_sizes_rejects_what_gov_rejects():
    from bsdb_amd.native import BsdbError, mph_sizes
    with pytest.raises(BsdbError):
        mph_sizes(10, 65)
    with pytest.raises(BsdbError):  # GOV:348: at most (2^31 - 2) * 1500 - 1 keys
        mph_sizes((0x7FFFFFFF) * 1500, 4)


def test_var_host_argument_checks():
    """The host var-len wrappers validate offsets before any device call."""
    import numpy as np
    from bsdb_amd.native import Context
    blob = np.arange(10, dtype=np.uint8)
    ok = np.array([0, 3, 3, 10], np.uint64)
    b, o, n = Context._var_host_args(blob, ok)
    assert n == 3 and o.dtype == np.uint64 and b.dtype == np.uint8
    for bad in (np.array([0, 4, 3], np.uint64),      # decreasing
                np.array([0, 11], np.uint64),        # past the blob
                np.zeros((2, 2), np.uint64),         # not 1-D
                np.zeros(0, np.uint64)):             # no n+1 entries
        with pytest.raises(ValueError):
            Context._var_host_args(blob, bad)


def test_graft_entry_build_checks_the_header_abi():
    # __graft_entry__.build() compares the library's ABI with the header's
    # (a hard-coded number there once went stale and failed the build check)
    src = open(os.path.join(ROOT, "__graft_entry__.py")).read()
    assert "bsdb_abi_version() ==" in src and "BSDB_ABI_VERSION" in src
