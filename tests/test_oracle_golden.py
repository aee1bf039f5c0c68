"""The CPU oracle against the reference's own C (golden vectors from
oracle/_ref = /root/reference/src/main/c/{spooky,mph}.c, see
tests/golden/make_golden.py).  Pins the checker before it checks the GPU."""
import ctypes as C

import numpy as np
import pytest

import oracle as O


def test_spooky_every_length_and_seed(golden):
    msg = golden["len_msg"].tobytes()
    for si, seed in enumerate(golden["len_seeds"]):
        for L in range(201):
            assert O.spooky_short(msg[:L], int(seed)) == tuple(int(x) for x in golden["len_sig"][si, L]), (seed, L)


def test_survey_known_answers():
    # SURVEY.md §8(c) C2 probe values of the reference C (seed 0)
    assert O.spooky_short(b"0")[:2] == (0x38c8c677ac681de3, 0x849781d69ea102eb)
    assert O.spooky_short(b"999999")[:2] == (0xc2788dc9159b2bbd, 0xe4fb169c0c958e58)
    assert O.spooky_short(b"abcdefghijklm")[:2] == (0x025fe6827d2a4fa1, 0x95eb248b5b184313)
    assert O.spooky_short(b"0123456789abcdef0123456789abcdef0")[:2] == (0x81495b9d533be272, 0xd4d03cae4087936f)
    assert O.spooky_rehash(0x0123456789abcdef, 0xfedcba9876543210, 0)[:3] == (
        0x97f8058a72de6c95, 0x9152e6ca14331ec7, 0x6933b1b768f78949)


def _ascii(lo, hi):
    keys = [str(i).encode() for i in range(lo, hi)]
    off = np.zeros(len(keys) + 1, np.uint64)
    off[1:] = np.cumsum([len(k) for k in keys])
    return np.frombuffer(b"".join(keys), np.uint8), off


def test_native_test_keys(golden):
    blob, off = _ascii(0, 1_000_000)
    sig = O.hash_var(blob, off)
    idx = golden["native_sample_idx"]
    np.testing.assert_array_equal(sig[idx], golden["native_sample_sig"])
    assert np.bitwise_xor.reduce(sig[:, 0]) == golden["native_xor_sig0"]
    assert np.bitwise_xor.reduce(sig[:, 1]) == golden["native_xor_sig1"]
    m = O.num_buckets(1_000_000)
    np.testing.assert_array_equal(O.histogram_var(blob, off, m), golden["native_counts"])


def test_writer_test_keys_histogram(golden):
    blob, off = _ascii(1, 200_001)
    m = O.num_buckets(200_000)
    np.testing.assert_array_equal(O.histogram_var(blob, off, m), golden["writer_counts"])


def test_k13_generator_and_hash(golden):
    keys = O.gen_keys13(0, 1_000_000)
    np.testing.assert_array_equal(keys[: 16 * 13].reshape(16, 13), golden["k13_head"])
    np.testing.assert_array_equal(O.hash_fixed(keys[: 8192 * 13], 13), golden["k13_sig"])
    m = O.num_buckets(1_000_000)
    np.testing.assert_array_equal(O.histogram_fixed(keys, 13, m), golden["k13_counts"])
    counts, _ = O.histogram_fixed_mt(keys, 13, m, threads=4)
    np.testing.assert_array_equal(counts, golden["k13_counts"])
    counts, _ = O.histogram_gen13_mt(0, 1_000_000, m, threads=3)
    np.testing.assert_array_equal(counts, golden["k13_counts"])


def test_var_len_keys(golden):
    np.testing.assert_array_equal(O.hash_var(golden["var_blob"], golden["var_off"]), golden["var_sig"])


def test_rehash(golden):
    for (a, b), s, out in zip(golden["rehash_in"], golden["rehash_seed"], golden["rehash_out"]):
        assert O.spooky_rehash(int(a), int(b), int(s)) == tuple(int(x) for x in out)


def test_edge_offsets(golden):
    c = golden["native_counts"]
    E = O.edge_offsets(c)
    assert E[0] == 0 and E[-1] == 1_000_000
    np.testing.assert_array_equal(np.diff(E.astype(np.int64)), c.astype(np.int64))


@pytest.mark.parametrize("name", ["lk_ascii", "lk_k13"])
def test_lookup_arithmetic(golden, name):
    blob, off = golden[name + "_blob"], golden[name + "_off"]
    E, arr, res = golden[name + "_E"], golden[name + "_array"], golden[name + "_res"]
    n = off.size - 1
    lm = E.size - 1
    mp = O.BoMph(n, 2 * lm, 0, lm, E.ctypes.data_as(C.POINTER(C.c_uint64)),
                 arr.ctypes.data_as(C.POINTER(C.c_uint64)), 0, None)
    sig = O.hash_var(blob, off)
    got = np.array([O.lib().bo_lookup_nocheck(C.byref(mp), s.ctypes.data_as(C.POINTER(C.c_uint64)))
                    for s in np.ascontiguousarray(sig)], np.int64)
    np.testing.assert_array_equal(got, res)


def parse_dump(data: bytes):
    """GOV.dump's raw layout (GOV:592-619 / mph.c:28-43): n, multiplier,
    globalSeed, len(E), E[], len(array), array[] (native-endian u64)."""
    w = np.frombuffer(data, "<u8")
    n, mult, seed, ne = (int(x) for x in w[:4])
    E = w[4: 4 + ne].copy()
    na = int(w[4 + ne])
    arr = w[5 + ne: 5 + ne + na].copy()
    assert 5 + ne + na == w.size
    return n, mult, seed, E, arr


def test_dump_fixture_oracle_equals_reference_load_mph(dump_golden):
    """A15: the committed GOV.dump file as the reference's load_mph +
    mph_get_byte_array read it (tests/golden/make_golden_dump.py); the oracle's
    reading of the same bytes gives the same ranks."""
    n, mult, seed, E, arr = parse_dump(dump_golden["dump"].tobytes())
    assert n == 30_000 and mult == 2 * (E.size - 1) and seed == 0 and E[-1] & ((1 << 56) - 1) == n
    sig = O.hash_var(dump_golden["blob"], dump_golden["off"])
    got = O.lookup_batch(sig, n, E, arr, 0, None, check=False)
    np.testing.assert_array_equal(got, dump_golden["ref_rank"])
    assert np.array_equal(np.sort(got), np.arange(n))


def test_bucket_map_edges():
    m = 8_795_859
    assert O.bucket(0, m) == 0
    assert O.bucket(2**64 - 1, m) == m - 1
    for s in [1 << 63, (1 << 63) - 1, 12345678901234567]:
        assert O.bucket(s, m) == ((s >> 1) * (2 * m)) >> 64


def test_against_reference_library_directly():
    R = O.ref_lib()
    if R is None:
        pytest.skip("oracle/_ref not built (reference sources absent)")
    rng = np.random.default_rng(7)
    for L in list(range(0, 100)) + [127, 128, 200, 255]:
        for _ in range(3):
            k = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
            seed = int(rng.integers(0, 2**63))
            out = (C.c_uint64 * 4)()
            R.spooky_short(C.create_string_buffer(k, L + 1), L, seed, out)
            assert O.spooky_short(k, seed) == tuple(out)
