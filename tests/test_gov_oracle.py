"""The oracle's GOV build (A5/A8/A11) is a valid MPHF under the REFERENCE's
own lookup (oracle/_ref: src/main/c/mph.c mph_get_byte_array): a bijection
onto [0, n); its checked lookup rejects absent keys at ~2^-width.  The
solver's specific solution is parity-unpinned (sux4j 5.4.1 absent)."""
import ctypes as C

import numpy as np
import pytest

import oracle as O


def ascii_set(lo, hi):
    keys = [str(i).encode() for i in range(lo, hi)]
    off = np.zeros(len(keys) + 1, np.uint64)
    off[1:] = np.cumsum([len(k) for k in keys])
    return keys, np.frombuffer(b"".join(keys), np.uint8), off


@pytest.mark.parametrize("n,width", [(1, 4), (2, 0), (1499, 4), (1500, 4), (30_000, 12)])
def test_gov_build_valid_under_reference_lookup(n, width):
    keys, blob, off = ascii_set(0, n)
    sig = O.hash_var(blob, off)
    rc, E, values, sigbits = O.gov_build(sig, width)
    assert rc == 0
    m = O.num_buckets(n)
    assert int(E[-1]) & ((1 << 56) - 1) == n
    ranks = O.lookup_batch(sig, n, E, values, width, sigbits, check=True)
    assert np.array_equal(np.sort(ranks), np.arange(n))
    R = O.ref_lib()
    if R is not None:
        mp = O.RefMph(n, 2 * m, 0, m + 1, E.ctypes.data_as(C.POINTER(C.c_uint64)), values.size,
                      values.ctypes.data_as(C.POINTER(C.c_uint64)))
        ref = np.array([R.mph_get_byte_array(C.byref(mp), k, len(k)) for k in keys])
        np.testing.assert_array_equal(ref, ranks)


def test_duplicate_keys_rejected():
    keys, blob, off = ascii_set(0, 100)
    sig = O.hash_var(blob, off)
    sig = np.concatenate([sig, sig[7:8]])
    rc, *_ = O.gov_build(sig, 4)
    assert rc == -1  # CBHS:969-972 DuplicateException -> build failure


def test_checksum_false_positive_rate():
    keys, blob, off = ascii_set(0, 20_000)
    sig = O.hash_var(blob, off)
    rc, E, values, sigbits = O.gov_build(sig, 8)
    assert rc == 0
    _, blob2, off2 = ascii_set(10**9, 10**9 + 100_000)
    miss = O.lookup_batch(O.hash_var(blob2, off2), 20_000, E, values, 8, sigbits, check=True)
    fp = float((miss >= 0).mean())
    assert 0.5 / 256 < fp < 2.0 / 256  # README.md:273-279: 2^-cb


def test_small_sets_all_sizes():
    for n in list(range(1, 40)) + [777, 1501]:
        keys = [("k%d" % i).encode() for i in range(n)]
        off = np.zeros(n + 1, np.uint64)
        off[1:] = np.cumsum([len(k) for k in keys])
        sig = O.hash_var(np.frombuffer(b"".join(keys), np.uint8), off)
        rc, E, values, sigbits = O.gov_build(sig, 4)
        assert rc == 0, n
        r = O.lookup_batch(sig, n, E, values, 4, sigbits)
        assert np.array_equal(np.sort(r), np.arange(n)), n


def test_seed_rule_retries_only_unsolvable_systems():
    """GOV:425-432: the local seed moves on only when the bucket's system has
    no solution (unorientable core, or an inconsistent block: sux4j's
    unorientable / unsolvable counters, GOV:427-428).  A singular but
    consistent block is solved (free columns 0), so such blocks occur among
    the solved attempts, and fewer seeds are tried per bucket than under a
    "fail on singular" rule (2.4 per bucket)."""
    n = 600_000
    keys = O.gen_keys13(77, n)
    sig = O.hash_fixed(keys, 13)
    O.solve_stats(reset=True)
    rc, E, values, sigbits = O.gov_build(sig, 4)
    st = O.solve_stats(reset=True)
    assert rc == 0
    m = O.num_buckets(n)
    assert st["singular_solved"] > 0 and st["inconsistent"] > 0
    fails = st["unorientable"] + st["inconsistent"] + st["degenerate"]
    assert st["attempts"] == m + fails  # every bucket ends on its first solvable seed
    assert st["attempts"] / m < 2.1
    r = O.lookup_batch(sig, n, E, values, 4, sigbits)
    assert np.array_equal(np.sort(r), np.arange(n))
    # the local seed in E's top 8 bits is the number of failed attempts of the bucket
    seeds = (E[:-1] >> np.uint64(56)).astype(np.int64)
    assert int(seeds.sum()) == fails
