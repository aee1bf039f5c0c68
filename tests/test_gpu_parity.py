"""GPU parity: the gfx950 kernels, called through the C ABI, against the CPU
oracle (itself pinned to the reference C by tests/test_oracle_golden.py).
Integer/byte work: every comparison is bit-exact."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from bsdb_amd import Context
    c = Context(0)
    yield c
    c.close()


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def u64(t):
    return t.cpu().numpy().view(np.uint64)


def rand_keys(n, L, seed=1):
    return np.random.default_rng(seed).integers(0, 256, n * L, dtype=np.uint8)


@pytest.mark.parametrize("L", [1, 2, 7, 8, 9, 12, 13, 14, 15, 16, 17, 26, 27, 31, 32, 33, 47, 52, 53, 64, 100, 255])
def test_hash_fixed_lengths(ctx, L):
    n = 20_001  # ragged: 2 full tiles + a partial one
    keys = rand_keys(n, L, L)
    got = u64(ctx.hash_fixed(dev(keys), L, seed=0))
    np.testing.assert_array_equal(got, O.hash_fixed(keys, L))


def test_hash_fixed_seed(ctx):
    keys = rand_keys(10_000, 13)
    for seed in (0x0123456789ABCDEF, 1 << 63):
        np.testing.assert_array_equal(u64(ctx.hash_fixed(dev(keys), 13, seed=seed)), O.hash_fixed(keys, 13, seed))


def test_hash_every_length_golden(ctx, golden):
    msg = golden["len_msg"]
    keys = [msg[:L].tobytes() for L in range(201)]
    off = np.zeros(len(keys) + 1, np.uint64)
    off[1:] = np.cumsum([len(k) for k in keys])
    blob = np.frombuffer(b"".join(keys), np.uint8)
    for si, seed in enumerate(golden["len_seeds"]):
        got = u64(ctx.hash_var(dev(blob), dev(off.view(np.int64)), seed=int(seed)))
        np.testing.assert_array_equal(got, golden["len_sig"][si, :, :2])


def test_hash_var_golden(ctx, golden):
    got = u64(ctx.hash_var(dev(golden["var_blob"]), dev(golden["var_off"].view(np.int64))))
    np.testing.assert_array_equal(got, golden["var_sig"])


def test_native_test_keys_histogram(ctx, golden):
    keys = [str(i).encode() for i in range(1_000_000)]
    off = np.zeros(len(keys) + 1, np.uint64)
    off[1:] = np.cumsum([len(k) for k in keys])
    blob = np.frombuffer(b"".join(keys), np.uint8)
    sig = u64(ctx.hash_var(dev(blob), dev(off.view(np.int64))))
    np.testing.assert_array_equal(sig[golden["native_sample_idx"]], golden["native_sample_sig"])
    m = O.num_buckets(1_000_000)
    counts = ctx.histogram_var(dev(blob), dev(off.view(np.int64)), m).cpu().numpy()
    np.testing.assert_array_equal(counts.view(np.uint32), golden["native_counts"])


@pytest.mark.parametrize("frontend", [0, 1, 2])
@pytest.mark.parametrize("mode", [0, 2])
def test_k13_histogram_golden(ctx, golden, mode, frontend):
    keys = O.gen_keys13(0, 1_000_000)
    m = O.num_buckets(1_000_000)
    ctx.set_histogram_mode(mode)
    ctx.set_frontend(frontend)
    try:
        counts = ctx.histogram_fixed(dev(keys), 13, m).cpu().numpy().view(np.uint32)
        sig = u64(ctx.hash_fixed(dev(keys[: 13 * 8192]), 13))
    finally:
        ctx.set_histogram_mode(0)
        ctx.set_frontend(0)
    np.testing.assert_array_equal(counts, golden["k13_counts"])
    np.testing.assert_array_equal(sig, golden["k13_sig"])


@pytest.mark.parametrize("frontend", [0, 1, 2])
def test_k13_ragged_tail(ctx, frontend):
    # last tile bounds-checked: the key buffer ends exactly at 13*n bytes
    ctx.set_frontend(frontend)
    try:
        for n in (1, 2, 3, 8191, 8192, 8193, 16385, 24575):
            keys = O.gen_keys13(9, n)
            np.testing.assert_array_equal(u64(ctx.hash_fixed(dev(keys), 13)), O.hash_fixed(keys, 13))
            m = 977
            np.testing.assert_array_equal(ctx.histogram_fixed(dev(keys), 13, m).cpu().numpy().view(np.uint32),
                                          O.histogram_fixed(keys, 13, m))
    finally:
        ctx.set_frontend(0)


def test_device_key_generator(ctx, golden):
    d = ctx.gen_keys13(0, 1_000_000)
    np.testing.assert_array_equal(d[: 13 * 1_000_000].cpu().numpy(), O.gen_keys13(0, 1_000_000))
    d = ctx.gen_keys13(123_456_789_000, 5_000)
    np.testing.assert_array_equal(d[: 13 * 5_000].cpu().numpy(), O.gen_keys13(123_456_789_000, 5_000))


@pytest.mark.parametrize("L", [13, 1, 5, 8, 12, 16, 20, 32, 33, 40, 80])
@pytest.mark.parametrize("m", [1, 667, 32_768, 32_769, 8_795_859])
def test_histogram_partitioned_many_partitions(ctx, L, m):
    # m up to the C4 bucket count: 269 partitions of 32768 buckets
    n = 300_007
    keys = rand_keys(n, L, m % 97 + L)
    counts = ctx.histogram_fixed(dev(keys), L, m).cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(counts, O.histogram_fixed(keys, L, m))


@pytest.mark.parametrize("L", [8, 12, 16])
def test_windowed_fixed_lengths_ragged(ctx, L):
    """8/12/16-byte keys on the windowed kernel (k_pass1_d13e<L>): the buffer
    ends exactly at L*n bytes (the last tiles go to the bounds-checked kernel),
    several chunks; counts == the oracle's."""
    m = 8_795_859
    for n in (1, 16383, 16384, 16385, 49_151, 200_003):
        keys = rand_keys(n, L, n % 89 + L)
        counts = ctx.histogram_fixed(dev(keys), L, m).cpu().numpy().view(np.uint32)
        np.testing.assert_array_equal(counts, O.histogram_fixed(keys, L, m))
    n = 300_001
    keys = rand_keys(n, L, 7)
    ctx.set_chunk_keys(8192 * 5)
    try:
        c = ctx.histogram_fixed(dev(keys), L, 66_667).cpu().numpy().view(np.uint32)
    finally:
        ctx.set_chunk_keys(0)
    np.testing.assert_array_equal(c, O.histogram_fixed(keys, L, 66_667))


def test_histogram_multi_chunk_and_accumulate(ctx):
    n = 100_003
    keys = O.gen_keys13(77, n)
    m = 5_000
    ctx.set_chunk_keys(8192 * 3)
    try:
        c = ctx.histogram_fixed(dev(keys), 13, m)
        c = ctx.histogram_fixed(dev(keys), 13, m, counts=c)  # accumulates
    finally:
        ctx.set_chunk_keys(0)
    np.testing.assert_array_equal(c.cpu().numpy().view(np.uint32), 2 * O.histogram_fixed(keys, 13, m))


def test_histogram_overflow_fallback(ctx):
    # one key repeated: every id lands in one partition region -> overflow ->
    # the in-stream fallback recounts the chunk with direct atomics
    n = 1_000_000
    keys = np.tile(np.frombuffer(b"abcdefghijklm", np.uint8), n)
    m = 8_795_859
    before = ctx.fallback_count()
    counts = ctx.histogram_fixed(dev(keys), 13, m).cpu().numpy().view(np.uint32)
    b = O.bucket(O.spooky_short(b"abcdefghijklm")[0], m)
    assert counts[b] == n and counts.sum() == n
    assert ctx.fallback_count() > before  # the LDS bin / region overflow was detected


@pytest.mark.parametrize("m", [1, 2, 300, 667, 66_667, 666_667, 8_795_859, 9_437_185, 20_000_000])
def test_binned_layouts_no_fallback(ctx, m):
    # every bucket count m maps to a bin layout (bucket >> shift, <= 288 bins)
    # or to the sort kernel; random distinct keys never take the fallback
    n = 3 * 16384 + 1234
    keys = O.gen_keys13(4242, n)
    before = ctx.fallback_count()
    counts = ctx.histogram_fixed(dev(keys), 13, m).cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(counts, O.histogram_fixed(keys, 13, m))
    assert ctx.fallback_count() == before


def test_empty_and_tiny(ctx):
    m = 10
    keys = torch.zeros(16, dtype=torch.uint8, device="cuda")
    c = ctx.histogram_fixed(keys, 13, m, n=0)
    assert int(c.sum()) == 0
    one = O.gen_keys13(5, 1)
    c = ctx.histogram_fixed(dev(one), 13, m).cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(c, O.histogram_fixed(one, 13, m))
    assert ctx.hash_fixed(keys, 13).shape[0] == 1  # 16 bytes -> one 13-byte key


def test_edge_offsets(ctx):
    rng = np.random.default_rng(3)
    for m in (1, 2, 1000, 8192, 8193, 3_000_001):
        c = rng.integers(0, 3000, m, dtype=np.int64).astype(np.int32)
        E = ctx.edge_offsets(dev(c)).cpu().numpy().view(np.uint64)
        np.testing.assert_array_equal(E, O.edge_offsets(c.view(np.uint32)))


def test_host_buffer_api(ctx):
    keys = O.gen_keys13(1000, 200_000)
    m = O.num_buckets(200_000)
    np.testing.assert_array_equal(ctx.histogram_fixed_host(keys, 13, m), O.histogram_fixed(keys, 13, m))
    np.testing.assert_array_equal(ctx.hash_fixed_host(keys, 13), O.hash_fixed(keys, 13))


def test_host_buffer_var_api(ctx, golden):
    """Host var-len entry points (what the JNI shim binds for byte[] keys):
    the reference's own NativeTest keys and random 0..255-byte keys, against
    the oracle; batch boundaries crossed by shrinking nothing (one batch) and
    by a key set over the 16 Mi-key batch."""
    rng = np.random.default_rng(31)
    lens = rng.integers(0, 256, 50_000)
    lens[:100] = 0
    off = np.zeros(lens.size + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    blob = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    m = 777
    np.testing.assert_array_equal(ctx.histogram_var_host(blob, off, m), O.histogram_var(blob, off, m))
    np.testing.assert_array_equal(ctx.hash_var_host(blob, off).reshape(-1), O.hash_var(blob, off).reshape(-1))
    gb, go = golden["var_blob"], golden["var_off"]
    np.testing.assert_array_equal(ctx.hash_var_host(gb, go).reshape(-1), golden["var_sig"].reshape(-1))
    # more keys than one batch (1 << 24): C5 keys from the device generator
    n = (1 << 24) + 12_345
    dblob, doff = ctx.gen_keys_var(3, n)
    hb, ho = dblob.cpu().numpy()[: int(doff[-1])], u64(doff)
    mm = O.num_buckets(n)
    np.testing.assert_array_equal(ctx.histogram_var_host(hb, ho, mm),
                                  ctx.histogram_var(dblob, doff, mm).cpu().numpy().view(np.uint32))
    with pytest.raises(ValueError):
        ctx.histogram_var_host(blob, off[::-1].copy(), m)


def test_generator_beyond_2e32_work_items(ctx):
    # 5e9 keys: more than 2^32 keys -> the generator must grid-stride
    n = 5_000_000_000
    keys = ctx.gen_keys13(0, n)
    for i in (0, 2**32 - 1, 2**32, 2**32 + 12345, n - 1):
        np.testing.assert_array_equal(keys[13 * i: 13 * i + 13].cpu().numpy(), O.gen_keys13(i, 1))
    m = O.num_buckets(n)
    c = ctx.histogram_fixed(keys, 13, m, n=n)
    assert int(c.sum(dtype=torch.int64)) == n
    assert int(c.max()) < 3000  # no hot bucket: distinct random-like keys
    del keys


def test_full_size_properties(ctx):
    """At a large size: total count, partitioned == atomic, sampled signatures."""
    n = 400_000_000
    keys = ctx.gen_keys13(0, n)
    m = O.num_buckets(n)
    f0 = ctx.fallback_count()
    c_part = ctx.histogram_fixed(keys, 13, m, n=n)
    assert ctx.fallback_count() == f0  # the fast path, not the overflow recount
    ctx.set_histogram_mode(2)
    try:
        c_atom = ctx.histogram_fixed(keys, 13, m, n=n)
    finally:
        ctx.set_histogram_mode(0)
    assert int(c_part.sum(dtype=torch.int64)) == n
    assert torch.equal(c_part, c_atom)
    E = ctx.edge_offsets(c_part)
    assert int(E[-1]) == n
    idx = np.arange(0, n, 9_999_991)
    sample = torch.cat([keys[13 * int(i): 13 * int(i) + 13] for i in idx]).cpu().numpy()
    np.testing.assert_array_equal(sample, O.gen_keys13(0, 1) if False else np.concatenate([O.gen_keys13(int(i), 1) for i in idx]))
    sig = u64(ctx.hash_fixed(dev(sample), 13))
    np.testing.assert_array_equal(sig, O.hash_fixed(sample, 13))
    del keys


# ---------------------------------------------------------------- A11-A13
@pytest.mark.parametrize("name", ["lk_ascii", "lk_k13"])
def test_lookup_golden_reference_vectors(ctx, golden, name):
    """Unchecked lookups == the reference's own mph_get_byte_array (golden)."""
    blob, off = golden[name + "_blob"], golden[name + "_off"]
    E, arr, res = golden[name + "_E"], golden[name + "_array"], golden[name + "_res"]
    sig = ctx.hash_var(dev(blob), dev(off.view(np.int64)))
    got = ctx.lookup(sig, off.size - 1, dev(E.view(np.int64)), dev(arr.view(np.int64)), check=False)
    np.testing.assert_array_equal(got.cpu().numpy(), res)


def _gov_set(n, width):
    keys = [str(i).encode() for i in range(n)]
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum([len(k) for k in keys])
    blob = np.frombuffer(b"".join(keys), np.uint8)
    sig = O.hash_var(blob, off)
    rc, E, values, sigbits = O.gov_build(sig, width)
    assert rc == 0
    return sig, E, values, sigbits


@pytest.mark.parametrize("width", [0, 4, 12, 16, 64])
def test_lookup_and_sign_match_oracle(ctx, width):
    n = 20_000
    sig, E, values, sigbits = _gov_set(n, width)
    dsig, dE, dv = dev(sig.view(np.int64)), dev(E.view(np.int64)), dev(values.view(np.int64))
    if width:
        dsb = ctx.sign(dsig, dE, dv, width)
        np.testing.assert_array_equal(dsb.cpu().numpy().view(np.uint64)[: sigbits.size - 1], sigbits[: sigbits.size - 1])
    else:
        dsb = None
    got = ctx.lookup(dsig, n, dE, dv, width, dsb, check=True).cpu().numpy()
    np.testing.assert_array_equal(got, O.lookup_batch(sig, n, E, values, width, sigbits))
    assert np.array_equal(np.sort(got), np.arange(n))
    # absent keys: same decisions as the oracle's checked lookup (GOV:567)
    absent = np.random.default_rng(5).integers(0, 2**63, size=(50_000, 2), dtype=np.int64)
    got2 = ctx.lookup(dev(absent), n, dE, dv, width, dsb, check=True).cpu().numpy()
    np.testing.assert_array_equal(got2, O.lookup_batch(absent.view(np.uint64), n, E, values, width, sigbits))


@pytest.mark.parametrize("approx", [False, True])
def test_index_scatter(ctx, approx):
    rng = np.random.default_rng(11)
    n = 30_000
    rank = rng.permutation(n).astype(np.int64)
    rank[::97] = -1                      # rejected lookups are skipped
    addr = rng.integers(0, 2**63, n, dtype=np.int64)
    v8 = rng.integers(0, 2**63, n, dtype=np.int64)
    vlen = rng.integers(1, 40, n).astype(np.uint8)
    for start, length in ((0, n), (5000, 7000), (29_990, 10)):   # W:112-150 passes
        idx = torch.zeros(length, dtype=torch.int64, device="cuda")
        ia = torch.zeros(length * 8, dtype=torch.uint8, device="cuda") if approx else None
        ctx.index_scatter(dev(rank), dev(addr), start, length, idx,
                          dev(v8) if approx else None, dev(vlen) if approx else None, ia)
        want = np.zeros(length, np.uint64)
        want_a = np.zeros(length * 8, np.uint8)
        for i in range(n):
            r = rank[i]
            if r < 0 or not (start <= r < start + length):
                continue
            # Long.reverseBytes(addr) (W:138, REVERSE_ORDER on little-endian hosts)
            want[r - start] = int.from_bytes(int(addr[i]).to_bytes(8, "little"), "big")
            if approx:
                b = int(v8[i]).to_bytes(8, "little")
                k = min(int(vlen[i]), 8)
                want_a[(r - start) * 8:(r - start) * 8 + k] = np.frombuffer(b[:k], np.uint8)
        np.testing.assert_array_equal(idx.cpu().numpy().view(np.uint64), want)
        if approx:
            np.testing.assert_array_equal(ia.cpu().numpy(), want_a)


# ---------------------------------------------------------------- A5/A6/A8/A11 device build
def _rand_sigs(n, seed):
    return np.random.default_rng(seed).integers(0, 2**63, size=(n, 2), dtype=np.int64).view(np.uint64) * np.uint64(2) \
        + np.random.default_rng(seed + 1).integers(0, 2, size=(n, 2), dtype=np.int64).view(np.uint64)


@pytest.mark.parametrize("n,width", [(1, 0), (2, 8), (9, 0), (10, 16), (12, 3), (39, 64), (777, 5),
                                     (1500, 0), (1501, 12), (3000, 1), (20_000, 4), (150_000, 32),
                                     (600_000, 4)])
def test_gov_build_matches_oracle(ctx, n, width):
    """Device GOV build (sort, E, solve, sign) is bit-identical to oracle/bo_gov_build."""
    sig = _rand_sigs(n, n * 7 + width)
    rc, E, values, sigbits = O.gov_build(sig, width)
    assert rc == 0
    dE, dv, dsb = ctx.gov_build(dev(sig.view(np.int64)), width)
    np.testing.assert_array_equal(dE.cpu().numpy().view(np.uint64), E)
    np.testing.assert_array_equal(dv.cpu().numpy().view(np.uint64), values)
    if width:
        np.testing.assert_array_equal(dsb.cpu().numpy().view(np.uint64), sigbits)
    got = ctx.lookup(dev(sig.view(np.int64)), n, dE, dv, width, dsb, check=True).cpu().numpy()
    assert np.array_equal(np.sort(got), np.arange(n))


def test_gov_build_string_keys_and_order_independence(ctx):
    """NativeTest-style keys; the device sorts, so input order does not matter (CBHS:939-955)."""
    n = 60_000
    sig, E, values, sigbits = _gov_set(n, 10)
    perm = np.random.default_rng(3).permutation(n)
    for s in (sig, sig[perm]):
        dE, dv, dsb = ctx.gov_build(dev(np.ascontiguousarray(s).view(np.int64)), 10)
        np.testing.assert_array_equal(dE.cpu().numpy().view(np.uint64), E)
        np.testing.assert_array_equal(dv.cpu().numpy().view(np.uint64), values)
        np.testing.assert_array_equal(dsb.cpu().numpy().view(np.uint64), sigbits)


def test_gov_build_empty(ctx):
    rc, E, values, _ = O.gov_build(np.zeros((0, 2), np.uint64), 0)
    dE, dv, _ = ctx.gov_build(torch.zeros((0, 2), dtype=torch.int64, device="cuda"), 0)
    np.testing.assert_array_equal(dE.cpu().numpy().view(np.uint64), E)
    np.testing.assert_array_equal(dv.cpu().numpy().view(np.uint64), values)


def test_gov_build_duplicate_rejected(ctx):
    """Duplicate signatures -> BSDB_EDUP (CBHS:969-972 DuplicateException)."""
    sig = _rand_sigs(5000, 99)
    sig[4321] = sig[17]
    with pytest.raises(Exception, match="EDUP"):
        ctx.gov_build(dev(sig.view(np.int64)), 0)


def test_gov_build_large_valid(ctx):
    """2 M keys: sizes the oracle is slow on; checked by the bijection + checksum properties."""
    n = 2_000_000
    sig = _rand_sigs(n, 2024)
    dsig = dev(sig.view(np.int64))
    dE, dv, dsb = ctx.gov_build(dsig, 8)
    assert int(dE[-1]) & ((1 << 56) - 1) == n
    got = ctx.lookup(dsig, n, dE, dv, 8, dsb, check=True)
    assert torch.equal(torch.sort(got).values, torch.arange(n, device="cuda"))
    # a sample of buckets against the oracle's per-bucket lookup on the device-built structure
    idx = np.arange(0, n, 997)
    np.testing.assert_array_equal(got.cpu().numpy()[idx],
                                  O.lookup_batch(sig[idx], n, dE.cpu().numpy().view(np.uint64),
                                                 dv.cpu().numpy().view(np.uint64), 8,
                                                 dsb.cpu().numpy().view(np.uint64)))


# ---------------------------------------------------------------- config C5 var-len keys
def _splitmix64_np(x):
    with np.errstate(over="ignore"):
        z = x.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _varkeys_np(first, n):
    """Python restatement of the C5 generator (hash_kernels.hip k_gen_var_*)."""
    w = [1 / r ** 1.1 for r in range(1, 58)]
    tot, c, thr = sum(w), 0.0, []
    for x in w[:-1]:
        c += x
        thr.append(int(c / tot * 2 ** 64))
    thr = np.array(thr, dtype=np.uint64)
    i = np.arange(first, first + n, dtype=np.uint64)
    u = _splitmix64_np(i ^ np.uint64(0xB5DB0005))
    lens = 8 + (u[:, None] >= thr[None, :]).sum(1)
    keys = []
    for k in range(n):
        ii = int(i[k])
        b = bytearray(ii.to_bytes(8, "big"))
        for wdx in range((lens[k] - 8 + 7) // 8):
            t = int(_splitmix64_np(np.array([((ii << 3) + wdx) ^ 0xB5DB0005A5A5A5A5], np.uint64))[0])
            b += t.to_bytes(8, "little")
        keys.append(bytes(b[: lens[k]]))
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    return np.frombuffer(b"".join(keys), np.uint8), off


def test_var_key_generator(ctx):
    for first, n in ((0, 3000), (2 ** 32 - 700, 1500)):
        blob, off = ctx.gen_keys_var(first, n)
        want_blob, want_off = _varkeys_np(first, n)
        np.testing.assert_array_equal(u64(off), want_off)
        np.testing.assert_array_equal(blob.cpu().numpy()[: want_blob.size], want_blob)


@pytest.mark.parametrize("mode", [0, 2])
def test_var_staged_matches_oracle_and_direct(ctx, mode):
    """LDS-staged var-len front end (default) == direct front end == oracle."""
    n = 300_001
    blob, off = ctx.gen_keys_var(5, n)
    hb, ho = blob.cpu().numpy(), u64(off)
    sig = u64(ctx.hash_var(blob, off))
    np.testing.assert_array_equal(sig, O.hash_var(hb[: int(ho[-1])], ho))
    m = O.num_buckets(n) * 7
    ctx.set_histogram_mode(mode)
    try:
        c0 = ctx.histogram_var(blob, off, m).cpu().numpy().view(np.uint32)
        ctx.set_frontend(2)
        c2 = ctx.histogram_var(blob, off, m).cpu().numpy().view(np.uint32)
    finally:
        ctx.set_frontend(0)
        ctx.set_histogram_mode(0)
    np.testing.assert_array_equal(c0, c2)
    np.testing.assert_array_equal(c0, O.histogram_var(hb[: int(ho[-1])], ho, m))


def test_var_staged_long_subtiles_fall_back(ctx):
    """Sub-tiles whose bytes exceed the LDS stage (long keys) hash from global memory."""
    rng = np.random.default_rng(17)
    lens = rng.integers(0, 30, 40_000)
    lens[9000:9600] = rng.integers(60, 180, 600)     # one sub-tile far over 32 KiB
    lens[20_000:20_512] = 63                          # exactly at the stage limit
    off = np.zeros(lens.size + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    blob = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    sig = u64(ctx.hash_var(dev(blob), dev(off.view(np.int64))))
    np.testing.assert_array_equal(sig, O.hash_var(blob, off))


@pytest.mark.parametrize("m", [1, 2, 5_000, 66_667, 2_666_667, 144 * 32768, 144 * 32768 + 1])
def test_var_binned_bucket_counts(ctx, m):
    """Persistent binned var-len kernel (k_pass1_vare) over bin layouts from 1
    bin to its 144-bin limit (and just past it: the generic kernel) == oracle,
    with no overflow fallback; n leaves a ragged tail for the generic kernel."""
    n = 300_001
    blob, off = ctx.gen_keys_var(11, n)
    hb, ho = blob.cpu().numpy(), u64(off)
    before = ctx.fallback_count()
    got = ctx.histogram_var(blob, off, m).cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(got, O.histogram_var(hb[: int(ho[-1])], ho, m))
    assert ctx.fallback_count() == before


def test_var_binned_ragged_groups(ctx):
    """Groups of 64 keys whose byte range is empty, over the 2 KiB prefetch
    (synchronous loads), or over the 4352-byte stage (hashed from global
    memory), and keys of 0..255 bytes, at tile and group boundaries."""
    rng = np.random.default_rng(23)
    n = 3 * 8192 + 777
    lens = rng.integers(8, 30, n)
    lens[0:64] = 0                                    # an all-empty group at the start
    lens[8192 - 32:8192 + 64] = 0                     # across a tile boundary
    lens[9000:9640] = rng.integers(40, 65, 640)       # 2.5-4 KiB groups
    lens[12000:12700] = rng.integers(70, 256, 700)    # > 4352-byte groups
    lens[20000:20064] = 64                            # exactly 64 x 64 B
    lens[-50:] = rng.integers(0, 256, 50)             # ragged tail
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    blob = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    before = ctx.fallback_count()
    for m in (3, 40_000):
        got = ctx.histogram_var(dev(blob), dev(off.view(np.int64)), m).cpu().numpy().view(np.uint32)
        np.testing.assert_array_equal(got, O.histogram_var(blob, off, m))
    assert ctx.fallback_count() == before


def test_var_full_size_properties(ctx):
    """C5 shape at scale: the binned var-len kernel equals the direct-atomics
    histogram (an independent kernel) on 1e8 keys, sums to n, no fallback."""
    n = 100_000_000
    m = 4_000_000_000 // 1500 + 1
    blob, off = ctx.gen_keys_var(0, n)
    f0 = ctx.fallback_count()
    c_bin = ctx.histogram_var(blob, off, m)
    assert ctx.fallback_count() == f0
    ctx.set_histogram_mode(2)
    try:
        c_atom = ctx.histogram_var(blob, off, m)
    finally:
        ctx.set_histogram_mode(0)
    assert int(c_bin.sum(dtype=torch.int64)) == n
    assert torch.equal(c_bin, c_atom)
    del blob, off
