"""GPU parity of the single-pass histogram (mode 3, k_hist13_fused): counts
bit-identical to the oracle and to the two-pass path, through the C ABI.
Integer work: every comparison is exact."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ROUND = 256 * 16384  # keys of one super-tile round (every workgroup one super-tile)


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from bsdb_amd import Context
    c = Context(0)
    yield c
    c.close()


def counts_of(ctx, keys, n, m, mode, seed=0, counts=None):
    ctx.set_histogram_mode(mode)
    try:
        return ctx.histogram_fixed(keys, 13, m, counts=counts, n=n, seed=seed)
    finally:
        ctx.set_histogram_mode(0)


def ran_fused(ctx, before):
    launches, timeouts = ctx.fused_status()
    assert timeouts == 0
    return launches > before


@pytest.mark.parametrize("m", [8_795_859, 11_194, 2_000, 256, 1])
def test_fused_equals_oracle(ctx, m):
    # 4 rounds + a ragged tail (the tail takes the two-pass path).  Owner
    # tables count in u16: above 16384 keys per bucket on average (m = 256,
    # 1) mode 3 takes the two-pass path
    n = 4 * ROUND + 12_345
    keys = ctx.gen_keys13(0, n)
    l0 = ctx.fused_status()[0]
    f0 = ctx.fallback_count()
    got = counts_of(ctx, keys, n, m, 3).cpu().numpy().view(np.uint32)
    fused = n // m <= 16384
    assert ran_fused(ctx, l0) == fused
    if fused:
        assert ctx.fallback_count() == f0  # random keys: no bin overflow
    np.testing.assert_array_equal(got, O.histogram_fixed(keys[: 13 * n].cpu().numpy(), 13, m))


def test_fused_equals_two_pass_large(ctx):
    """2^31 + 1 device-generated keys at the C4 bucket count: identical to the
    two-pass path, sum = n."""
    n = (1 << 31) + 1
    m = 8_795_859
    keys = ctx.gen_keys13(5_000_000_000, n)
    l0 = ctx.fused_status()[0]
    a = counts_of(ctx, keys, n, m, 3)
    assert ran_fused(ctx, l0)
    b = counts_of(ctx, keys, n, m, 1)
    assert torch.equal(a, b)
    assert int(a.to(torch.int64).sum().item()) == n
    del keys


def test_fused_accumulates_and_seed(ctx):
    n = 5 * ROUND
    m = 66_667
    keys = ctx.gen_keys13(77, n)
    host = keys[: 13 * n].cpu().numpy()
    seed = 0x0123456789ABCDEF
    c = counts_of(ctx, keys, n, m, 3, seed=seed)
    c = counts_of(ctx, keys, n, m, 3, seed=seed, counts=c)  # accumulates
    np.testing.assert_array_equal(c.cpu().numpy().view(np.uint32), 2 * O.histogram_fixed(host, 13, m, seed))


def test_fused_overflow_falls_back(ctx):
    # one key repeated: every id of a round lands in one owner's bin -> the
    # bin overflows -> nothing is added and the keys are recounted with
    # direct atomics
    n = 4 * ROUND + 7
    key = b"abcdefghijklm"
    keys = torch.from_numpy(np.tile(np.frombuffer(key, np.uint8), n)).cuda()
    m = 8_795_859
    l0 = ctx.fused_status()[0]
    before = ctx.fallback_count()
    counts = counts_of(ctx, keys, n, m, 3).cpu().numpy().view(np.uint32)
    assert ran_fused(ctx, l0)
    b = O.bucket(O.spooky_short(key)[0], m)
    assert counts[b] == n and counts.sum() == n
    assert ctx.fallback_count() > before


def test_fused_small_sets_take_two_pass(ctx):
    # fewer than 4 rounds: mode 3 runs the two-pass path, same counts
    for n in (0, 1, 16_385, 3 * ROUND + 5):
        keys = ctx.gen_keys13(9, max(n, 1))
        m = 977
        l0 = ctx.fused_status()[0]
        got = counts_of(ctx, keys, n, m, 3)
        assert ctx.fused_status()[0] == l0
        if n:
            np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32),
                                          O.histogram_fixed(keys[: 13 * n].cpu().numpy(), 13, m))


# ---- pass 2 of chunk i beside pass 1 of chunk i + 1 (bsdb_set_pipeline) ----

def pipelined(ctx, keys, n, m, on, chunks=0, p2_cus=0):
    ctx.set_pipeline(1 if on else 0, chunks, p2_cus)
    try:
        return ctx.histogram_fixed(keys, 13, m, n=n)
    finally:
        ctx.set_pipeline(-1)


@pytest.mark.parametrize("chunks,p2_cus", [(2, 32), (5, 16), (16, 64)])
def test_pipelined_chunks_equal_oracle(ctx, chunks, p2_cus):
    n = 3_000_017  # ragged: chunk ends mid-tile, the last tile bounds-checked
    m = 8_795_859
    keys = ctx.gen_keys13(31, n)
    got = pipelined(ctx, keys, n, m, True, chunks, p2_cus).cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(got, O.histogram_fixed(keys[: 13 * n].cpu().numpy(), 13, m))


def test_pipelined_equals_serial_large(ctx):
    n = (1 << 30) + 12_345
    m = n // 1500 + 1
    keys = ctx.gen_keys13(7_000_000_000, n)
    a = pipelined(ctx, keys, n, m, True, 8, 32)
    b = pipelined(ctx, keys, n, m, False)
    assert torch.equal(a, b)
    assert int(a.to(torch.int64).sum().item()) == n


def test_pipelined_overflow_falls_back(ctx):
    # one key repeated: both id buffers overflow, each chunk is recounted
    n = 600_000
    key = b"abcdefghijklm"
    keys = torch.from_numpy(np.tile(np.frombuffer(key, np.uint8), n)).cuda()
    m = 8_795_859
    before = ctx.fallback_count()
    counts = pipelined(ctx, keys, n, m, True, 4, 32).cpu().numpy().view(np.uint32)
    b = O.bucket(O.spooky_short(key)[0], m)
    assert counts[b] == n and counts.sum() == n
    assert ctx.fallback_count() >= before + 4
