"""GPU: every BASELINE.json config at its own size (SURVEY.md §8 sizes),
through the C ABI, against the CPU oracle (C restatement pinned to the
reference's spooky.c/mph.c) -- whole arrays where the oracle finishes in
about a minute on the box's cores, size-independent properties and samples
where it does not.

  C2  1e8 x 13 B, exact index, cb = 4      full host-buffer build + index.db
                                            (pass loop and the F2 one-call form)
  C3  1e9 x 13 B, index.approximate = true  full build + index.db/index_a.db
  C4  13 193 787 549 x 13 B (README shape)  full-size histogram == oracle
  C5  4e9 var-len 8-64 B Zipf, cb = 16      full-size histogram == oracle,
                                            cb = 16 build on a sample
"""
import os
import shutil
import tempfile
import threading

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

THREADS = O.cpu_threads()
README_N = 13_193_787_549


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from bsdb_amd import Context
    c = Context(0)
    yield c
    c.close()
    torch.cuda.empty_cache()


def u64(t):
    return t.cpu().numpy().view(np.uint64)


def in_background(fn, *args):
    """Runs an oracle call (ctypes releases the GIL) beside the GPU work."""
    box = {}
    th = threading.Thread(target=lambda: box.setdefault("r", fn(*args)))
    th.start()
    return th, box


@pytest.mark.timeout(900)
def test_c4_full_size_histogram_equals_oracle(ctx):
    n, m = README_N, README_N // 1500 + 1
    th, box = in_background(O.histogram_gen13_mt, 0, n, m, THREADS)
    keys = ctx.gen_keys13(0, n)                      # 171.5 GB in HBM
    counts = ctx.histogram_fixed(keys, 13, m)
    E = ctx.edge_offsets(counts)
    sig = ctx.hash_fixed(keys[: 13 * 100_000], 13)
    torch.cuda.synchronize()
    got_counts, got_E = counts.cpu().numpy().view(np.uint32), u64(E)
    tail = keys[13 * (n - 100_000):].cpu().numpy()
    del keys, counts, E
    torch.cuda.empty_cache()
    assert ctx.fallback_count() == 0
    assert int(got_E[-1]) == n
    np.testing.assert_array_equal(u64(sig), O.hash_fixed(O.gen_keys13(0, 100_000), 13))
    np.testing.assert_array_equal(tail, O.gen_keys13(n - 100_000, 100_000))
    th.join()
    exp, _ = box["r"]
    np.testing.assert_array_equal(got_counts, exp)      # the whole 35 MB histogram
    np.testing.assert_array_equal(got_E, O.edge_offsets(exp))


@pytest.mark.timeout(900)
def test_c4_exact_full_build_one_gpu(ctx):
    """C4's exact index on ONE GPU: all 13 193 787 549 keys resident (171.5 GB),
    the GOV structure and index.db by sequential bucket-range passes (the
    reference's segment-by-segment solve, CBHS:852-978 / GOV:385-448), the
    index slots (rank -> byte-reversed record address, W:129-145) copied to
    host memory pass by pass.  Checked: E[m] = n; the device's bijection check
    of every range's ranks (bsdb_set_verify); checked lookups of 200 000 keys
    in 20 blocks == the oracle's lookup on the exported structure, and their
    index slots; no slot left empty."""
    n, m, width, base, stride = README_N, README_N // 1500 + 1, 4, 0x1000, 48
    keys = ctx.gen_keys13(0, n)                          # 171.5 GB in HBM
    index = np.empty(n, np.uint64)                       # 105.6 GB of host memory: index.db
    ctx.set_verify(True)
    try:
        E, vals, sb, used = ctx.mph_build_index_passes(keys, 13, n, width, 0, addr_base=base, addr_stride=stride,
                                                       index=index)
    finally:
        ctx.set_verify(False)
    del keys
    hE, hv, hs = u64(E), u64(vals), u64(sb)
    del E, vals, sb
    torch.cuda.empty_cache()
    assert used >= 2 and int(hE[-1]) & ((1 << 56) - 1) == n
    rng = np.random.default_rng(44)
    for first in np.sort(rng.integers(0, n - 10_000, 20)):
        first = int(first)
        sig = O.hash_fixed(O.gen_keys13(first, 10_000), 13)
        r = O.lookup_batch_mt(sig, n, hE, hv, width, hs, True, THREADS)
        assert r.min() >= 0
        exp = (np.uint64(base) + np.uint64(stride) * np.arange(first, first + 10_000, dtype=np.uint64)).byteswap()
        np.testing.assert_array_equal(index[r], exp)
    for lo in range(0, n, 1 << 30):
        assert np.count_nonzero(index[lo: lo + (1 << 30)] == 0) == 0


@pytest.mark.timeout(900)
def test_c5_full_size_histogram_equals_oracle(ctx):
    n, m = 4_000_000_000, 4_000_000_000 // 1500 + 1
    th, box = in_background(O.histogram_genvar_mt, 0, n, m, THREADS)
    blob, off = ctx.gen_keys_var(0, n)               # ~103 GB: offsets + blob
    binned = ctx.histogram_var(blob, off, m)
    ctx.set_histogram_mode(2)
    try:
        atomic = ctx.histogram_var(blob, off, m)
    finally:
        ctx.set_histogram_mode(0)
    torch.cuda.synchronize()
    head_off = u64(off[:10_001])
    head = blob[: int(head_off[-1])].cpu().numpy()
    b_np, a_np = binned.cpu().numpy().view(np.uint32), atomic.cpu().numpy().view(np.uint32)
    del blob, off, binned, atomic
    torch.cuda.empty_cache()
    assert ctx.fallback_count() == 0
    assert int(b_np.astype(np.uint64).sum()) == n
    np.testing.assert_array_equal(b_np, a_np)
    eb, eo = O.gen_keys_var(0, 10_000)                 # the device generator is the C5 recipe
    np.testing.assert_array_equal(head_off, eo)
    np.testing.assert_array_equal(head, eb)
    th.join()
    exp, _ = box["r"]
    np.testing.assert_array_equal(b_np, exp)


@pytest.mark.timeout(900)
def test_c5_full_build_one_gpu(ctx):
    """C5 at its full size on ONE GPU: 4e9 variable-length keys (8-64 B Zipf,
    ~103 GB with offsets), hash.checksum.bits = 16, the whole GOV structure and
    index by sequential bucket-range passes; index slots to host memory.
    Checked as C4: E[m] = n, the device's bijection check, checked lookups of
    100 000 keys in 10 blocks == the oracle's on the exported structure (with
    their 16 checksum bits), their index slots, no slot left empty."""
    n, width, base, stride = 4_000_000_000, 16, 0x2000, 64
    blob, off = ctx.gen_keys_var(0, n)
    index = np.empty(n, np.uint64)
    ctx.set_verify(True)
    try:
        E, vals, sb, used = ctx.mph_build_index_passes(blob, 0, n, width, 0, offsets=off, addr_base=base,
                                                       addr_stride=stride, index=index)
    finally:
        ctx.set_verify(False)
    del blob, off
    hE, hv, hs = u64(E), u64(vals), u64(sb)
    del E, vals, sb
    torch.cuda.empty_cache()
    assert int(hE[-1]) & ((1 << 56) - 1) == n
    rng = np.random.default_rng(45)
    for first in np.sort(rng.integers(0, n - 10_000, 10)):
        first = int(first)
        kb, ko = O.gen_keys_var(first, 10_000)
        r = O.lookup_batch_mt(O.hash_var(kb, ko), n, hE, hv, width, hs, True, THREADS)
        assert r.min() >= 0
        exp = (np.uint64(base) + np.uint64(stride) * np.arange(first, first + 10_000, dtype=np.uint64)).byteswap()
        np.testing.assert_array_equal(index[r], exp)
    for lo in range(0, n, 1 << 30):
        assert np.count_nonzero(index[lo: lo + (1 << 30)] == 0) == 0


@pytest.mark.timeout(600)
def test_c5_checksum16_build_on_a_sample(ctx):
    """cb = 16 (C5's hash.checksum.bits) on the first 2e6 C5 keys, device
    path end to end (generator -> hash -> GOV build -> sign) vs the oracle."""
    n = 2_000_000
    blob, off = ctx.gen_keys_var(0, n)
    sig = ctx.hash_var(blob, off)
    E, vals, sb = ctx.gov_build(sig, 16)
    hb, ho = O.gen_keys_var(0, n)
    osig = O.hash_var(hb, ho)
    np.testing.assert_array_equal(u64(sig), osig)
    rc, oE, ov, osb, _ = O.gov_build_mt(osig, 16, THREADS)
    assert rc == 0
    np.testing.assert_array_equal(u64(E), oE)
    np.testing.assert_array_equal(u64(vals), ov)
    np.testing.assert_array_equal(u64(sb)[: osb.size], osb)


def solver_report(name, n, E, extra=None):
    """What the solve went through on a key set: seeds per
    bucket (E's top byte, GOV:434-436) and the oversized buckets that take
    k_gov_solve_mid (> 1 664 keys) or the global-slab solver (> 2 048).  With
    BSDB_TEST_REPORT=<file> it is appended there as one JSON line."""
    import json
    seeds = (E[:-1] >> np.uint64(56)).astype(np.int64)
    size = np.diff((E & np.uint64((1 << 56) - 1)).astype(np.int64))
    rep = {"test": name, "n": int(n), "buckets": int(size.size),
           "buckets_seed_ge1": int((seeds >= 1).sum()), "buckets_seed_ge2": int((seeds >= 2).sum()),
           "buckets_seed_ge4": int((seeds >= 4).sum()), "max_seed": int(seeds.max()),
           "mean_attempts": float(seeds.mean() + 1), "max_bucket": int(size.max()),
           "buckets_mid_solver": int(((size > 1664) & (size <= 2048)).sum()),
           "buckets_global_slab": int((size > 2048).sum())}
    rep.update(extra or {})
    print(rep)
    path = os.environ.get("BSDB_TEST_REPORT")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(rep) + "\n")
    return rep


def gov_profile_counts(text):
    """The counters of the last `[gov-profile] m=...` line (BSDB_GOV_PROFILE)."""
    lines = [ln for ln in text.splitlines() if ln.startswith("[gov-profile] m=")]
    out = {}
    for tok in (lines[-1].split() if lines else []):
        if "=" in tok:
            k, v = tok.split("=", 1)
            try:
                out[k] = float(v)
            except ValueError:
                pass
    return out


@pytest.mark.timeout(900)
def test_c2_passes_build_equals_oracle_field_for_field(ctx, capfd):
    """the production solver pinned at C2's size.  1e8
    13-byte keys, cb = 4, built by the bucket-range pass path (3 passes, the
    C4 form) and compared FIELD FOR FIELD with the oracle's independent build
    (bo_gov_build_mt, oracle/bsdb_oracle.c): every E word (offsets + local
    seeds, GOV:385-436), every 2-bit value word (GOV:438-442,483-485), every
    checksum word (GOV:492-508), and every index.db slot against W:129-145
    (slot = getLong(key), byte-reversed address).  At 1e8 keys the rare paths
    fire naturally: buckets over 1 664 keys (k_gov_solve_mid), high seeds, the
    FVS blocks; the report counts them, and a second build through the
    profiling solver instance must give the same structure."""
    n, width, passes, base, stride = 100_000_000, 4, 3, 0x1000, 48
    keys = O.gen_keys13_mt(0, n, THREADS)

    def oracle():
        sig = O.hash_fixed_mt(keys, 13, THREADS)
        O.solve_stats(True)
        rc, E, vals, sb, dt = O.gov_build_mt(sig, width, THREADS)
        st = O.solve_stats(True)
        ranks = O.lookup_batch_mt(sig, n, E, vals, width, sb, True, THREADS) if rc == 0 else None
        return rc, E, vals, sb, dt, st, ranks

    th, box = in_background(oracle)
    dk = torch.from_numpy(keys).cuda()
    d_index = torch.zeros(n, dtype=torch.int64, device="cuda")
    E, vals, sb, used = ctx.mph_build_index_passes(dk, 13, n, width, passes, addr_base=base, addr_stride=stride,
                                                   index=d_index)
    torch.cuda.synchronize()
    assert used == passes
    hE, hv, hs, hidx = u64(E), u64(vals), u64(sb), u64(d_index)
    del E, vals, sb, d_index
    # the same build through the profiling instance of the solver, its counters
    os.environ["BSDB_GOV_PROFILE"] = "1"
    try:
        capfd.readouterr()
        E2, v2, s2, _ = ctx.mph_build_index_passes(dk, 13, n, width, passes)
        torch.cuda.synchronize()
        prof_text = capfd.readouterr().err
    finally:
        del os.environ["BSDB_GOV_PROFILE"]
    np.testing.assert_array_equal(u64(E2), hE)
    np.testing.assert_array_equal(u64(v2), hv)
    np.testing.assert_array_equal(u64(s2), hs)
    del E2, v2, s2, dk
    torch.cuda.empty_cache()
    th.join()
    rc, oE, ov, osb, dt, st, ranks = box["r"]
    assert rc == 0
    np.testing.assert_array_equal(hE, oE)                 # offsets + every bucket's seed
    np.testing.assert_array_equal(hv, ov)                 # every 2-bit value word
    np.testing.assert_array_equal(hs[: osb.size], osb)    # every checksum word
    assert ranks.min() >= 0 and np.array_equal(np.bincount(ranks, minlength=n), np.ones(n, np.int64))
    exp = np.zeros(n, np.uint64)
    exp[ranks] = (np.uint64(base) + np.uint64(stride) * np.arange(n, dtype=np.uint64)).byteswap()
    np.testing.assert_array_equal(hidx, exp)              # index.db slots (W:129-145)
    # the last profile line is the last pass's; the passes together:
    lines = [ln for ln in prof_text.splitlines() if ln.startswith("[gov-profile] m=")]
    tot = {}
    for ln in lines:
        for k, v in gov_profile_counts(ln).items():
            if k.startswith("n_"):
                tot[k] = tot.get(k, 0) + v
    rep = solver_report("c2_passes_1e8", n, hE, {
        "oracle_seconds": dt, "oracle_attempts": st["attempts"], "oracle_unorientable": st["unorientable"],
        "oracle_inconsistent": st["inconsistent"], "oracle_degenerate": st["degenerate"],
        "oracle_singular_solved": st["singular_solved"], "profile_passes": len(lines),
        **{"device_" + k: int(v) for k, v in tot.items() if k in (
            "n_seeds", "n_fvs_blocks", "n_singular_solved", "n_null_vectors", "n_speculative_lost",
            "n_fail_degenerate", "n_fail_orient", "n_fail_inconsistent", "n_small_scc_fallbacks",
            "n_rows_in_blocks_over_440", "n_heavy")}})
    assert len(lines) == passes
    # the rare paths did fire at this size
    assert rep["buckets_seed_ge4"] > 0
    assert rep["buckets_mid_solver"] >= 1  # (this key set's largest bucket: 1 669 keys)


@pytest.mark.timeout(900)
def test_c5_varlen_passes_build_equals_oracle_on_1e8_keys(ctx):
    """The same pin for C5's shape: the first 1e8 C5 keys (8-64 B Zipf,
    device-generated = the oracle's recipe), hash.checksum.bits = 16, through
    the variable-length bucket-range pass path (2 passes): E, values and the
    16-bit checksums field for field against the oracle's build, and every
    index slot against the W:129-145 restatement."""
    n, width, passes, base, stride = 100_000_000, 16, 2, 0x2000, 64
    hb, ho = O.gen_keys_var(0, n)

    def oracle():
        sig = O.hash_var(hb, ho)
        rc, E, vals, sb, _ = O.gov_build_mt(sig, width, THREADS)
        ranks = O.lookup_batch_mt(sig, n, E, vals, width, sb, True, THREADS) if rc == 0 else None
        return rc, E, vals, sb, ranks

    th, box = in_background(oracle)
    blob, off = ctx.gen_keys_var(0, n)
    d_index = torch.zeros(n, dtype=torch.int64, device="cuda")
    E, vals, sb, used = ctx.mph_build_index_passes(blob, 0, n, width, passes, offsets=off, addr_base=base,
                                                   addr_stride=stride, index=d_index)
    torch.cuda.synchronize()
    assert used == passes
    head = blob[: int(ho[1000])].cpu().numpy()
    hE, hv, hs, hidx = u64(E), u64(vals), u64(sb), u64(d_index)
    del blob, off, E, vals, sb, d_index
    torch.cuda.empty_cache()
    np.testing.assert_array_equal(head, hb[: int(ho[1000])])   # (the device generator is the oracle's recipe)
    th.join()
    rc, oE, ov, osb, ranks = box["r"]
    assert rc == 0
    np.testing.assert_array_equal(hE, oE)
    np.testing.assert_array_equal(hv, ov)
    np.testing.assert_array_equal(hs[: osb.size], osb)
    exp = np.zeros(n, np.uint64)
    exp[ranks] = (np.uint64(base) + np.uint64(stride) * np.arange(n, dtype=np.uint64)).byteswap()
    np.testing.assert_array_equal(hidx, exp)
    solver_report("c5_varlen_passes_1e8", n, hE)


@pytest.mark.timeout(900)
def test_c3_approx_host_passes_equals_oracle_on_a_2e8_slice(ctx, tmp_path):
    """VERDICT r4 item 1, C3's mode: index.approximate = true from host
    buffers through the streaming builder's bucket-range passes (4 passes),
    on the first 2e8 C3 keys.  The MPHF equals the oracle's build field for
    field, index.db and index_a.db equal the W:129-145 restatement (slot =
    getLong(key): byte-reversed address, and the value's first 8 bytes) byte
    for byte."""
    n, width, passes = 200_000_000, 4, 4
    keys = O.gen_keys13_mt(0, n, THREADS)

    def oracle():
        sig = O.hash_fixed_mt(keys, 13, THREADS)
        rc, E, vals, sb, dt = O.gov_build_mt(sig, width, THREADS)
        ranks = O.lookup_batch_mt(sig, n, E, vals, width, sb, True, THREADS) if rc == 0 else None
        return rc, E, vals, sb, ranks

    th, box = in_background(oracle)
    addr, value8, vlen = records(0, n)
    d = big_tmp(tmp_path, 16 * n)
    ip, ap = os.path.join(d, "index.db"), os.path.join(d, "index_a.db")
    mph, used = ctx.mph_build_index_passes_host(keys, 13, width, ip, addr_np=addr, value8_np=value8, vlen_np=vlen,
                                                approximate=True, index_a_path=ap, passes=passes)
    assert used == passes
    dE, dv, ds = mph.export()
    mph.close()
    th.join()
    rc, E, vals, sb, ranks = box["r"]
    assert rc == 0
    np.testing.assert_array_equal(dE, E)
    np.testing.assert_array_equal(dv, vals)
    np.testing.assert_array_equal(ds[: sb.size], sb)
    exp = np.zeros(n, ">u8")
    exp[ranks] = addr
    assert np.array_equal(np.fromfile(ip, ">u8"), exp)
    expa = np.zeros(n, "<u8")
    expa[ranks] = value8
    assert np.array_equal(np.fromfile(ap, "<u8"), expa)
    solver_report("c3_approx_host_passes_2e8", n, dE)


def big_tmp(tmp_path, need_bytes):
    """A directory with room for the index files: the candidate with the most
    free space among pytest's tmp, /dev/shm, /tmp and the tree's build/.  A box
    without room FAILS the config test (it never skips: VERDICT r2)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    best, free = None, -1
    for d in (str(tmp_path), "/dev/shm", "/tmp", os.path.join(root, "build")):
        try:
            os.makedirs(d, exist_ok=True)
            f = shutil.disk_usage(d).free
        except OSError:
            continue
        if f > free:
            best, free = d, f
    assert free > need_bytes * 1.1, f"no {need_bytes / 1e9:.0f} GB of scratch space for the index files (best {best}: {free / 1e9:.0f} GB)"
    d = tempfile.mkdtemp(dir=best)
    _SCRATCH.append(d)
    return d


_SCRATCH = []


@pytest.fixture(autouse=True)
def _remove_scratch():
    """The multi-GB index files go away even when a test fails (/dev/shm is RAM)."""
    yield
    while _SCRATCH:
        shutil.rmtree(_SCRATCH.pop(), ignore_errors=True)


def records(first, n):
    i = np.arange(first, first + n, dtype=np.uint64)
    addr = np.uint64(0x1000) + np.uint64(48) * i      # SimpleCompact record = 1+2+13+32 B
    value8 = O.splitmix64_np(np.uint64(0xB5DB0002) + i)  # first 8 bytes of the 32-B value (D2)
    return addr, value8, np.full(n, 8, np.uint8)


def full_build_and_index(ctx, tmp_path, n, width, approx, pass_cache):
    keys = O.gen_keys13_mt(0, n, THREADS)
    ctx.set_verify(True)  # on-device check: every key's rank, a permutation of [0, n)
    try:
        mph = ctx.mph_build_fixed(keys, 13, width)
    finally:
        ctx.set_verify(False)
    addr, value8, vlen = records(0, n)
    d = big_tmp(tmp_path, 8 * n * (2 if approx else 1))
    ip, ap = os.path.join(d, "index.db"), os.path.join(d, "index_a.db")
    B = 50_000_000

    def feed(w):
        for lo in range(0, n, B):
            hi = min(n, lo + B)
            w.put_fixed(keys[13 * lo: 13 * hi], 13, addr[lo:hi], value8[lo:hi] if approx else None,
                        vlen[lo:hi] if approx else None)
    passes = mph.write_index(ip, ap, approx, pass_cache, feed)
    assert passes == -(-n // min(n, pass_cache // 8))
    return keys, mph, addr, value8, ip, ap


@pytest.mark.timeout(900)
def test_c2_exact_full_build_1e8(ctx, tmp_path):
    n, width = 100_000_000, 4
    keys, mph, addr, _, ip, ap = full_build_and_index(ctx, tmp_path, n, width, False, 1 << 30)
    E, vals, sb = mph.export()
    # every key: the device's checked getLong == the oracle's lookup on the exported structure
    ranks = mph.lookup_fixed(keys, 13)
    sig = O.hash_fixed_mt(keys, 13, THREADS)
    np.testing.assert_array_equal(ranks, O.lookup_batch_mt(sig, n, E, vals, width, sb, True, THREADS))
    assert np.array_equal(np.bincount(ranks, minlength=n), np.ones(n, np.int64))
    # index.db == the W:129-145 restatement, byte for byte; index_a.db empty
    exp = np.zeros(n, ">u8")
    exp[ranks] = addr
    assert os.path.getsize(ip) == 8 * n
    assert np.array_equal(np.fromfile(ip, ">u8"), exp)
    assert os.path.getsize(ap) == 0
    mph.close()
    # F2 at C2 size: one call (ranks from the solve) writes the same index.db
    ip2 = ip + ".f2"
    m2 = ctx.mph_build_index_fixed(keys, 13, width, addr, ip2)
    for x, y in zip(m2.export(), (E, vals, sb)):
        np.testing.assert_array_equal(x, y)
    assert np.array_equal(np.fromfile(ip2, ">u8"), exp)
    m2.close()
    shutil.rmtree(os.path.dirname(ip), ignore_errors=True)


@pytest.mark.timeout(900)
def test_c3_approx_full_build_1e9(ctx, tmp_path):
    n, width = 1_000_000_000, 4
    # the reference default -ps 1024 (MiB): passSize 2^27 slots, 8 passes (SURVEY.md §8 sizes)
    keys, mph, addr, value8, ip, ap = full_build_and_index(ctx, tmp_path, n, width, True, 1 << 30)
    assert os.path.getsize(ip) == 8 * n and os.path.getsize(ap) == 8 * n
    E, vals, sb = mph.export()
    rng = np.random.default_rng(33)
    s = np.sort(rng.choice(n, 200_000, replace=False))
    skeys = keys.reshape(n, 13)[s].reshape(-1)
    ssig = O.hash_fixed(skeys, 13)
    r = O.lookup_batch_mt(ssig, n, E, vals, width, sb, True, THREADS)
    np.testing.assert_array_equal(mph.lookup_fixed(skeys, 13), r)
    assert r.min() >= 0 and np.unique(r).size == r.size
    idx = np.memmap(ip, ">u8", mode="r")
    ida = np.memmap(ap, "<u8", mode="r")
    np.testing.assert_array_equal(np.asarray(idx[r]), addr[s])
    np.testing.assert_array_equal(np.asarray(ida[r]), value8[s])
    del idx, ida
    mph.close()
    shutil.rmtree(os.path.dirname(ip), ignore_errors=True)
