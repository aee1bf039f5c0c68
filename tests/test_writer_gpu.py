"""GPU: the BSDBWriter mirror end to end -- put -> build -> the reference's
file set -- read back the way the serve path reads it (Reader.getLong ->
index.db slot -> kv.db record -> key compare, SyncReader.java:44-57), in
the style of BSDBWriterTest.runBuildAndRead (BSDBWriterTest.java:31-134)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def read_record(base, addr):
    p, off = addr >> 56, addr & ((1 << 56) - 1)
    with open(os.path.join(base, f"kv.db.{p}"), "rb") as f:
        f.seek(off)
        h = f.read(3)
        kl, vl = h[0], int.from_bytes(h[1:3], "big")
        return f.read(kl), f.read(vl)


@pytest.mark.parametrize("approx,partitions,pass_cache,fused,files", [
    (False, 3, 8 * 40_000, False, False), (True, 1, 1 << 30, False, False), (True, 2, 0, False, False),
    (True, 2, 0, True, False), (False, 1, 0, True, False), (True, 3, 0, True, True), (False, 4, 0, True, True)])
def test_build_and_read_back(tmp_path, approx, partitions, pass_cache, fused, files):
    """files: the index built from the data files through the native kv.db
    scan (bsdb_kv_build_index, F3) instead of the records held in memory."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from bsdb_amd.writer import BSDBWriter
    n = 100_000
    rng = np.random.default_rng(1)
    keys = [str(i).encode() for i in range(1, n + 1)]  # BSDBWriterTest keys "1".."n"
    vals = [rng.integers(0, 256, int(rng.integers(1, 60)), dtype=np.uint8).tobytes() for _ in range(n)]
    base = str(tmp_path / "db")
    w = BSDBWriter(base, checksum_bits=4, pass_cache_size=pass_cache, approximate_mode=approx,
                   partitions=partitions, fused_index=fused, from_files=files)
    for k, v in zip(keys[: n // 2], vals[: n // 2]):
        w.put(k, v)
    rest = keys[n // 2:]
    off = np.zeros(len(rest) + 1, np.uint64)
    off[1:] = np.cumsum([len(k) for k in rest])
    w.put_batch(np.frombuffer(b"".join(rest), np.uint8), off, vals[n // 2:])
    mph = w.build()
    for f in ("config.properties", "hash.dump", "index.db", "index_a.db"):
        assert os.path.exists(os.path.join(base, f)), f
    cfg = open(os.path.join(base, "config.properties")).read()
    assert f"kv.count = {n}" in cfg and f"index.approximate = {str(approx).lower()}" in cfg
    idx = np.fromfile(os.path.join(base, "index.db"), ">u8")
    assert idx.size == n
    blob = np.frombuffer(b"".join(keys), np.uint8)
    koff = np.zeros(n + 1, np.uint64)
    koff[1:] = np.cumsum([len(k) for k in keys])
    r = mph.lookup_var(blob, koff, check=True)
    assert np.array_equal(np.sort(r), np.arange(n))
    for i in np.random.default_rng(2).choice(n, 3000, replace=False):
        k, v = read_record(base, int(idx[r[i]]))
        assert k == keys[i] and v == vals[i]
    ia = np.fromfile(os.path.join(base, "index_a.db"), np.uint8)
    if approx:
        ia = ia.reshape(n, 8)
        for i in range(0, n, 997):
            head = vals[i][:8]
            assert ia[r[i]].tobytes() == head + bytes(8 - len(head))
    else:
        assert ia.size == 0
    # absent keys: checksum rejects (-1) or the stored key differs (null)
    absent = [b"a" + str(i).encode() for i in range(10_000)]
    ab = np.frombuffer(b"".join(absent), np.uint8)
    ao = np.zeros(len(absent) + 1, np.uint64)
    ao[1:] = np.cumsum([len(k) for k in absent])
    ra = mph.lookup_var(ab, ao, check=True)
    for j in np.flatnonzero(ra >= 0):
        k, _ = read_record(base, int(idx[ra[j]]))
        assert k != absent[j]
    assert (ra >= 0).mean() < 0.1  # ~1/16 false positives at 4 checksum bits
    mph.close()
    w.close()


@pytest.mark.parametrize("var,approx,n", [(False, False, 200_000), (True, True, 150_000), (False, True, 1)])
def test_build_index_in_one_call_equals_the_pass_loop(tmp_path, var, approx, n):
    """F2 (bsdb_mph_build_index_*): the index files from the solve's ranks are
    byte-identical to the reference's pass loop (lookup per record, W:129-145)
    over the same records, and the MPHF is the same."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import oracle as O
    from bsdb_amd import Context
    ctx = Context(0)
    rng = np.random.default_rng(5)
    if var:
        blob, off = O.gen_keys_var(0, n)
    else:
        keys = O.gen_keys13(77, n)
    addr = rng.integers(0, 1 << 62, n, dtype=np.uint64)
    value8 = rng.integers(0, 1 << 63, n, dtype=np.uint64) if approx else None
    vlen = rng.integers(0, 9, n).astype(np.uint8) if approx else None
    d1, d2 = tmp_path / "fused", tmp_path / "loop"
    d1.mkdir(); d2.mkdir()
    ip1, ap1, ip2, ap2 = (str(d / f) for d in (d1, d2) for f in ("index.db", "index_a.db"))
    if var:
        m1 = ctx.mph_build_index_var(blob, off, 4, addr, ip1, ap1, approx, value8, vlen)
        m2 = ctx.mph_build_var(blob, off, 4)
    else:
        m1 = ctx.mph_build_index_fixed(keys, 13, 4, addr, ip1, ap1, approx, value8, vlen)
        m2 = ctx.mph_build_fixed(keys, 13, 4)
    for a, b in zip(m1.export(), m2.export()):
        np.testing.assert_array_equal(a, b)
    B = 64_000

    def feed(w):
        for lo in range(0, n, B):
            hi = min(n, lo + B)
            v8 = value8[lo:hi] if approx else None
            vl = vlen[lo:hi] if approx else None
            if var:
                w.put_var(blob, off[lo: hi + 1], addr[lo:hi], v8, vl)
            else:
                w.put_fixed(keys[13 * lo: 13 * hi], 13, addr[lo:hi], v8, vl)
    passes = m2.write_index(ip2, ap2, approx, 8 * 70_000, feed)
    assert passes == -(-n // min(n, 70_000))
    for a, b in ((ip1, ip2), (ap1, ap2)):
        assert open(a, "rb").read() == open(b, "rb").read()
    assert os.path.getsize(ip1) == 8 * n and os.path.getsize(ap1) == (8 * n if approx else 0)
    m1.close(); m2.close(); ctx.close()


@pytest.mark.parametrize("block", [4096, 8192])
def test_kv_build_from_blocked_files(tmp_path, block):
    """F3 over SimpleBlockedKVWriter's layout (large records included): the
    scan's addresses land in index.db at each key's rank; read back through
    the block address (BlockedKVWriter.java:124-136)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import oracle as O
    from bsdb_amd import Context, kvfiles
    n = 30_000
    rng = np.random.default_rng(8)
    kb, ko = O.gen_keys_var(5, n)
    vals = [rng.integers(0, 256, int(rng.integers(1, 200)) if i % 53 else 5000, dtype=np.uint8).tobytes()
            for i in range(n)]
    vb, vo = kvfiles.pack_values(vals)
    base = str(tmp_path / "kv.db")
    addr = kvfiles.write_blocked(base, 3, kb, ko, vb, vo, block)
    ctx = Context(0)
    ip, ap = str(tmp_path / "index.db"), str(tmp_path / "index_a.db")
    mph = ctx.kv_build_index(base, 3, 4, ip, ap, approximate=True, fmt=1, block_size=block)
    r = mph.lookup_var(kb, ko, check=True)
    assert np.array_equal(np.sort(r), np.arange(n))
    idx = np.fromfile(ip, ">u8")
    np.testing.assert_array_equal(idx[r], addr)
    ia = np.fromfile(ap, np.uint8).reshape(n, 8)
    for i in range(0, n, 211):
        head = vals[i][:8]
        assert ia[r[i]].tobytes() == head + bytes(8 - len(head))
    mph.close()
    ctx.close()


def test_empty_key_set(tmp_path):
    """n = 0 (a writer with no records): m = 1, E = [0, 0], empty index files,
    through both the pass loop and the one-call form."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from bsdb_amd import Context
    ctx = Context(0)
    keys = np.zeros(0, np.uint8)
    addr = np.zeros(0, np.uint64)
    m1 = ctx.mph_build_index_fixed(keys, 13, 4, addr, str(tmp_path / "a.db"), str(tmp_path / "aa.db"))
    E, vals, sb = m1.export()
    assert list(E) == [0, 0]
    assert os.path.getsize(tmp_path / "a.db") == 0 and os.path.getsize(tmp_path / "aa.db") == 0
    m2 = ctx.mph_build_fixed(keys, 13, 4)
    passes = m2.write_index(str(tmp_path / "b.db"), str(tmp_path / "ba.db"), False, 1 << 30, lambda w: None)
    assert passes == 0 and os.path.getsize(tmp_path / "b.db") == 0
    m2.dump(str(tmp_path / "h.dump"))
    m3 = ctx.mph_load(str(tmp_path / "h.dump"))
    assert list(m3.export()[0]) == [0, 0]
    for m in (m1, m2, m3):
        m.close()
    ctx.close()


@pytest.mark.parametrize("G,var,approx,width,n", [(2, False, False, 4, 1_000_000), (3, True, True, 4, 300_000),
                                                  (4, False, True, 7, 50_000), (3, False, False, 4, 10),
                                                  (2, False, False, 64, 0), (2, True, False, 0, 120_000)])
def test_multi_device_full_build_equals_one_device(tmp_path, G, var, approx, width, n):
    """E4 behind the C ABI (bsdb_multi_mph_build_index_*): the key set sharded
    over G device contexts (this box's one GPU listed G times -- the exchange
    is then a copy within it), bucket-range owners, one exchange, range
    solves, slices written in place.  The structure and the files equal the
    one-device F2 build byte for byte; with more devices than buckets (n = 10)
    the empty ranges do nothing."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import oracle as O
    from bsdb_amd import Context
    from bsdb_amd.native import Multi
    rng = np.random.default_rng(11)
    if var:
        blob, off = O.gen_keys_var(3, n)
    else:
        keys = O.gen_keys13(91, n)
    addr = rng.integers(0, 1 << 62, n, dtype=np.uint64)
    value8 = rng.integers(0, 1 << 63, n, dtype=np.uint64) if approx else None
    vlen = rng.integers(0, 9, n).astype(np.uint8) if approx else None
    index = width != 0
    d1, d2 = tmp_path / "one", tmp_path / "multi"
    d1.mkdir(); d2.mkdir()
    ip1, ap1, ip2, ap2 = (str(d / f) for d in (d1, d2) for f in ("index.db", "index_a.db"))
    with Context(0) as ctx:
        if var:
            m1 = ctx.mph_build_index_var(blob, off, width, addr, ip1, ap1, approx, value8, vlen)
        else:
            m1 = ctx.mph_build_index_fixed(keys, 13, width, addr, ip1, ap1, approx, value8, vlen)
        ref = m1.export()
        m1.close()
    with Multi(G, [0] * G) as mc:
        args = (addr, ip2 if index else None, ap2 if index else None, approx, value8, vlen)
        got = mc.mph_build_index_var(blob, off, width, *args) if var else mc.mph_build_index_fixed(keys, 13, width, *args)
    for a, b in zip(got, ref):
        if a is None or b is None:
            assert a is None and b is None
        else:
            np.testing.assert_array_equal(a, b)
    if index:
        for a, b in ((ip1, ip2), (ap1, ap2)):
            assert open(a, "rb").read() == open(b, "rb").read()
        assert os.path.getsize(ip2) == 8 * n and os.path.getsize(ap2) == (8 * n if approx else 0)


def test_multi_device_full_build_rejects_duplicates(tmp_path):
    """A key repeated in two shards meets itself at its bucket's owner: the
    multi-device build reports the duplicate (BSDB_EDUP, CBHS:969-972) like
    the one-device build."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import oracle as O
    from bsdb_amd.native import BsdbError, Multi
    n = 200_000
    keys = O.gen_keys13(5, n).copy()
    keys[13 * (n - 1): 13 * n] = keys[0:13]  # the last key (shard 2) == the first (shard 1)
    addr = np.arange(n, dtype=np.uint64)
    with Multi(2, [0, 0]) as mc:
        with pytest.raises(BsdbError) as e:
            mc.mph_build_index_fixed(keys, 13, 4, addr, str(tmp_path / "i.db"))
        assert e.value.code == -17
        E, vals, sb = mc.mph_build_index_fixed(keys[: 13 * (n - 1)], 13, 4)  # the same contexts build after it
    assert E[-1] == n - 1


@pytest.mark.parametrize("devices", [None, [0, 0, 0]])
def test_concurrent_puts_and_multi_device_writer(tmp_path, devices):
    """put() from an 8-thread pool, as the reference's Builder calls it
    (Builder.java:144-160, BSDBWriterTest.java:60-78): every record reads back
    through index.db -> kv.db; with devices=[...] the writer's one-call build
    runs over several device contexts (E4) and the files are the same."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from concurrent.futures import ThreadPoolExecutor
    from bsdb_amd.writer import BSDBWriter
    n = 60_000
    keys = [str(i).encode() for i in range(1, n + 1)]
    vals = [(b"v%d-" % i) * (1 + i % 7) for i in range(n)]
    base = str(tmp_path / "db")
    w = BSDBWriter(base, checksum_bits=4, approximate_mode=True, partitions=2, fused_index=True, devices=devices)
    with ThreadPoolExecutor(8) as ex:
        list(ex.map(lambda i: w.put(keys[i], vals[i]), range(n)))
    mph = w.build()
    idx = np.fromfile(os.path.join(base, "index.db"), ">u8")
    blob = np.frombuffer(b"".join(keys), np.uint8)
    koff = np.zeros(n + 1, np.uint64)
    koff[1:] = np.cumsum([len(k) for k in keys])
    r = mph.lookup_var(blob, koff, check=True)
    assert np.array_equal(np.sort(r), np.arange(n))
    ia = np.fromfile(os.path.join(base, "index_a.db"), np.uint8).reshape(n, 8)
    for i in range(0, n, 101):
        k, v = read_record(base, int(idx[r[i]]))
        assert k == keys[i] and v == vals[i]
        assert ia[r[i]].tobytes() == vals[i][:8].ljust(8, b"\0")
    mph.close()
    w.close()
