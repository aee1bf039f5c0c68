"""GPU: the bounded-memory build from host records (bsdb_builder_* and
bsdb_mph_build_index_passes_{fixed,var}) -- keys streamed into HBM, the
bucket-range passes of the C4 one-GPU build, each pass's index slots written
at their file offset.  The files and the MPHF must be byte-identical to the
one-shot F2 build (bsdb_mph_build_index_*) on the same records, which the
round-3 suite pins to the reference's pass loop (W:107-155) and the oracle.

Every address mode is covered: record addresses resident in HBM (stored by
the solve itself, or gathered from the solve's input positions in
approximate mode), gathered from host memory by the writer threads
(BSDB_BUILDER_HOST_GATHER=1, what README-size sets with explicit addresses
take), and addresses as a formula of the add order (fixed-size records)."""
import os
import shutil
import tempfile

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
    torch.cuda.empty_cache()


@pytest.fixture
def host_gather(request):
    on = request.param if hasattr(request, "param") else False
    if on:
        os.environ["BSDB_BUILDER_HOST_GATHER"] = "1"
    yield on
    os.environ.pop("BSDB_BUILDER_HOST_GATHER", None)


def same_files(a, b, chunk=1 << 28):
    if os.path.getsize(a) != os.path.getsize(b):
        return False
    with open(a, "rb") as fa, open(b, "rb") as fb:
        while True:
            x, y = fa.read(chunk), fb.read(chunk)
            if x != y:
                return False
            if not x:
                return True


def same_mph(m1, m2):
    for x, y in zip(m1.export(), m2.export()):
        if (x is None) != (y is None) or (x is not None and not np.array_equal(x, y)):
            return False
    return True


def make_records(n, var, approx, seed=5, first=77):
    rng = np.random.default_rng(seed)
    if var:
        blob, off = O.gen_keys_var(first, n)
        keys = None
    else:
        keys = O.gen_keys13(first, n)
        blob = off = None
    addr = rng.integers(0, 1 << 62, n, dtype=np.uint64)
    value8 = rng.integers(0, 1 << 63, n, dtype=np.uint64) if approx else None
    vlen = rng.integers(0, 9, n).astype(np.uint8) if approx else None
    return keys, blob, off, addr, value8, vlen


def f2_reference(ctx, d, n, var, approx, keys, blob, off, addr, value8, vlen, width=4):
    ip, ap = os.path.join(d, "f2_index.db"), os.path.join(d, "f2_index_a.db")
    if var:
        m = ctx.mph_build_index_var(blob, off, width, addr, ip, ap, approx, value8, vlen)
    else:
        m = ctx.mph_build_index_fixed(keys, 13, width, addr, ip, ap, approx, value8, vlen)
    return m, ip, ap


@pytest.mark.parametrize("host_gather", [False, True], indirect=True)
@pytest.mark.parametrize("var,approx,stride,passes", [
    (False, False, False, 3), (False, True, False, 4), (True, True, False, 3), (True, False, False, 1),
    (False, False, True, 5), (False, True, True, 3), (True, False, True, 2)])
def test_host_passes_equal_one_shot(ctx, tmp_path, host_gather, var, approx, stride, passes):
    n = 400_000
    keys, blob, off, addr, value8, vlen = make_records(n, var, approx)
    if stride:
        addr = np.uint64(0x1000) + np.uint64(48) * np.arange(n, dtype=np.uint64)
    m1, ip1, ap1 = f2_reference(ctx, str(tmp_path), n, var, approx, keys, blob, off, addr, value8, vlen)
    ip2, ap2 = str(tmp_path / "index.db"), str(tmp_path / "index_a.db")
    kw = dict(addr_np=None, addr_base=0x1000, addr_stride=48) if stride else dict(addr_np=addr)
    if var:
        m2, used = ctx.mph_build_index_passes_host(blob, 0, 4, ip2, ap2, approximate=approx, value8_np=value8,
                                                   vlen_np=vlen, passes=passes, offsets_np=off, **kw)
    else:
        m2, used = ctx.mph_build_index_passes_host(keys, 13, 4, ip2, ap2, approximate=approx, value8_np=value8,
                                                   vlen_np=vlen, passes=passes, **kw)
    assert used == passes
    assert same_mph(m1, m2)
    assert same_files(ip1, ip2) and same_files(ap1, ap2)
    assert os.path.getsize(ip2) == 8 * n and os.path.getsize(ap2) == (8 * n if approx else 0)
    m1.close(); m2.close()


@pytest.mark.parametrize("host_gather", [False, True], indirect=True)
@pytest.mark.parametrize("var,approx", [(False, True), (True, False), (True, True)])
def test_streamed_adds_in_any_order(ctx, tmp_path, host_gather, var, approx):
    """The builder fed in uneven batches, in a shuffled batch order, gives the
    same MPHF and files: the MPHF is insertion-order independent and every
    slot gets its own record's address."""
    n = 300_000
    keys, blob, off, addr, value8, vlen = make_records(n, var, approx, seed=9)
    m1, ip1, ap1 = f2_reference(ctx, str(tmp_path), n, var, approx, keys, blob, off, addr, value8, vlen)
    cuts = np.unique(np.concatenate([[0, n], np.random.default_rng(3).integers(0, n, 17)]))
    order = np.random.default_rng(4).permutation(len(cuts) - 1)
    b = ctx.builder(0 if var else 13, key_capacity=n // 3, blob_capacity=1000, approximate=approx)
    for j in order:
        lo, hi = int(cuts[j]), int(cuts[j + 1])
        v8 = value8[lo:hi] if approx else None
        vl = vlen[lo:hi] if approx else None
        if var:
            b.add_var(blob, off[lo:hi + 1], addr[lo:hi], v8, vl)
        else:
            b.add_fixed(keys[13 * lo:13 * hi], 13, addr[lo:hi], v8, vl)
    assert b.count() == n
    ip2, ap2 = str(tmp_path / "index.db"), str(tmp_path / "index_a.db")
    m2, used = b.finish(4, ip2, ap2, passes=3)
    assert used == 3
    assert same_mph(m1, m2)
    assert same_files(ip1, ip2) and same_files(ap1, ap2)
    b.close(); m1.close(); m2.close()


@pytest.mark.parametrize("var", [False, True])
def test_concurrent_adds_from_threads(ctx, tmp_path, var):
    """Round 4: adds from several threads at once (a JVM's put threads) are
    serialised by the builder: the same MPHF and files as one-call build."""
    import threading
    n = 240_000
    keys, blob, off, addr, value8, vlen = make_records(n, var, True, seed=21)
    m1, ip1, ap1 = f2_reference(ctx, str(tmp_path), n, var, True, keys, blob, off, addr, value8, vlen)
    b = ctx.builder(0 if var else 13, key_capacity=n // 4, blob_capacity=1000, approximate=True)
    cuts = np.linspace(0, n, 25).astype(np.int64)
    errors = []

    def worker(t):
        try:
            for j in range(t, len(cuts) - 1, 6):
                lo, hi = int(cuts[j]), int(cuts[j + 1])
                if var:
                    b.add_var(blob, off[lo:hi + 1], addr[lo:hi], value8[lo:hi], vlen[lo:hi])
                else:
                    b.add_fixed(keys[13 * lo:13 * hi], 13, addr[lo:hi], value8[lo:hi], vlen[lo:hi])
        except Exception as e:  # noqa: BLE001 (reported below)
            errors.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors
    assert b.count() == n
    ip2, ap2 = str(tmp_path / "index.db"), str(tmp_path / "index_a.db")
    m2, _ = b.finish(4, ip2, ap2, passes=2)
    assert same_mph(m1, m2)
    assert same_files(ip1, ip2) and same_files(ap1, ap2)
    b.close(); m1.close(); m2.close()


def test_var_builder_with_one_key_length_takes_the_fixed_kernels(ctx, tmp_path):
    """A variable-length builder whose keys all have one length (the kv.db
    scan of fixed-size keys) builds over the fixed-length kernels: same files;
    add_fixed and add_var mix in one builder."""
    n = 200_000
    keys, _, _, addr, _, _ = make_records(n, False, False, seed=11)
    m1, ip1, _ = f2_reference(ctx, str(tmp_path), n, False, False, keys, None, None, addr, None, None)
    b = ctx.builder(0)
    h = n // 2
    b.add_fixed(keys[:13 * h], 13, addr[:h])
    off = (13 * np.arange(n - h + 1, dtype=np.uint64))
    b.add_var(keys[13 * h:], off, addr[h:])
    ip2 = str(tmp_path / "index.db")
    m2, _ = b.finish(4, ip2, None, passes=2)
    assert same_mph(m1, m2) and same_files(ip1, ip2)
    b.close(); m1.close(); m2.close()


def test_builder_errors(ctx, tmp_path):
    from bsdb_amd.native import BsdbError
    keys = O.gen_keys13(0, 1000)
    addr = np.arange(1000, dtype=np.uint64)
    # array mode needs addresses; approximate mode needs value bytes
    b = ctx.builder(13)
    with pytest.raises(BsdbError) as e:
        b.add_fixed(keys, 13, None)
    assert e.value.code == -22
    with pytest.raises(BsdbError):
        b.add_fixed(keys, 12, addr)  # another key length than the builder's
    b.close()
    b = ctx.builder(13, approximate=True)
    with pytest.raises(BsdbError):
        b.add_fixed(keys, 13, addr)
    b.close()
    # a duplicate key fails the finish with EDUP (CBHS:969-972), nothing built
    b = ctx.builder(13)
    b.add_fixed(keys, 13, addr)
    b.add_fixed(keys[:13 * 5], 13, addr[:5])
    with pytest.raises(BsdbError) as e:
        b.finish(4, str(tmp_path / "i.db"), None)
    assert e.value.code == -17
    # a finished builder takes no more adds
    with pytest.raises(BsdbError):
        b.add_fixed(keys, 13, addr)
    b.close()


def test_empty_builder(ctx, tmp_path):
    b = ctx.builder(13)
    m, _ = b.finish(4, str(tmp_path / "i.db"), str(tmp_path / "ia.db"))
    E, _, _ = m.export()
    assert list(E) == [0, 0]
    assert os.path.getsize(tmp_path / "i.db") == 0 and os.path.getsize(tmp_path / "ia.db") == 0
    b.close(); m.close()


_WRITE_FAIL_CHILD = r"""
import resource, signal, sys
import numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[1] + "/oracle"]
import oracle as O
from bsdb_amd.native import BsdbError, Context
signal.signal(signal.SIGXFSZ, signal.SIG_IGN)  # (a write past the limit then fails with EFBIG)
ctx = Context(0)
n = 200_000
keys = O.gen_keys13(0, n)
addr = np.arange(n, dtype=np.uint64)
resource.setrlimit(resource.RLIMIT_FSIZE, (1 << 16, resource.getrlimit(resource.RLIMIT_FSIZE)[1]))
for path in sys.argv[2:]:
    b = ctx.builder(13)
    b.add_fixed(keys, 13, addr)
    try:
        b.finish(4, path, None)
        print("ok", path)
    except BsdbError as e:
        print("code", e.code, path)
    b.close()
"""


def test_index_write_failures_return_efile(tmp_path):
    """an index file the file system cannot hold is an error code,
    not a SIGBUS from a mapped store: a regular file past RLIMIT_FSIZE (its
    size reservation fails, 1.6 MB > 64 KiB) and /dev/full (written with
    pwrite: ENOSPC).  In a child process, which must survive both."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _WRITE_FAIL_CHILD, repo, str(tmp_path / "i.db"), "/dev/full"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [l.split() for l in r.stdout.splitlines() if l.startswith(("ok", "code"))]
    assert lines == [["code", "-9", str(tmp_path / "i.db")], ["code", "-9", "/dev/full"]], r.stdout


def test_index_open_out_of_memory_returns(ctx, tmp_path):
    """bsdb_index_open whose second pass buffer (index_a) cannot be
    allocated must return ENOMEM, not deadlock on the context lock."""
    from bsdb_amd.native import BsdbError
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info()
    n = int(0.6 * free / 8)                     # one 8n buffer fits, two do not
    m = n // 1500 + 1
    E = np.zeros(m + 1, np.uint64)
    from bsdb_amd.native import lib
    vals = np.zeros(int(lib().bsdb_values_words(n)), np.uint64)
    mph = ctx.mph_import(n, 0, E, vals)
    with pytest.raises(BsdbError) as e:
        mph.write_index(str(tmp_path / "i.db"), str(tmp_path / "ia.db"), True, 8 * n, lambda w: None)
    assert e.value.code == -12
    mph.close()
    del E, vals


def big_tmp(need_bytes):
    best, free = None, -1
    for d in ("/tmp", "/dev/shm", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build")):
        try:
            os.makedirs(d, exist_ok=True)
            f = shutil.disk_usage(d).free
        except OSError:
            continue
        if f > free:
            best, free = d, f
    assert free > need_bytes * 1.1, f"no {need_bytes / 1e9:.0f} GB of scratch space (best {best}: {free / 1e9:.0f} GB)"
    return tempfile.mkdtemp(dir=best)


@pytest.mark.timeout(900)
def test_c3_size_host_passes_equal_one_shot():
    """at C3 size (1e9 x 13 B, index.approximate) the host
    passes form with P = 4 writes index.db / index_a.db byte-identical to the
    one-call build, and the same MPHF."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from bsdb_amd import Context
    n = 1_000_000_000
    ctx = Context(0)
    keys = O.gen_keys13_mt(0, n, O.cpu_threads())
    i = np.arange(n, dtype=np.uint64)
    addr = np.uint64(0x1000) + np.uint64(48) * i
    value8 = O.splitmix64_np(np.uint64(0xB5DB0002) + i)
    vlen = np.full(n, 8, np.uint8)
    vlen[::7] = 5
    del i
    d = big_tmp(4 * 8 * n)
    try:
        ip1, ap1 = os.path.join(d, "f2.db"), os.path.join(d, "f2_a.db")
        m1 = ctx.mph_build_index_fixed(keys, 13, 4, addr, ip1, ap1, True, value8, vlen)
        ip2, ap2 = os.path.join(d, "index.db"), os.path.join(d, "index_a.db")
        m2, used = ctx.mph_build_index_passes_host(keys, 13, 4, ip2, ap2, addr_np=addr, approximate=True,
                                                   value8_np=value8, vlen_np=vlen, passes=4)
        assert used == 4
        assert same_mph(m1, m2)
        assert same_files(ip1, ip2) and same_files(ap1, ap2)
        m1.close(); m2.close()
    finally:
        shutil.rmtree(d, ignore_errors=True)
        ctx.close()


@pytest.mark.parametrize("chunk", [None, "997", "0"])
@pytest.mark.parametrize("fmt,var,approx,partitions", [(0, False, False, 4), (0, True, True, 7), (1, True, True, 3),
                                                       (0, False, True, 1)])
def test_kv_streamed_build_equals_in_memory_scan(ctx, tmp_path, monkeypatch, fmt, var, approx, partitions, chunk):
    """F3 in bounded host memory: bsdb_kv_build_index hands
    each kv.db partition to the builder while it is parsed, in chunks of
    BSDB_KV_CHUNK records (default 2 M: one chunk a partition here; 997: many,
    cut anywhere in a partition; 0: one add a partition); its files and MPHF
    equal those of the in-memory scan (bsdb_kv_scan) fed to the one-call
    build."""
    if chunk is not None:
        monkeypatch.setenv("BSDB_KV_CHUNK", chunk)
    from bsdb_amd import kvfiles
    from bsdb_amd.native import kv_scan
    n = 60_000 if fmt == 1 else 250_000
    rng = np.random.default_rng(21)
    if var:
        kb, ko = O.gen_keys_var(3, n)
    else:
        kb = O.gen_keys13(3, n)
        ko = 13 * np.arange(n + 1, dtype=np.uint64)
    vals = [rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8).tobytes() for _ in range(n)]
    vb, vo = kvfiles.pack_values(vals)
    base = str(tmp_path / "kv.db")
    if fmt == 0:
        kvfiles.write_compact(base, partitions, kb, ko, vb, vo)
    else:
        kvfiles.write_blocked(base, partitions, kb, ko, vb, vo, 4096)
    s = kv_scan(base, partitions, fmt, 4096)
    ip1, ap1 = str(tmp_path / "a.db"), str(tmp_path / "a_a.db")
    if s["fixed_len"]:
        m1 = ctx.mph_build_index_fixed(s["blob"], s["fixed_len"], 4, s["addr"], ip1, ap1, approx, s["value8"],
                                       s["vlen"])
    else:
        m1 = ctx.mph_build_index_var(s["blob"], s["offsets"], 4, s["addr"], ip1, ap1, approx, s["value8"], s["vlen"])
    ip2, ap2 = str(tmp_path / "index.db"), str(tmp_path / "index_a.db")
    m2 = ctx.kv_build_index(base, partitions, 4, ip2, ap2, approximate=approx, fmt=fmt, block_size=4096, threads=3)
    assert same_mph(m1, m2)
    assert same_files(ip1, ip2) and same_files(ap1, ap2)
    m1.close(); m2.close()


@pytest.fixture
def device_key_cap(request):
    """BSDB_BUILDER_DEVICE_KEY_BYTES: the builder's device key area capped (read
    at bsdb_builder_open), so adds past it take the spill path."""
    os.environ["BSDB_BUILDER_DEVICE_KEY_BYTES"] = str(request.param)
    yield request.param
    os.environ.pop("BSDB_BUILDER_DEVICE_KEY_BYTES", None)


@pytest.mark.parametrize("device_key_cap", [1_000_000], indirect=True)
@pytest.mark.parametrize("host_gather", [False, True], indirect=True)
@pytest.mark.parametrize("var,approx,stride,threads", [
    (False, False, False, 1), (False, True, False, 3), (True, True, False, 1), (True, False, True, 4),
    (False, False, True, 2)])
def test_spill_mode_equals_one_shot(ctx, tmp_path, device_key_cap, host_gather, var, approx, stride, threads):
    """keys beyond the device key area.  With the key area
    capped at 1 MB, the first adds stay resident, the add that outgrows it
    moves them (hashed on the device) into the 256 host segments of (sig0,
    sig1, add position) by sig0's top byte (CBHS:379-395), and every later add
    is hashed and appended there; the finish uploads each pass's segments.
    MPHF and files byte-identical to the one-shot build."""
    import threading
    n = 300_000
    keys, blob, off, addr, value8, vlen = make_records(n, var, approx, seed=31)
    if stride:
        addr = np.uint64(0x2000) + np.uint64(64) * np.arange(n, dtype=np.uint64)
    m1, ip1, ap1 = f2_reference(ctx, str(tmp_path), n, var, approx, keys, blob, off, addr, value8, vlen)
    kw = dict(addr_base=0x2000, addr_stride=64) if stride else {}
    b = ctx.builder(0 if var else 13, key_capacity=n // 8, blob_capacity=1000, approximate=approx, **kw)
    cuts = np.linspace(0, n, 13).astype(np.int64)
    errors = []

    def worker(t):
        try:
            for j in range(t, len(cuts) - 1, threads):
                lo, hi = int(cuts[j]), int(cuts[j + 1])
                a = None if stride else addr[lo:hi]
                v8 = value8[lo:hi] if approx else None
                vl = vlen[lo:hi] if approx else None
                if var:
                    b.add_var(blob, off[lo:hi + 1], a, v8, vl)
                else:
                    b.add_fixed(keys[13 * lo:13 * hi], 13, a, v8, vl)
        except Exception as e:  # noqa: BLE001 (reported below)
            errors.append(e)

    if stride:  # (addresses by the add order: one thread, in order)
        worker_threads, threads = [threading.Thread(target=worker, args=(0,))], 1
    else:
        worker_threads = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    for t in worker_threads:
        t.start()
    for t in worker_threads:
        t.join()
    assert not errors
    assert b.count() == n
    ip2, ap2 = str(tmp_path / "index.db"), str(tmp_path / "index_a.db")
    m2, used = b.finish(4, ip2, ap2, passes=3)
    assert used == 3
    assert same_mph(m1, m2)
    assert same_files(ip1, ip2) and same_files(ap1, ap2)
    b.close(); m1.close(); m2.close()


@pytest.mark.parametrize("device_key_cap", [1_000_000], indirect=True)
def test_spill_mode_duplicates_and_empty(ctx, tmp_path, device_key_cap):
    from bsdb_amd.native import BsdbError
    keys = O.gen_keys13(0, 200_000)
    addr = np.arange(200_000, dtype=np.uint64)
    b = ctx.builder(13)
    b.add_fixed(keys, 13, addr)                     # 2.6 MB: past the cap, spilled
    b.add_fixed(keys[:13 * 5], 13, addr[:5])
    with pytest.raises(BsdbError) as e:
        b.finish(4, str(tmp_path / "i.db"), None, passes=2)
    assert e.value.code == -17                      # EDUP (CBHS:969-972) found in the spilled segments
    b.close()


@pytest.mark.timeout(900)
def test_spill_build_2e8_keys_equals_resident_build():
    """VERDICT r4 item 6 at size: 2e8 13-byte keys (2.6 GB) through a builder
    whose device key area is capped at 0.8 GB, so ~70 % of the keys are
    spilled to the host segments, added by 4 threads at once, in approximate
    mode with explicit addresses; 4 passes.  The MPHF, index.db and
    index_a.db are byte-identical to the same records' build with every key
    resident in HBM."""
    import threading
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from bsdb_amd import Context
    n = 200_000_000
    ctx = Context(0)
    keys = O.gen_keys13_mt(0, n, O.cpu_threads())
    i = np.arange(n, dtype=np.uint64)
    addr = np.uint64(0x1000) + np.uint64(48) * i
    value8 = O.splitmix64_np(np.uint64(0xB5DB0002) + i)
    vlen = np.full(n, 8, np.uint8)
    vlen[::5] = 3
    del i
    d = big_tmp(4 * 8 * n)
    try:
        ip1, ap1 = os.path.join(d, "resident.db"), os.path.join(d, "resident_a.db")
        m1, used1 = ctx.mph_build_index_passes_host(keys, 13, 4, ip1, ap1, addr_np=addr, approximate=True,
                                                    value8_np=value8, vlen_np=vlen, passes=4)
        os.environ["BSDB_BUILDER_DEVICE_KEY_BYTES"] = str(800_000_000)
        try:
            b = ctx.builder(13, key_capacity=n, approximate=True)
        finally:
            os.environ.pop("BSDB_BUILDER_DEVICE_KEY_BYTES", None)
        cuts = np.linspace(0, n, 41).astype(np.int64)
        errors = []

        def worker(t):
            try:
                for j in range(t, len(cuts) - 1, 4):
                    lo, hi = int(cuts[j]), int(cuts[j + 1])
                    b.add_fixed(keys[13 * lo:13 * hi], 13, addr[lo:hi], value8[lo:hi], vlen[lo:hi])
            except Exception as e:  # noqa: BLE001 (reported below)
                errors.append(e)

        th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errors and b.count() == n
        ip2, ap2 = os.path.join(d, "index.db"), os.path.join(d, "index_a.db")
        m2, used2 = b.finish(4, ip2, ap2, passes=4)
        assert used1 == used2 == 4
        assert same_mph(m1, m2)
        assert same_files(ip1, ip2) and same_files(ap1, ap2)
        b.close(); m1.close(); m2.close()
    finally:
        shutil.rmtree(d, ignore_errors=True)
        ctx.close()
