"""F3: the native kv.db scan (bsdb_kv_scan) over the two uncompressed layouts
of the reference's data files -- host code, CPU only.  The expected records
are the writer's own (bsdb_amd/kvfiles.py restates SimpleCompactKVWriter /
BlockedKVWriter's layouts); the scan must return them in partition order
(PartitionedKVWriter.forEach, one partition after another) with the
addresses the reference's partitionForEach hands to buildIndex
(SimpleCompactKVWriter.java:55-70, BlockedKVWriter.java:84-136)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from bsdb_amd import kvfiles
from bsdb_amd.native import BsdbError, kv_scan


def records(n, seed, key_len=None, big_every=0):
    rng = np.random.default_rng(seed)
    klen = np.full(n, key_len) if key_len else rng.integers(1, 256, n)
    vlen = rng.integers(1, 120, n)
    if big_every:
        vlen[::big_every] = rng.integers(4200, 9000, vlen[::big_every].size)
    koff = np.zeros(n + 1, np.uint64)
    koff[1:] = np.cumsum(klen)
    voff = np.zeros(n + 1, np.uint64)
    voff[1:] = np.cumsum(vlen)
    kblob = rng.integers(0, 256, int(koff[-1]), dtype=np.uint8)
    vblob = rng.integers(0, 256, int(voff[-1]), dtype=np.uint8)
    return kblob, koff, vblob, voff


def expected(kblob, koff, vblob, voff, addr, partitions):
    """Records in scan order: partition by partition, each in file order
    (a large record reaches the file before the block still being filled,
    BlockedKVWriter.java:48-59)."""
    n = koff.size - 1
    per = []
    for p in range(partitions):
        idx = np.arange(p, n, partitions)
        pos = ((addr[idx] >> np.uint64(16)) & np.uint64(0xFFFFFFFF)) * np.uint64(1 << 16) + (addr[idx] & np.uint64(0xFFFF))
        per.append(idx[np.argsort(pos, kind="stable")])
    order = np.concatenate(per).astype(np.int64)
    keys = [kblob[int(koff[i]): int(koff[i + 1])].tobytes() for i in order]
    heads = [vblob[int(voff[i]): int(min(voff[i + 1], voff[i] + 8))].tobytes() for i in order]
    return order, keys, heads


def check(scan, kblob, koff, vblob, voff, addr, partitions):
    order, keys, heads = expected(kblob, koff, vblob, voff, addr, partitions)
    off = scan["offsets"]
    assert off.size == len(keys) + 1
    got_keys = [scan["blob"][int(off[i]): int(off[i + 1])].tobytes() for i in range(len(keys))]
    assert got_keys == keys
    np.testing.assert_array_equal(scan["addr"], addr[order])
    np.testing.assert_array_equal(scan["vlen"], [len(h) for h in heads])
    np.testing.assert_array_equal(scan["value8"], [int.from_bytes(h, "little") for h in heads])


@pytest.mark.parametrize("partitions", [1, 3, 8])
def test_compact_layout(tmp_path, partitions):
    kb, ko, vb, vo = records(20_000, 1)
    base = str(tmp_path / "kv.db")
    addr = kvfiles.write_compact(base, partitions, kb, ko, vb, vo)
    s = kv_scan(base, partitions, 0, threads=4)
    check(s, kb, ko, vb, vo, addr, partitions)
    assert s["fixed_len"] == 0


def test_compact_fixed_keys_and_empty_partitions(tmp_path):
    kb, ko, vb, vo = records(5, 2, key_len=13)
    base = str(tmp_path / "kv.db")
    addr = kvfiles.write_compact(base, 8, kb, ko, vb, vo)   # partitions 5..7 stay empty
    s = kv_scan(base, 8, 0)
    check(s, kb, ko, vb, vo, addr, 8)
    assert s["fixed_len"] == 13
    assert os.path.getsize(base + ".7") == 0


@pytest.mark.parametrize("block", [4096, 8192])
def test_blocked_layout_with_large_records(tmp_path, block):
    kb, ko, vb, vo = records(6_000, 3, big_every=97)
    base = str(tmp_path / "kv.db")
    addr = kvfiles.write_blocked(base, 3, kb, ko, vb, vo, block)
    s = kv_scan(base, 3, 1, block, threads=2)
    check(s, kb, ko, vb, vo, addr, 3)
    # a record's address names its block (pages, position) and offset (BlockedKVWriter.java:124-136)
    a = s["addr"]
    assert set(((a >> np.uint64(48)) & np.uint64(0xFF)).tolist()) >= {block // 4096, 2, 3}


@pytest.mark.parametrize("read", ["mapped", "window"])
def test_files_longer_than_the_read_window(tmp_path, read):
    """Files longer than the 4 MiB read window (capi_kv.hip FileWindow, the
    BSDB_KV_READ=window form; mapped whole by default): records straddling
    the window's end, in both layouts.  The library reads the knob once, so
    the window form runs in a child process."""
    if read == "window" and os.environ.get("BSDB_KV_READ") != "window":
        env = dict(os.environ, BSDB_KV_READ="window")
        r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider",
                            f"{__file__}::test_files_longer_than_the_read_window[window]"],
                           env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        return
    kb, ko, vb, vo = records(60_000, 5)  # ~11 MB in one partition: two refills
    base = str(tmp_path / "kv.db")
    addr = kvfiles.write_compact(base, 1, kb, ko, vb, vo)
    assert os.path.getsize(base + ".0") > 2 * (4 << 20)
    check(kv_scan(base, 1, 0), kb, ko, vb, vo, addr, 1)
    kb, ko, vb, vo = records(30_000, 6, big_every=97)
    base = str(tmp_path / "kvb.db")
    addr = kvfiles.write_blocked(base, 1, kb, ko, vb, vo, 8192)
    assert os.path.getsize(base + ".0") > (4 << 20)
    check(kv_scan(base, 1, 1, 8192), kb, ko, vb, vo, addr, 1)


def test_bad_inputs(tmp_path):
    kb, ko, vb, vo = records(100, 4)
    base = str(tmp_path / "kv.db")
    kvfiles.write_compact(base, 1, kb, ko, vb, vo)
    data = open(base + ".0", "rb").read()
    open(base + ".0", "wb").write(data[:-5])  # a truncated record
    with pytest.raises(BsdbError) as e:
        kv_scan(base, 1, 0)
    assert e.value.code == -9  # EFILE
    with pytest.raises(BsdbError):
        kv_scan(str(tmp_path / "missing.db"), 1, 0)
    with pytest.raises(BsdbError):
        kv_scan(base, 1, 1, 1000)  # block size not a multiple of 4096


def test_blocked_layout_matches_the_reference_writers_bytes(tmp_path):
    """the blocked layout pinned by a byte-level fixture built from
    BlockedKVWriter.java:45-74 (tests/golden/make_blocked_fixture.py): a large
    record written before the block still pending, blocks after a longer one
    carrying its stale bytes past their 0 end mark.  The scan returns the
    reference's partitionForEach stream (file order, addresses :124-136; the
    large record's value is read where the reference hands null), and the
    test writer's file of the same records scans to the same stream."""
    g = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "blocked_kv_v1.npz"), allow_pickle=False))
    bs = int(g["block_size"][0])
    base = str(tmp_path / "kv.db")
    g["file0"].tofile(base + ".0")
    open(base + ".1", "wb").close()                  # an empty partition
    s = kv_scan(base, 2, 1, bs, threads=2)
    np.testing.assert_array_equal(s["addr"], g["addr"])
    np.testing.assert_array_equal(s["offsets"], g["key_off"])
    np.testing.assert_array_equal(s["blob"], g["keys"])
    np.testing.assert_array_equal(s["value8"], g["value8"])
    np.testing.assert_array_equal(s["vlen"], g["vlen"])
    # kvfiles (the tests' writer) on the same records, written in the fixture's
    # put order (r0, r1, r2, r3 = scan order 1, 0, 2, 3): same scan stream
    put = [1, 0, 2, 3]
    ko, vo = g["key_off"].astype(np.int64), g["value_off"].astype(np.int64)
    kb = np.concatenate([g["keys"][ko[i]:ko[i + 1]] for i in put])
    vb = np.concatenate([g["values"][vo[i]:vo[i + 1]] for i in put])
    kl = np.cumsum([0] + [ko[i + 1] - ko[i] for i in put]).astype(np.uint64)
    vl = np.cumsum([0] + [vo[i + 1] - vo[i] for i in put]).astype(np.uint64)
    base2 = str(tmp_path / "mine.db")
    kvfiles.write_blocked(base2, 1, kb, kl, vb, vl, bs)
    s2 = kv_scan(base2, 1, 1, bs)
    np.testing.assert_array_equal(s2["addr"], g["addr"])
    np.testing.assert_array_equal(s2["blob"], g["keys"])
    f2 = np.fromfile(base2 + ".0", np.uint8)
    assert f2.size == g["file0"].size
    # every byte up to each block's end mark agrees (the tails past it are unspecified)
    np.testing.assert_array_equal(f2[:5013], g["file0"][:5013])
