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


@pytest.mark.parametrize("approx,partitions,pass_cache", [(False, 3, 8 * 40_000), (True, 1, 1 << 30), (True, 2, 0)])
def test_build_and_read_back(tmp_path, approx, partitions, pass_cache):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from bsdb_amd.writer import BSDBWriter
    n = 100_000
    rng = np.random.default_rng(1)
    keys = [str(i).encode() for i in range(1, n + 1)]  # BSDBWriterTest keys "1".."n"
    vals = [rng.integers(0, 256, int(rng.integers(1, 60)), dtype=np.uint8).tobytes() for _ in range(n)]
    base = str(tmp_path / "db")
    w = BSDBWriter(base, checksum_bits=4, pass_cache_size=pass_cache, approximate_mode=approx,
                   partitions=partitions)
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
