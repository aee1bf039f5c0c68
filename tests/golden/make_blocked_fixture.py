#!/usr/bin/env python3
"""Writes tests/golden/blocked_kv_v1.npz: the bytes SimpleBlockedKVWriter
(src/main/java/tech/bsdb/write/BlockedKVWriter.java:45-74, SimpleBlockedKVWriter
.java:37-40) puts in kv.db.0 for one hand-picked record sequence, and the
(address, key, value) stream its partitionForEach (BlockedKVWriter.java:84-121,
address :124-136) hands to buildIndex.  The Java is not runnable here (no JDK),
so the bytes are assembled step by step below from those lines, including
what a reused direct ByteBuffer leaves behind: clear() resets the position
without zeroing, so a block written after a longer one carries the longer
one's stale bytes past its 0 end mark (BlockedKVWriter.java:58-61,66-74).

Sequence (block size 4096, partition 0):
  r0 small            -> pending in the block buffer
  r1 larger than a block -> written AT ONCE in its own page-aligned block
                          (before the pending block, :47-55)
  r2 does not fit beside r0 -> the pending block (r0) is flushed, r2 starts a new one
  r3 does not fit beside r2 -> r2's block flushed, r3 starts a new one
  end of partition    -> r3's block flushed with r2's stale bytes after its mark
"""
import os

import numpy as np

PAGE = 4096
BLOCK = 4096


def rec(key: bytes, value: bytes) -> bytes:      # BaseKVWriter.java:44-49
    return bytes([len(key)]) + len(value).to_bytes(2, "big") + key + value


def main():
    rng = np.random.default_rng(1234)
    recs = [(b"alpha", rng.integers(0, 256, 10, dtype=np.uint8).tobytes()),
            (b"LARGE", rng.integers(1, 256, 5000, dtype=np.uint8).tobytes()),
            (b"bb", rng.integers(1, 256, 4080, dtype=np.uint8).tobytes()),
            (b"c3", rng.integers(0, 256, 20, dtype=np.uint8).tobytes())]
    out = bytearray()
    buf = bytearray(BLOCK)                       # the partition's direct buffer (zeroed once)
    pos = 0

    def flush_block():                           # flushBlocks (:66-74) + flushBlocks0 (channel.write)
        nonlocal pos
        if pos > 0:
            if pos < BLOCK:
                buf[pos] = 0                     # "mark data finished"
            out.extend(buf)                      # position(0), limit(capacity): the WHOLE buffer
    # r0 (:57-61): fits the empty buffer
    r = rec(*recs[0]); buf[pos:pos + len(r)] = r; pos += len(r)
    # r1 (:47-55): large -> a fresh page-aligned buffer, written now
    r = rec(*recs[1]); size = -(-len(r) // PAGE) * PAGE
    big = bytearray(size); big[:len(r)] = r
    if len(r) < size:
        big[len(r)] = 0
    out.extend(big)
    # r2: remaining < recLen -> flush, clear (no zeroing), write at 0
    r = rec(*recs[2]); assert BLOCK - pos < len(r)
    flush_block(); pos = 0
    buf[pos:pos + len(r)] = r; pos += len(r)
    # r3: same
    r = rec(*recs[3]); assert BLOCK - pos < len(r)
    flush_block(); pos = 0
    buf[pos:pos + len(r)] = r; pos += len(r)
    flush_block()                                # flushPartition (:40-43)
    # the scan's stream, in file order (partitionForEach), addresses per :124-136
    def addr(block_bytes, block_pos, off):
        return (0 << 56) | (block_bytes // PAGE) << 48 | (block_pos // PAGE) << 16 | off
    order = [1, 0, 2, 3]
    addrs = [addr(8192, 0, 0), addr(BLOCK, 8192, 0), addr(BLOCK, 8192 + BLOCK, 0), addr(BLOCK, 8192 + 2 * BLOCK, 0)]
    keys = b"".join(recs[i][0] for i in order)
    koff = np.cumsum([0] + [len(recs[i][0]) for i in order]).astype(np.uint64)
    v8 = np.array([int.from_bytes(recs[i][1][:8], "little") for i in order], np.uint64)
    vlen = np.array([min(8, len(recs[i][1])) for i in order], np.uint8)
    assert len(out) == 8192 + 3 * BLOCK
    assert bytes(out[8192 + 2 * BLOCK + 26: 8192 + 3 * BLOCK]) == bytes(buf[26:]) != bytes(BLOCK - 26)  # stale tail
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "blocked_kv_v1.npz"),
                        file0=np.frombuffer(bytes(out), np.uint8), block_size=np.array([BLOCK]),
                        addr=np.array(addrs, np.uint64), keys=np.frombuffer(keys, np.uint8), key_off=koff,
                        value8=v8, vlen=vlen,
                        values=np.frombuffer(b"".join(recs[i][1] for i in order), np.uint8),
                        value_off=np.cumsum([0] + [len(recs[i][1]) for i in order]).astype(np.uint64))


if __name__ == "__main__":
    main()
