"""Minimal writers of the two uncompressed kv.db layouts the index build scans
(the data-file formats themselves are out of scope: the north star leaves
them untouched; these produce the files and the record addresses that
bsdb_kv_scan / the index stage consume, for the writer mirror, the tests and
the end-to-end bench).

  compact  SimpleCompactKVWriter (src/main/java/tech/bsdb/write/
           SimpleCompactKVWriter.java:36-42): records [kLen u8][vLen u16 BE]
           [key][value] back to back in kv.db.<p>; address = p << 56 | offset
  blocked  SimpleBlockedKVWriter / BlockedKVWriter (BlockedKVWriter.java:
           36-82): records packed into block_size blocks, a 0 byte after a
           block's last record when room is left, a record longer than a block
           flushed at once into a page-aligned block of its own; address = p <<
           56 | block pages << 48 | block position in pages << 16 | offset

Record i goes to partition i % partitions (the reference picks the next free
partition lock, PartitionedKVWriter.java:82-96: any assignment is valid).
"""
from __future__ import annotations

import os

import numpy as np

RECORD_HEADER = 3
PAGE = 4096


def _ranges(starts: np.ndarray, lens: np.ndarray) -> np.ndarray:
    """Concatenated index ranges [starts[i], starts[i] + lens[i])."""
    lens = lens.astype(np.int64)
    total = int(lens.sum())
    if total == 0:
        return np.zeros(0, np.int64)
    rep = np.repeat(starts.astype(np.int64) - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens)
    return rep + np.arange(total, dtype=np.int64)


def write_compact(base: str, partitions: int, kblob, koff, vblob, voff) -> np.ndarray:
    """Writes base.<p> for p < partitions; returns every record's address."""
    koff = np.asarray(koff, np.uint64).astype(np.int64)
    voff = np.asarray(voff, np.uint64).astype(np.int64)
    kblob = np.asarray(kblob, np.uint8)
    vblob = np.asarray(vblob, np.uint8)
    n = koff.size - 1
    klen, vlen = np.diff(koff), np.diff(voff)
    if n and (klen.min() < 1 or klen.max() > 255 or vlen.max() > 0xFFFF):
        raise ValueError("key length 1..255, value length < 65536")
    addr = np.zeros(n, np.uint64)
    for p in range(partitions):
        idx = np.arange(p, n, partitions)
        size = RECORD_HEADER + klen[idx] + vlen[idx]
        pos = np.concatenate([[0], np.cumsum(size)[:-1]]).astype(np.int64) if idx.size else np.zeros(0, np.int64)
        out = np.zeros(int(size.sum()) if idx.size else 0, np.uint8)
        if idx.size:
            out[pos] = klen[idx]
            out[pos + 1] = vlen[idx] >> 8
            out[pos + 2] = vlen[idx] & 0xFF
            out[_ranges(pos + 3, klen[idx])] = kblob[_ranges(koff[idx], klen[idx])]
            out[_ranges(pos + 3 + klen[idx], vlen[idx])] = vblob[_ranges(voff[idx], vlen[idx])]
            addr[idx] = (np.uint64(p) << np.uint64(56)) | pos.astype(np.uint64)
        out.tofile(f"{base}.{p}")
    return addr


def write_blocked(base: str, partitions: int, kblob, koff, vblob, voff, block_size: int = PAGE) -> np.ndarray:
    """BlockedKVWriter's layout, record by record (test sizes); returns addresses."""
    if block_size % PAGE:
        raise ValueError("block size must be a multiple of 4096")
    koff = np.asarray(koff, np.uint64)
    voff = np.asarray(voff, np.uint64)
    n = koff.size - 1
    addr = np.zeros(n, np.uint64)
    for p in range(partitions):
        with open(f"{base}.{p}", "wb") as f:
            buf = bytearray()        # the partition's write buffer (one block)
            pending = []             # (offset in block, record index)
            fpos = 0                 # file position of the next block written

            def flush_block():
                nonlocal buf, pending, fpos
                if not buf:
                    return
                if len(buf) < block_size:
                    buf.append(0)    # end of the block's records
                blk = bytes(buf) + bytes(block_size - len(buf))
                for o, i in pending:
                    addr[i] = (p << 56) | ((block_size // PAGE) << 48) | ((fpos // PAGE) << 16) | o
                f.write(blk)
                fpos += block_size
                buf, pending = bytearray(), []

            for i in range(p, n, partitions):
                k = kblob[int(koff[i]): int(koff[i + 1])].tobytes()
                v = vblob[int(voff[i]): int(voff[i + 1])].tobytes()
                rec = bytes([len(k)]) + len(v).to_bytes(2, "big") + k + v
                if len(rec) > block_size:    # a large record: its own page-aligned block, at once
                    size = -(-len(rec) // PAGE) * PAGE
                    blk = rec + (b"\0" if len(rec) < size else b"")
                    f.write(blk + bytes(size - len(blk)))
                    addr[i] = (p << 56) | ((size // PAGE) << 48) | ((fpos // PAGE) << 16)
                    fpos += size
                    continue
                if block_size - len(buf) < len(rec):
                    flush_block()
                pending.append((len(buf), i))
                buf += rec
            flush_block()
    return addr


def pack_values(values) -> tuple:
    """list of bytes -> (blob, offsets)."""
    off = np.zeros(len(values) + 1, np.uint64)
    if values:
        off[1:] = np.cumsum([len(v) for v in values])
    return np.frombuffer(b"".join(values), np.uint8) if values else np.zeros(0, np.uint8), off
