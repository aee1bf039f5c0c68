"""Host-side mirror of the reference's BSDBWriter (the drop-in seam, B1/B2).

``BSDBWriter`` keeps the reference constructor's arguments and the call
sequence put* -> build() = buildHash() + buildIndex(), and produces the same
file set in ``base_path`` (src/main/java/tech/bsdb/write/BSDBWriter.java, "W"):

  kv.db.<p>          records [kLen u8][vLen u16 BE][key][value] of
                     SimpleCompactKVWriter (SimpleCompactKVWriter.java:36-42;
                     the kv.db format is out of scope, this is the minimal
                     writer that produces the record addresses the index needs:
                     addr = p << 56 | byte offset, :62-73)
  config.properties  the keys BSDBWriter sets (W:54-58) + record statistics
  hash.dump          the MPHF in GOV.dump's raw layout (GOV:592-619), the
                     layout the reference's own load_mph reads (mph.c:28-43);
                     hash.db itself is a Java-serialized object that the Java
                     host writes from the same arrays
  index.db           big-endian record address per rank (W:107-155)
  index_a.db         approximate mode: first <= 8 value bytes per rank;
                     created empty otherwise (W:126)

Every compute step is the C ABI (bsdb_mph_build_var, bsdb_index_*): no CPU
fallback.  ``fused_index=True`` builds hash + index in one call whose solve
returns every key's rank (bsdb_mph_build_index_var): no
per-pass rescan, the same files.  ``devices=[...]`` makes that one call the
multi-device build over those GPUs (bsdb_multi_mph_build_index_var, E4).
``from_files=True`` builds from the data files it wrote instead: the native
kv.db scan (bsdb_kv_build_index, F3) reads every kv.db.<p> back as
buildIndex's kvWriter.forEach does (W:134) and runs the same one-call build.
``put`` is per record and safe to call from concurrent threads, as the
reference's Builder does (Builder.java:144-160); ``put_batch`` takes a whole
key blob at once.  The kv.db writer is the minimal compact layout of
bsdb_amd/kvfiles.py (numpy, whole arrays): a test and bench harness for the
index path, not a replacement of the reference's KV writers.
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np

from . import kvfiles
from .native import Context, Mph

SLOT_SIZE = 8          # Common.java SLOT_SIZE
MAX_KEY_SIZE = 255     # Common.java MAX_KEY_SIZE
RECORD_HEADER = 3      # Common.java RECORD_HEADER_SIZE


class BSDBWriter:
    def __init__(self, base_path: str, tmp_dir: Optional[str] = None, checksum_bits: int = 4,
                 pass_cache_size: int = 1 << 30, compact: bool = True, compress: bool = False,
                 compress_block_size: int = 8192, shared_dict_size: int = 0, approximate_mode: bool = False,
                 partitions: int = 1, device: int = 0, fused_index: bool = False, devices=None,
                 from_files: bool = False):
        if compress or not compact:
            raise NotImplementedError("only the compact kv.db layout is mirrored (kv.db formats are out of scope)")
        self.base = base_path
        os.makedirs(base_path, exist_ok=True)
        self.checksum_bits = checksum_bits
        self.pass_cache_size = pass_cache_size
        self.approximate = approximate_mode
        self.partitions = partitions
        self.compress_block_size = compress_block_size
        self.fused_index = fused_index or devices is not None or from_files
        self.from_files = from_files
        self.devices = list(devices) if devices is not None else None
        self._puts: list = []  # (key, value) pairs: one list.append per put, atomic across threads
        self._batches: list = []  # (blob, offsets, value8, vlen, value bytes total)
        self.ctx = Context(device)

    # W:75-89
    def put(self, key: bytes, value: bytes):
        if key is None or value is None:
            raise RuntimeError("currently null key/value is not support.")
        if not 0 < len(key) <= MAX_KEY_SIZE:
            raise ValueError("key length must be 1..255 bytes")
        self._puts.append((bytes(key), bytes(value)))

    def put_batch(self, blob: np.ndarray, offsets: np.ndarray, values: list):
        """Keys blob[offsets[i]:offsets[i+1]] with values[i] (bytes each)."""
        off = np.ascontiguousarray(offsets, np.uint64)
        lens = np.diff(off)
        if lens.size and (lens.min() == 0 or lens.max() > MAX_KEY_SIZE):
            raise ValueError("key length must be 1..255 bytes")
        if len(values) != lens.size:
            raise ValueError("one value per key")
        self._batches.append((np.ascontiguousarray(blob, np.uint8), off, list(values)))

    def _records(self):
        """All records as (key blob, offsets, values list)."""
        blobs, offs, vals, base = [], [np.zeros(1, np.uint64)], [], 0
        if self._puts:
            keys = [k for k, _ in self._puts]
            lens = np.fromiter((len(k) for k in keys), np.uint64, len(keys))
            blobs.append(np.frombuffer(b"".join(keys), np.uint8))
            offs.append(np.cumsum(lens, dtype=np.uint64))
            vals += [v for _, v in self._puts]
            base = int(offs[-1][-1])
        for blob, off, v in self._batches:
            blobs.append(blob[int(off[0]): int(off[-1])])
            offs.append(off[1:] - off[0] + np.uint64(base))
            vals += v
            base += int(off[-1] - off[0])
        blob = np.concatenate(blobs) if blobs else np.zeros(0, np.uint8)
        return blob, np.concatenate(offs), vals

    def _write_kv(self, blob, off, vals):
        """kv.db.<p>: record i goes to partition i % partitions; returns addresses."""
        vblob, voff = kvfiles.pack_values(vals)
        self._vblob, self._voff = vblob, voff
        return kvfiles.write_compact(os.path.join(self.base, "kv.db"), self.partitions, blob, off, vblob, voff)

    def _write_config(self, off, vals):
        n = off.size - 1
        klen = np.diff(off)
        vlen = np.fromiter((len(v) for v in vals), np.int64, n)
        props = {
            "kv.compressed": "false", "kv.compact": "true", "kv.compress.block.size": self.compress_block_size,
            "index.approximate": str(self.approximate).lower(), "hash.checksum.bits": self.checksum_bits,
            "kv.count": n, "kv.key.len.max": int(klen.max()) if n else 0,
            "kv.key.len.avg": float(klen.mean()) if n else 0.0, "kv.value.len.max": int(vlen.max()) if n else 0,
            "kv.value.len.avg": float(vlen.mean()) if n else 0.0,
        }
        with open(os.path.join(self.base, "config.properties"), "w") as f:
            for k, v in props.items():
                f.write(f"{k} = {v}\n")

    # W:91-97
    def build(self):
        blob, off, vals = self._records()
        self._addr = self._write_kv(blob, off, vals)
        self._write_config(off, vals)
        self._blob, self._off, self._vals = blob, off, vals
        if self.fused_index:
            paths = (os.path.join(self.base, "index.db"), os.path.join(self.base, "index_a.db"))
            if self.from_files:  # F3: the native scan of the data files just written
                mph = self.ctx.kv_build_index(os.path.join(self.base, "kv.db"), self.partitions, self.checksum_bits,
                                              *paths, self.approximate)
                mph.dump(os.path.join(self.base, "hash.dump"))
                return mph
            value8, vlen = self._value_heads()
            if self.devices is not None:
                from .native import Multi
                with Multi(len(self.devices), self.devices) as mc:
                    E, values, sigbits = mc.mph_build_index_var(blob, off, self.checksum_bits, self._addr, *paths,
                                                                self.approximate, value8, vlen)
                # the assembled fields, resident on this writer's device for dump / lookups
                mph = self.ctx.mph_import(off.size - 1, self.checksum_bits, E, values, sigbits)
            else:
                mph = self.ctx.mph_build_index_var(blob, off, self.checksum_bits, self._addr, *paths,
                                                   self.approximate, value8, vlen)
            mph.dump(os.path.join(self.base, "hash.dump"))
            return mph
        mph = self.build_hash()
        self.build_index(mph)
        return mph

    # W:99-105
    def build_hash(self) -> Mph:
        mph = self.ctx.mph_build_var(self._blob, self._off, self.checksum_bits)
        mph.dump(os.path.join(self.base, "hash.dump"))
        return mph

    # W:107-155
    def build_index(self, mph: Mph, batch: int = 1 << 22):
        n = self._off.size - 1
        value8, vlen = self._value_heads()
        off = self._off

        def feed(w):  # one kv.db scan per pass (W:134)
            for lo in range(0, n, batch):
                hi = min(n, lo + batch)
                w.put_var(self._blob, off[lo: hi + 1], self._addr[lo:hi], value8[lo:hi] if self.approximate else None,
                          vlen[lo:hi] if self.approximate else None)
        return mph.write_index(os.path.join(self.base, "index.db"), os.path.join(self.base, "index_a.db"),
                               self.approximate, self.pass_cache_size, feed)

    def _value_heads(self):
        """index_a.db payload: the first <= 8 value bytes per record (W:140-142)."""
        n = self._off.size - 1
        value8 = np.zeros(n, np.uint64)
        vlen = np.zeros(n, np.uint8)
        if self.approximate and n:
            voff = self._voff.astype(np.int64)
            vlen = np.minimum(np.diff(voff), 8).astype(np.uint8)
            padded = np.concatenate([self._vblob, np.zeros(8, np.uint8)])
            heads = padded[voff[:-1, None] + np.arange(8)[None, :]]       # 8 bytes from each value's start
            heads[np.arange(8)[None, :] >= vlen[:, None]] = 0             # bytes past the value: 0
            value8 = heads.copy().view(np.uint64).reshape(n)
        return value8, vlen

    def close(self):
        self.ctx.close()
