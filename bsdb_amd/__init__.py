"""bsdb_amd -- MI355X-native index-build hot path for yc-huang/bsdb.

The package holds only what the path needs:
  csrc/           hand-written gfx950 HIP kernels + the C ABI (include/bsdb_mi355x.h)
  native.py       ctypes binding of that C ABI (the product path; no CPU fallback)
  distributed.py  key shards, the histogram collective, the multi-GPU full build
  writer.py       host-side mirror of the reference's BSDBWriter build stages
"""
from .native import BsdbError, Context, IndexWriter, Mph, Multi, lib, num_buckets  # noqa: F401

__all__ = ["BsdbError", "Context", "IndexWriter", "Mph", "Multi", "lib", "num_buckets"]
