"""One end-to-end C2 build (bench.e2e_host_to_disk: host keys -> index.db +
hash.dump) for a kernel / memory-copy trace (measurement tool):
    rocprofv3 --kernel-trace --memory-copy-trace --stats -d DIR -- python3 tools/e2e_trace.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bsdb_amd import Context  # noqa: E402

ctx = Context(0)
bench.e2e_host_to_disk(ctx, 100_000_000, 4)  # warm
print(json.dumps(bench.e2e_host_to_disk(ctx, 100_000_000, 4)))
