"""The one-process E4 build with eight device contexts on this box's one GPU
(the layout bench.py uses on an 8-GPU node, every context on device 0 here):
C3-size host keys, the fields must equal the one-context build's."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bsdb_amd import Context  # noqa: E402
from bsdb_amd.native import Multi  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
ctx = Context(0)
keys = ctx.gen_keys13(0, n)[: 13 * n].cpu().numpy()
ctx.close()
torch.cuda.empty_cache()
res = {}
for G in (1, 8):
    with Multi(G, [0] * G) as mc:
        t = time.perf_counter()
        res[G] = mc.mph_build_index_fixed(keys, 13, 4)
        print(f"G={G}: {time.perf_counter() - t:.2f} s", flush=True)
same = all(np.array_equal(a, b) for a, b in zip(res[1], res[8]))
print("fields equal:", same)
assert same
