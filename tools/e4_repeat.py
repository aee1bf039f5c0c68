import sys, time, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch
from bsdb_amd import Context
from bsdb_amd.native import Multi
n = 1_000_000_000
ctx = Context(0)
keys = ctx.gen_keys13(0, n)[: 13 * n].cpu().numpy()
torch.cuda.empty_cache()
with Multi(1) as mc:
    for r in range(3):
        t = time.perf_counter()
        E, v, s = mc.mph_build_index_fixed(keys, 13, 4)
        print("rep", r, time.perf_counter() - t, flush=True)
