"""Diagnoses throughput vs buffer size / offset on a large HBM allocation."""
import sys, os, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bsdb_amd import Context
def T(label, fn):
    torch.cuda.synchronize(); t = time.time(); r = fn(); torch.cuda.synchronize()
    print(f"{label}: {1e3*(time.time()-t):.1f} ms", flush=True); return r
free, total = torch.cuda.mem_get_info(); print("mem free/total GB", free/1e9, total/1e9, flush=True)
n = int(sys.argv[1])
ctx = Context(0)
keys = T("alloc", lambda: torch.empty(13 * n + 16, dtype=torch.uint8, device="cuda"))
print("mem free after alloc GB", torch.cuda.mem_get_info()[0]/1e9, flush=True)
T("gen", lambda: ctx.gen_keys13(0, n, out=keys))
T("gen again", lambda: ctx.gen_keys13(0, n, out=keys))
for m in (1_333_334, 8_795_859):
    counts = torch.zeros(m, dtype=torch.int32, device="cuda")
    for off in (0, n - 200_000_000):
        for mode in (2, 0):
            ctx.set_histogram_mode(mode)
            counts.zero_()
            T(f"m={m} off={off/1e9:.1f}B mode={mode} 200M keys", lambda: ctx.histogram_fixed(keys[13*off:], 13, m, counts=counts, n=200_000_000))
            print("   total", int(counts.sum(dtype=torch.int64)), flush=True)
ctx.set_histogram_mode(0)
m = 8_795_859
counts = torch.zeros(m, dtype=torch.int32, device="cuda")
for nk in (500_000_000, 1_000_000_000, 2_147_483_648):
    counts.zero_()
    T(f"m={m} off=0 part {nk} keys", lambda: ctx.histogram_fixed(keys, 13, m, counts=counts, n=nk))
    print("   total", int(counts.sum(dtype=torch.int64)), flush=True)
