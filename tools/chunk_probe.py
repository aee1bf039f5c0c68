"""Times the histogram chunk by chunk over a large HBM-resident key set."""
import sys, os, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bsdb_amd import Context
n = int(sys.argv[1]); fe = int(sys.argv[2]) if len(sys.argv) > 2 else 0
m = n // 1500 + 1
ctx = Context(0); ctx.set_frontend(fe)
keys = torch.empty(13 * n + 16, dtype=torch.uint8, device="cuda")
ctx.gen_keys13(0, n, out=keys); torch.cuda.synchronize()
print("gen done", flush=True)
counts = torch.zeros(m, dtype=torch.int32, device="cuda")
CH = 1 << 31
for k0 in range(0, n, CH):
    nk = min(CH, n - k0)
    t = time.time()
    ctx.histogram_fixed(keys[13 * k0:], 13, m, counts=counts, n=nk)
    torch.cuda.synchronize()
    print(f"chunk at {k0/1e9:.2f}B keys ({13*k0/1e9:.0f} GB): {1e3*(time.time()-t):.1f} ms", flush=True)
print("total", int(counts.sum(dtype=torch.int64)), "expected", n, flush=True)
