"""Diagnostic: per-wave phase cycles of k_pass1_d13e (BSDB_D13_VARIANT=4
writes s_memtime sums over the counts array; pass 2 then adds its counts on
top, ~244 per word at 2^31 keys, negligible against the cycle sums)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["BSDB_D13_VARIANT"] = "4"
from bsdb_amd import Context  # noqa: E402
n, m = 2147483648, 8795859
ctx = Context(0)
keys = ctx.gen_keys13(0, n)
for rep in range(2):
    counts = torch.zeros(m, dtype=torch.int32, device="cuda")
    ctx.histogram_fixed(keys, 13, m, counts=counts, n=n)
    torch.cuda.synchronize()
c = counts[: 8 * 4096].view(-1, 8).cpu().double()
c = c[c[:, 4] > 1000]
h, wo, b, o, tot = (c[:, i] * 16 for i in range(5))
print(f"waves {len(c)}  tiles/wave ~{(c[:, 5] - 244).mean():.0f}  cycles/wave {tot.mean():.3e}")
for name, x in (("hash", h), ("write-out", wo), ("barrier", b), ("owner", o)):
    print(f"{name:10s} {100 * (x / tot).mean():5.1f}%  (p10 {100 * (x / tot).quantile(0.1):.1f}, p90 {100 * (x / tot).quantile(0.9):.1f})")
