"""Diagnostic: per-wave barrier-wait fractions of the 13-byte pass-1 kernel
(BSDB_D13_VARIANT=11 build writes s_memtime sums over the counts array)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bsdb_amd import Context  # noqa: E402
os.environ.setdefault("BSDB_D13_VARIANT", "11")
n = 2147483648
m = 8795859
ctx = Context(0)
keys = ctx.gen_keys13(0, n)
for rep in range(2):
    counts = torch.zeros(m, dtype=torch.int32, device="cuda")
    ctx.histogram_fixed(keys, 13, m, counts=counts, n=n)
    torch.cuda.synchronize()
c = counts[: 4 * 4096].view(-1, 4).cpu().double() * 16
c = c[c[:, 2] > 0]
a, cc, tot, nt = c[:, 0], c[:, 1], c[:, 2], c[:, 3] / 16
print(f"waves {len(c)}  tiles/wave {nt.mean():.1f}  loop cycles/wave {tot.mean():.3e}")
print(f"barrier A wait {100 * (a / tot).mean():.1f}% (p10 {100 * (a / tot).quantile(0.1):.1f}, p90 {100 * (a / tot).quantile(0.9):.1f})")
print(f"barrier C wait {100 * (cc / tot).mean():.1f}%")
print(f"cycles per tile {(tot / nt).mean():.0f}, A per tile {(a / nt).mean():.0f}, C per tile {(cc / nt).mean():.0f}")
