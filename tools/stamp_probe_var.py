"""Diagnostic: per-wave phase cycles of k_pass1_vare (BSDB_D13_VARIANT=4
writes s_memtime sums over the counts array; pass 2 then adds its counts on
top, ~190 per word, negligible against the cycle sums)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["BSDB_D13_VARIANT"] = "4"
from bsdb_amd import Context  # noqa: E402
n = 500_000_000
m = 4_000_000_000 // 1500 + 1
ctx = Context(0)
blob, off = ctx.gen_keys_var(0, n)
for rep in range(2):
    counts = torch.zeros(m, dtype=torch.int32, device="cuda")
    ctx.histogram_var(blob, off, m, counts=counts)
    torch.cuda.synchronize()
c = counts[: 8 * 4096].view(-1, 8).cpu().double()
c = c[c[:, 6] > 1000]
tot = c[:, 6] * 16
print(f"waves {len(c)}  cycles/wave {tot.mean():.3e}")
for i, name in enumerate(("stage", "issue", "hash", "barriers", "owner+write-out", "misc")):
    x = c[:, i] * 16
    print(f"{name:10s} {100 * (x / tot).mean():5.1f}%  (p10 {100 * (x / tot).quantile(0.1):.1f}, p90 {100 * (x / tot).quantile(0.9):.1f})")
