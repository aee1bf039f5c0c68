"""How many failed attempts had a full-row-rank core matrix (i.e. SOME hinge
set would have been nonsingular)?  Oracle edges, python peel, F3 rank."""
import sys
import numpy as np
sys.path.insert(0, "/root/repo/oracle")
import oracle as O

n = 300_000
keys = O.gen_keys13(7, n)
sig = O.hash_fixed(keys, 13)
rc, E, vals, sb = O.gov_build(sig, 0)
m = n // 1500 + 1
b = O.buckets(sig, m)
order = np.lexsort((sig[:, 1], sig[:, 0], b))
sig = sig[order]
b = b[order]
starts = np.searchsorted(b, np.arange(m + 1))
OFF = np.uint64((1 << 56) - 1)


def vo(x):
    return ((int(x) & ((1 << 56) - 1)) * 281) >> 8


def f3_rank(A):
    A = A.copy() % 3
    r = 0
    rows, cols = A.shape
    for c in range(cols):
        piv = np.nonzero(A[r:, c])[0]
        if piv.size == 0:
            continue
        p = r + piv[0]
        A[[r, p]] = A[[p, r]]
        if A[r, c] == 2:
            A[r] = (A[r] * 2) % 3
        nz = np.nonzero(A[:, c])[0]
        nz = nz[nz != r]
        if nz.size:
            A[nz] = (A[nz] - A[nz, c][:, None] * A[r][None, :]) % 3
        r += 1
        if r == rows:
            break
    return r


stats = {"fail": 0, "fail_fullrank": 0, "ok": 0, "ok_fullrank": 0}
for bk in range(0, m, max(1, m // 60)):
    lo, hi = int(starts[bk]), int(starts[bk + 1])
    cnt = hi - lo
    nv = vo(E[bk + 1]) - vo(E[bk])
    seed_ok = int(E[bk]) >> 56
    for s in range(seed_ok + 1):
        e = np.array([O.signature_to_equation(int(sig[k, 0]), int(sig[k, 1]), s << 56, nv) for k in range(lo, hi)])
        # peel
        alive = np.ones(cnt, bool)
        deg = np.zeros(nv, int)
        for k in range(cnt):
            for v in e[k]:
                deg[v] += 1
        changed = True
        while changed:
            changed = False
            for k in np.nonzero(alive)[0]:
                if any(deg[v] == 1 for v in e[k]):
                    alive[k] = False
                    for v in e[k]:
                        deg[v] -= 1
                    changed = True
        core = np.nonzero(alive)[0]
        verts = sorted(set(e[core].reshape(-1).tolist()))
        col = {v: i for i, v in enumerate(verts)}
        A = np.zeros((core.size, len(verts)), np.int64)
        for i, k in enumerate(core):
            for v in e[k]:
                A[i, col[v]] += 1
        full = core.size == 0 or f3_rank(A) == core.size
        key = "ok" if s == seed_ok else "fail"
        stats[key] += 1
        stats[key + "_fullrank"] += int(full)
    print(bk, stats, flush=True)
print(stats)
