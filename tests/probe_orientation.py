"""TEST INFRASTRUCTURE (a probe script, not collected by pytest).  Probe (round 5): how many unorientable seed attempts a count of the peeled
core's edges against its vertices catches.  Oracle edges (signatureToEquation,
mph.c:63-71), a plain peel, Kuhn matching of core edges to vertices."""
import sys, numpy as np
import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'oracle'))
import oracle as O
sys.setrecursionlimit(100000)
n = 2_000_000
keys = O.gen_keys13_mt(0, n, 8)
sig = O.hash_fixed_mt(keys, 13, 8)
m = O.num_buckets(n)
b = O.buckets(sig, m)
order = np.lexsort((sig[:, 1], sig[:, 0], b))
sig, b = sig[order], b[order]
cnts = np.bincount(b, minlength=m)
E = np.concatenate([[0], np.cumsum(cnts)]).astype(np.uint64)
vo = lambda x: (int(x) * 281) >> 8
tot = caught = unor = 0
for bk in range(0, 300):
    lo, hi = int(E[bk]), int(E[bk + 1]); nv = vo(hi) - vo(lo)
    for seed in range(0, 6):
        edges = [O.signature_to_equation(int(sig[i, 0]), int(sig[i, 1]), seed << 56, nv) for i in range(lo, hi)]
        if any(e[0] == e[1] == e[2] for e in edges): continue
        deg = [0] * nv; inc = [[] for _ in range(nv)]
        for k, e in enumerate(edges):
            for v in e: deg[v] += 1; inc[v].append(k)
        alive = [True] * len(edges)
        stack = [v for v in range(nv) if deg[v] == 1]
        while stack:
            v = stack.pop()
            if deg[v] != 1: continue
            k = next(k for k in inc[v] if alive[k])
            alive[k] = False
            for u in edges[k]:
                deg[u] -= 1
                if deg[u] == 1: stack.append(u)
        core = [k for k in range(len(edges)) if alive[k]]
        ce = len(core); cv = sum(1 for v in range(nv) if deg[v] > 0)
        # matching core edges -> vertices (Kuhn)
        owner = {}
        def aug(k, seen):
            for v in set(edges[k]):
                if v in seen: continue
                seen.add(v)
                if v not in owner or aug(owner[v], seen):
                    owner[v] = k; return True
            return False
        ok = ce <= cv and all(aug(k, set()) for k in core)
        tot += 1
        if not ok: unor += 1
        if ce > cv: caught += 1
print("attempts", tot, "unorientable", unor, "caught by count", caught)
