#!/bin/bash
# A/B recorded in DESIGN §3.1 (profiles/r3/d2h/ab_bounce_vs_runtime.jsonl): the
# C4 exact build with the pass slices copied by the in-tree library against a
# variant build bsdb_amd/libbsdb_rtd2h.so (the same sources with d2h_pageable
# replaced by one runtime hipMemcpyAsync; built from a scratch copy of
# bsdb_amd/csrc, not kept).  At the time of the A/B the in-tree library used
# the parallel pinned-bounce copy, now replaced by the runtime copy.
set -o pipefail
mkdir -p gpurun_out/abd2h
for i in 1 2; do
 for lib in libbsdb_mi355x libbsdb_rtd2h; do
  BSDB_LIB=$PWD/bsdb_amd/$lib.so timeout -k 10 200 python -c "
import bench, json, torch
from bsdb_amd import Context
ctx = Context(0)
n = 13_193_787_549
keys = torch.empty(13 * n + 16, dtype=torch.uint8, device='cuda')
ctx.gen_keys13(0, n, out=keys)
torch.cuda.synchronize()
r = bench.c4_exact_passes(ctx, keys, n, 4)
print(json.dumps({'lib': '$lib', 's': r['ms'] / 1e3, 'Mkeys': r['keys_per_s'] / 1e6, 'passes': r['passes']}))
" >> gpurun_out/abd2h/ab.jsonl 2>> gpurun_out/abd2h/ab.err || exit 1
 done
done
timeout -k 10 200 python tools/e2e_host.py --n 2000000000 > gpurun_out/abd2h/e2e_host.json 2>> gpurun_out/abd2h/ab.err
cat gpurun_out/abd2h/ab.jsonl
