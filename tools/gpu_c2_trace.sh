#!/bin/bash
# C2 (1e8 keys) per-kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/c2tr
mkdir -p $out
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/rp -o c2 --output-format csv -- python tools/full_build.py --n 100000000 --reps 2 > $out/rp.log 2>&1 || { tail -5 $out/rp.log; exit 3; }
tail -1 $out/rp.log | cut -c1-300
cut -d, -f1-4 $out/rp/c2_kernel_stats.csv | cut -c1-150 | head -14
