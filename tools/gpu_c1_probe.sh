#!/bin/bash
# C1 (1e6 keys) anatomy: phase profile, per-kernel trace of 5 builds.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/c1
mkdir -p $out
BSDB_GOV_PROFILE=1 timeout -k 10 120 python tools/full_build.py --n 1000000 --reps 3 > $out/prof.log 2>&1 || { tail -5 $out/prof.log; exit 1; }
grep "gov-profile\] m=" $out/prof.log | tail -1
timeout -k 10 120 python tools/full_build.py --n 1000000 --reps 5 > $out/c1.log 2>&1 || { tail -5 $out/c1.log; exit 2; }
tail -1 $out/c1.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $out/rp -o c1 -- python tools/full_build.py --n 1000000 --reps 5 > $out/rp.log 2>&1 || { tail -5 $out/rp.log; exit 3; }
find $out/rp -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $out/kernel_stats.csv
head -12 $out/kernel_stats.csv
