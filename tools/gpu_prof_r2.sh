#!/bin/bash
# rocprofv3 kernel-trace summary of the bench (histogram stage + full-build figures).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/run -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err || { tail -20 gpurun_out/prof/bench.err; exit 1; }
find gpurun_out/prof/run -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof/kernel_stats.csv \;
head -30 gpurun_out/prof/kernel_stats.csv | cut -c1-200
