#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 tools/alu_probe > gpurun_out/alu_probe.log 2>&1 || { cat gpurun_out/alu_probe.log; exit 1; }
cat gpurun_out/alu_probe.log
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "var or gov_build" > gpurun_out/pytest_var.log 2>&1 || { tail -40 gpurun_out/pytest_var.log; exit 1; }
tail -3 gpurun_out/pytest_var.log
timeout -k 10 300 python tools/varlen_bench.py --n 500000000 > gpurun_out/varlen_500m.log 2>&1 || { cat gpurun_out/varlen_500m.log; exit 1; }
tail -1 gpurun_out/varlen_500m.log
timeout -k 10 200 python tools/full_build.py --n 10000000 --reps 2 > gpurun_out/fb_10m.log 2>&1 || { cat gpurun_out/fb_10m.log; exit 1; }
cat gpurun_out/fb_10m.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fb -o fb -- python3 tools/full_build.py --n 100000000 --reps 2 > gpurun_out/fb_100m.log 2>&1
rc=$?
cat gpurun_out/fb_100m.log | grep -v "^W2" | tail -20
find gpurun_out/prof_fb -name "*kernel_stats.csv" -exec cp {} gpurun_out/fb_kernel_stats.csv \;
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/e2e_host.py --n 2000000000 > gpurun_out/e2e_host.log 2>&1
rc=$?
cat gpurun_out/e2e_host.log | tail -5
exit $rc
