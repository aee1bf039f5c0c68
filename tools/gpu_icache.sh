#!/bin/bash
# Instruction-cache counters for the var-len and 13-byte pass-1 kernels.
set -o pipefail
TAG=${1:-ic}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/$TAG; export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ -d gpurun_out/$TAG/p1 -o p1 --output-format csv -- python3 tools/varlen_bench.py --fe 0 --reps 1 > gpurun_out/$TAG/p1.log 2>&1 || { echo "var pass failed"; tail -3 gpurun_out/$TAG/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ -d gpurun_out/$TAG/p2 -o p2 --output-format csv -- python3 tools/kbench.py --n 2147483648 --m 8795859 --reps 1 > gpurun_out/$TAG/p2.log 2>&1 || { echo "k13 pass failed"; tail -3 gpurun_out/$TAG/p2.log; exit 2; }
echo done
