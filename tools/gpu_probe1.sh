#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe1
timeout -k 10 120 ./tools/mall_probe > gpurun_out/probe1/mall.log 2>&1 || exit 1
timeout -k 10 120 ./tools/stream_probe > gpurun_out/probe1/stream.log 2>&1 || exit 2
for v in 0 1 3; do BSDB_D13_VARIANT=$v timeout -k 10 120 python tools/kbench.py --n 2147483648 --m 8795859 --reps 3 > gpurun_out/probe1/kb_v$v.log 2>&1 || exit 3; done
cat gpurun_out/probe1/*.log
