#!/bin/bash
# Secondary measurements for DESIGN.md section 5 (one GPU call).
set -o pipefail
TAG=${1:-meas}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/$TAG; export TMPDIR=/tmp
timeout -k 10 200 python tools/full_build.py --n 100000000 > gpurun_out/$TAG/full_c2.log 2>&1 || { echo "full_build c2 failed"; tail -5 gpurun_out/$TAG/full_c2.log; exit 1; }
tail -1 gpurun_out/$TAG/full_c2.log
timeout -k 10 300 python tools/full_build.py --n 1000000000 --approx > gpurun_out/$TAG/full_c3.log 2>&1 || { echo "full_build c3 failed"; tail -5 gpurun_out/$TAG/full_c3.log; exit 2; }
tail -1 gpurun_out/$TAG/full_c3.log
timeout -k 10 200 python tools/varlen_bench.py > gpurun_out/$TAG/varlen.log 2>&1 || { echo "varlen failed"; tail -5 gpurun_out/$TAG/varlen.log; exit 3; }
tail -1 gpurun_out/$TAG/varlen.log
timeout -k 10 300 python tools/e2e_host.py --n 2000000000 > gpurun_out/$TAG/e2e.log 2>&1 || { echo "e2e failed"; tail -5 gpurun_out/$TAG/e2e.log; exit 4; }
tail -1 gpurun_out/$TAG/e2e.log
bash tools/gpu_pmc1.sh ${TAG}_pmc 0 || exit 5
