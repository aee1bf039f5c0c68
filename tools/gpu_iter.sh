#!/bin/bash
# Iteration call: gpu tests, kernel microbench (variants), full bench line.
# usage (via gpurun): bash tools/gpu_iter.sh TAG [variants]
set -o pipefail
TAG=${1:-iter}; VARS=${2:-0}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/$TAG/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest_gpu.log
for v in ${VARS//,/ }; do
  BSDB_D13_VARIANT=$v timeout -k 10 120 python tools/kbench.py --n 2147483648 --m 8795859 --reps 3 > gpurun_out/$TAG/kb_v$v.log 2>&1 || { echo "kbench $v failed"; tail gpurun_out/$TAG/kb_v$v.log; exit 2; }
  echo "v$v: $(tail -1 gpurun_out/$TAG/kb_v$v.log)"
done
timeout -k 10 420 python -u bench.py --no-cpu > gpurun_out/$TAG/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/$TAG/bench.log; exit 3; }
tail -1 gpurun_out/$TAG/bench.log
