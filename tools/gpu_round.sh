#!/bin/bash
# One GPU call: gpu tests, bench line (with cpu_baseline), rocprof kernel stats
# of the bench, PMC traffic passes (FETCH_SIZE, WRITE_SIZE) over one bench step.
# usage (via gpurun): bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-run}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$TAG/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest_gpu.log
timeout -k 10 420 python -u bench.py > gpurun_out/$TAG/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/$TAG/bench.log; exit 2; }
tail -1 gpurun_out/$TAG/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/kt -o kt --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/$TAG/bench_prof.log 2>&1 || { echo "rocprof failed"; exit 3; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/$TAG/pmc_fetch -o fetch --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/$TAG/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 4; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/$TAG/pmc_write -o write --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/$TAG/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 5; }
echo done
