set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
grep -q "passed" gpurun_out/pytest_gpu.log || exit 1
timeout -k 10 300 python tools/kbench.py --n 2000000000 --frontends 0,1 --chunks 0,268435456 > gpurun_out/kbench.log 2>&1 || exit 2
