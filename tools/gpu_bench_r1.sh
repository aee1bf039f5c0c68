set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
grep -q "pytest rc=0" gpurun_out/pytest_gpu.log || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_full.log 2>&1 || exit 2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/bench_kt -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_prof.log 2>&1 || exit 3
