set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 400 python bench.py > gpurun_out/bench_full.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/bench_kt -o bench --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_prof.log 2>&1 || exit 2
