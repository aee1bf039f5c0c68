set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 300 python bench.py > gpurun_out/bench_full.log 2>&1 || exit 2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/bench_kt -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_prof.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pmc_fetch -o fetch --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc_fetch.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/pmc_write -o write --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc_write.log 2>&1 || exit 5
