set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for n in 2000000000 4000000000; do
  timeout -k 10 120 python bench.py --num-keys $n --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_n$n.log 2>&1 || exit 1
done
