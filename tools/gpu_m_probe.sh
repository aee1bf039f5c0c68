set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python tools/kbench.py --n 500000000 --m 8795859 --reps 2 --frontends 0,2 --chunks 0 > gpurun_out/kbench_m.log 2>&1 || exit 1
timeout -k 10 120 python tools/kbench.py --n 500000000 --m 2666667 --reps 2 --frontends 0,2 --chunks 0 > gpurun_out/kbench_m2.log 2>&1 || exit 2
