cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
BSDB_D13_THREADS=256 timeout -k 10 300 python -m pytest tests -m gpu -q -x -k "k13 or histogram or smoke or full" > gpurun_out/pytest_gpu.log 2>&1; echo "rc=$?" >> gpurun_out/pytest_gpu.log
for t in 512 256; do BSDB_D13_THREADS=$t timeout -k 10 100 python tools/kbench.py --n 2147483648 --m 8795859 --reps 3 --frontends 0 --chunks 0 > gpurun_out/kbt_$t.log 2>&1 || exit 2; done
