cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; echo "rc=$?" >> gpurun_out/pytest_gpu.log
grep -q "rc=0" gpurun_out/pytest_gpu.log || exit 1
for v in 0 1 3; do BSDB_D13_VARIANT=$v timeout -k 10 100 python tools/kbench.py --n 2147483648 --m 8795859 --reps 3 --frontends 0 --chunks 0 > gpurun_out/kbv_$v.log 2>&1 || exit 2; done
