set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -c "
import time, bench
t=time.time(); r = bench.cpu_baseline(8795859, 12.0, 16); print(r, time.time()-t, flush=True)
" > gpurun_out/cpu_probe.log 2>&1; echo "cpu rc=$?" >> gpurun_out/cpu_probe.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_fullnocpu.log 2>&1 || exit 1
