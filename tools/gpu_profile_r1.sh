set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
grep -q "pytest rc=0" gpurun_out/pytest_gpu.log || grep -q "passed" gpurun_out/pytest_gpu.log || exit 1
timeout -k 10 300 python tools/kbench.py --n 1000000000 --chunks 0,268435456,67108864 > gpurun_out/kbench.log 2>&1 || exit 2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt -o kt --output-format csv -- python3 bench.py --n 2000000000 --steps 5 --warmup 2 --no-cpu > gpurun_out/prof_bench.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -d gpurun_out/prof/pmc1 -o pmc1 --output-format csv -- python3 tools/kbench.py --n 200000000 --reps 1 > gpurun_out/prof_pmc1.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE SQ_ACTIVE_INST_VALU SQ_WAIT_ANY -d gpurun_out/prof/pmc2 -o pmc2 --output-format csv -- python3 tools/kbench.py --n 200000000 --reps 1 > gpurun_out/prof_pmc2.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d gpurun_out/prof/pmc3 -o pmc3 --output-format csv -- python3 tools/kbench.py --n 200000000 --reps 1 > gpurun_out/prof_pmc3.log 2>&1 || exit 6
