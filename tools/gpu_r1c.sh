set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
for v in 0 1 2; do BSDB_D13_VARIANT=$v timeout -k 10 200 python tools/kbench.py --n 2000000000 --frontends 0 --chunks 0 --reps 5 > gpurun_out/kbench_v$v.log 2>&1 || exit 1; done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d gpurun_out/prof/pmcA -o pmcA --output-format csv -- python3 tools/kbench.py --n 500000000 --reps 1 > gpurun_out/prof_pmcA.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD TA_BUSY_avr TA_TA_BUSY_sum SQ_INSTS_SALU -d gpurun_out/prof/pmcB -o pmcB --output-format csv -- python3 tools/kbench.py --n 500000000 --reps 1 > gpurun_out/prof_pmcB.log 2>&1 || exit 3
