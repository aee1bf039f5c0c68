#!/bin/bash
# Kernel trace + PMC passes over the var-len pass-1 kernel (varlen_bench, binned front end).
set -o pipefail
TAG=${1:-pmcvar}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/$TAG; export TMPDIR=/tmp
CMD="python3 tools/varlen_bench.py --fe 0 --reps 2"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/kt -o kt --output-format csv -- $CMD > gpurun_out/$TAG/kt.log 2>&1 || { echo "kernel trace failed"; tail -5 gpurun_out/$TAG/kt.log; exit 1; }
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d gpurun_out/$TAG/p$i -o p$i --output-format csv -- $CMD > gpurun_out/$TAG/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/$TAG/p$i.log; exit 1; }
done
echo done
