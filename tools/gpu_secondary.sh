#!/bin/bash
# Secondary-row profiles at HEAD (one GPU call): var-len kernel trace + PMC,
# var-len and fixed-length benches.  usage (via gpurun): bash tools/gpu_secondary.sh TAG
set -o pipefail
TAG=${1:-sec}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/$TAG; export TMPDIR=/tmp
bash tools/gpu_pmc_var.sh ${TAG}_pmc > gpurun_out/$TAG/pmc.log 2>&1 || { echo "var-len pmc failed"; tail -3 gpurun_out/$TAG/pmc.log; exit 1; }
timeout -k 10 200 python tools/varlen_bench.py > gpurun_out/$TAG/varlen.log 2>&1 || { echo "varlen bench failed"; exit 2; }
tail -1 gpurun_out/$TAG/varlen.log
timeout -k 10 300 python tools/fixed_len_bench.py > gpurun_out/$TAG/fixed.log 2>&1 || { echo "fixed bench failed"; exit 3; }
tail -1 gpurun_out/$TAG/fixed.log
echo done
