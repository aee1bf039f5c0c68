#!/bin/bash
# Stall breakdown of the headline pass-1 kernel k_pass1_d13e (kbench, 2^31 keys at the C4 bucket count):
# one counter group per rocprofv3 run (gfx950: <= 8 SQ, 4 TCC, 4 TCP, 2 GRBM counters a pass).
# Counters the box does not list are dropped from their group first; a pass that fails ends the call.
set -o pipefail
TAG=${TAG:-pmc_stalls}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || { echo "counter list failed"; exit 1; }
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT SQ_INST_LEVEL_VMEM SQ_IFETCH GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  keep=""
  for c in $grp; do grep -qw "${c%_sum}" $OUT/counters_list.txt && keep="$keep $c"; done
  [ -z "$keep" ] && continue
  echo "pass $i:$keep"
  timeout -s KILL 90 rocprofv3 --pmc $keep -d $OUT/p$i -o p$i --output-format csv -- python3 tools/kbench.py --n 2147483648 --m 8795859 --reps 1 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_sum.py $OUT d13e > $OUT/summary.txt 2>&1
cat $OUT/summary.txt
