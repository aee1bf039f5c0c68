#!/bin/bash
# Where the GOV solver's waves wait (k_gov_solve, C2's shape at 1e7 keys via tools/full_build.py):
# one counter group per rocprofv3 run (gfx950: <= 8 SQ counters a pass), summed by tools/pmc_sum.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-pmc_solver}; mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || { echo "counter list failed"; exit 1; }
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INSTS_SALU SQ_INST_LEVEL_LDS"; do
  i=$((i+1))
  keep=""
  for c in $grp; do grep -qw "$c" $OUT/counters_list.txt && keep="$keep $c"; done
  [ -z "$keep" ] && continue
  echo "pass $i:$keep"
  timeout -s KILL 120 rocprofv3 --pmc $keep -d $OUT/p$i -o p$i --output-format csv -- python3 tools/full_build.py --n 10000000 --reps 1 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_sum.py $OUT k_gov_solve > $OUT/summary.txt 2>&1
cat $OUT/summary.txt
