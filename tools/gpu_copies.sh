#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/copies
for k in ${1//,/ }; do
  BSDB_D13_COPIES=$k BSDB_D13_VARIANT=22 timeout -k 10 120 python tools/kbench.py --n 2147483648 --m 8795859 --reps 3 > gpurun_out/copies/k$k.log 2>&1 || { echo "copies $k failed"; tail -3 gpurun_out/copies/k$k.log; exit 2; }
  echo "copies $k: $(tail -1 gpurun_out/copies/k$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read())["part_fe0_chunk0"]; print("pass1 %.3f ms pass2 %.3f ms" % (d["pass1_ms"], d["pass2_ms"]))')"
done
