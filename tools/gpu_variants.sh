#!/bin/bash
# kbench of pass-1 variants at 2^31 keys (no tests)
set -o pipefail
TAG=${1:-var}; VARS=${2:-0}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/$TAG
for v in ${VARS//,/ }; do
  BSDB_D13_VARIANT=$v timeout -k 10 120 python tools/kbench.py --n 2147483648 --m 8795859 --reps 3 > gpurun_out/$TAG/kb_v$v.log 2>&1 || { echo "kbench $v failed"; tail gpurun_out/$TAG/kb_v$v.log; exit 2; }
  echo "v$v: $(tail -1 gpurun_out/$TAG/kb_v$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read())["part_fe0_chunk0"]; print("pass1 %.3f ms pass2 %.3f ms" % (d["pass1_ms"], d["pass2_ms"]))')"
done
