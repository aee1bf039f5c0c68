#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/occ
summ='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=[d[k]["gov_build_ms"] for k in d if k.startswith("rep")][1:]; print("gov ms median %.3f" % sorted(r)[len(r)//2])'
for v in two one two one; do
  if [ $v = one ]; then export BSDB_GOV_ONE_PER_CU=1; else unset BSDB_GOV_ONE_PER_CU; fi
  BSDB_GOV_PROFILE=1 timeout -k 10 200 python tools/full_build.py --n 100000000 --reps 2 > gpurun_out/occ/$v.log 2>&1 || { tail -5 gpurun_out/occ/$v.log; exit 1; }
  echo "$v: $(python3 -c "$summ" < gpurun_out/occ/$v.log) $(grep 'workgroups per CU' gpurun_out/occ/$v.log | tail -1)"
done
