#!/bin/bash
# Speculation policy A/B (BSDB_GOV_SPEC = "K[,P]") at C1 and C2, same library.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/spec
mkdir -p $out
summ='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=[d[k]["gov_build_ms"] for k in d if k.startswith("rep")][1:]; print("gov ms median %.3f min %.3f" % (sorted(r)[len(r)//2], min(r)))'
BSDB_GOV_SPEC=2,1 timeout -k 10 300 python -u -m pytest tests/test_build_gpu.py -m gpu -x -q -k "gov or range" --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
echo "tests (2,1): $(tail -1 $out/pytest.log)"
for rep in 1 2; do
  for v in none 2 3 4 0,1 2,1 3,1; do
    if [ $v = none ]; then unset BSDB_GOV_SPEC; else export BSDB_GOV_SPEC=$v; fi
    timeout -k 10 120 python tools/full_build.py --n 1000000 --reps 9 > $out/c1_$v.$rep.log 2>&1 || { tail -5 $out/c1_$v.$rep.log; exit 2; }
    echo "C1 spec=$v rep $rep: $(python3 -c "$summ" < $out/c1_$v.$rep.log)"
  done
done
for v in none 3,1; do
  if [ $v = none ]; then unset BSDB_GOV_SPEC; else export BSDB_GOV_SPEC=$v; fi
  timeout -k 10 200 python tools/full_build.py --n 100000000 --reps 3 > $out/c2_$v.log 2>&1 || { tail -5 $out/c2_$v.log; exit 3; }
  echo "C2 spec=$v: $(python3 -c "$summ" < $out/c2_$v.log)"
done
