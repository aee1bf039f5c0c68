#!/bin/bash
# A/B of var-len pass-1 variants (BSDB_D13_VARIANT) on one box: parity tests
# of the var-len path per variant, then tools/varlen_bench.py alternated.
#   tools/gpu_ab_var.sh TAG "0 10" [rounds]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-abv}; VARS=${2:-"0 10"}; R=${3:-2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for v in $VARS; do
  BSDB_D13_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "var" > $OUT/parity_v$v.log 2>&1 || { tail -n 20 $OUT/parity_v$v.log; exit 1; }
  echo "v$v parity: $(tail -n 1 $OUT/parity_v$v.log)"
done
for r in $(seq 1 $R); do
  for v in $VARS; do
    BSDB_D13_VARIANT=$v timeout -k 10 200 python -u tools/varlen_bench.py --fe 0 --reps 5 > $OUT/v_${v}_$r.json 2> $OUT/v_${v}_$r.err || { tail -n 20 $OUT/v_${v}_$r.err; exit 2; }
    echo "v$v: $(tail -n 1 $OUT/v_${v}_$r.json)"
  done
done
