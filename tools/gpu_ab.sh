#!/bin/bash
# A/B of pass-1 kernel variants (BSDB_D13_VARIANT) on one box: bench lines
# alternated, histogram-stage ms/step and pass-1 ms compared.
#   tools/gpu_ab.sh TAG "0 7" [rounds]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-ab}; VARS=${2:-"0 7"}; R=${3:-2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -n "$PARITY" ]; then
  for v in $VARS; do
    BSDB_D13_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "$PARITY" > $OUT/parity_v$v.log 2>&1 || { tail -n 20 $OUT/parity_v$v.log; exit 1; }
    echo "v$v parity: $(tail -n 1 $OUT/parity_v$v.log)"
  done
fi
for r in $(seq 1 $R); do
  for v in $VARS; do
    BSDB_D13_VARIANT=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-full-build > $OUT/b_${v}_$r.json 2> $OUT/b_${v}_$r.err || { tail -n 20 $OUT/b_${v}_$r.err; exit 2; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('v'+sys.argv[2], round(d['ms_per_step'],3), 'ms/step', 'pass1', round(d['kernel_ms_per_step']['pass1'],3), 'pass2', round(d['kernel_ms_per_step']['pass2'],3), round(d['value']/1e9,1), 'G')" $OUT/b_${v}_$r.json $v
  done
done
