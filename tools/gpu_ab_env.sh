#!/bin/bash
# A/B of an environment switch on one box: parity tests with the switch on,
# then bench lines alternated off/on.
#   tools/gpu_ab_env.sh TAG VAR=VALUE [rounds] [pytest -k expression]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-abe}; KV=$2; R=${3:-3}; K=${4:-"k13 or binned_layouts or ragged or multi_chunk or var or windowed or many_partitions"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
env $KV timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > $OUT/parity_on.log 2>&1 || { tail -n 20 $OUT/parity_on.log; exit 1; }
echo "on parity: $(tail -n 1 $OUT/parity_on.log)"
for r in $(seq 1 $R); do
  for mode in off on; do
    if [ $mode = on ]; then E="$KV"; else E="BSDB_AB_NONE=1"; fi
    env $E timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-full-build > $OUT/b_${mode}_$r.json 2> $OUT/b_${mode}_$r.err || { tail -n 20 $OUT/b_${mode}_$r.err; exit 2; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],3), 'ms/step', 'pass1', round(d['kernel_ms_per_step']['pass1'],3), 'pass2', round(d['kernel_ms_per_step']['pass2'],3))" $OUT/b_${mode}_$r.json $mode
  done
done
