#!/bin/bash
# Round 5, GPU call O: the kv.db parity tests over chunk sizes, then the
# kv leg as the bench runs it (one cold call per process, three processes).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5o; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_builder_gpu.py -k "kv" > $OUT/pytest.log 2>&1 || { tail -n 30 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
for i in 1 2 3; do
  BSDB_BUILDER_PROFILE=1 timeout -k 10 300 python -u tools/e2e_legs.py --kv --reps 1 >> $OUT/kv.json 2>> $OUT/kv.err || { tail -n 20 $OUT/kv.err; exit 5; }
done
echo "cold kv legs: $(python3 -c 'import json,sys; print([round(json.loads(l)["keys_per_s"]/1e6,1) for l in open(sys.argv[1])])' $OUT/kv.json)"
grep "records:" $OUT/kv.err | cut -c1-200
