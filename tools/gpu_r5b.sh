#!/bin/bash
# Round 5, GPU call B: kv.db scan + builder tests after the lean parse /
# concurrent adds, the 1e9 C3-size builder test, and the kv.db -> index leg
# with its phases (BSDB_BUILDER_PROFILE=1), twice.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r5b}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_builder_gpu.py tests/test_kv_scan.py -k "kv or c3_size or concurrent" -x -v --timeout 500 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -n 40 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
for i in 1 2; do
  BSDB_BUILDER_PROFILE=1 timeout -k 10 300 python -u tools/e2e_legs.py --kv > $OUT/kv$i.json 2> $OUT/kv$i.err || { tail -n 20 $OUT/kv$i.err; exit 2; }
  tail -n 1 $OUT/kv$i.json | cut -c1-200; grep "bsdb" $OUT/kv$i.err
done
