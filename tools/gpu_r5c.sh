#!/bin/bash
# Round 5, GPU call C: builder/kv tests after the pinned-bounce adds and the
# device record arrays, the kv.db -> index leg with phases, then the solver
# variants (256-thread workgroups, the register Gauss-Jordan): GOV parity,
# phase profile at 1e7 keys, C2 build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r5c}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_builder_gpu.py -k "not c3_size and not 2e8" -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -n 40 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
for i in 1 2; do
  BSDB_BUILDER_PROFILE=1 timeout -k 10 300 python -u tools/e2e_legs.py --kv > $OUT/kv$i.json 2> $OUT/kv$i.err || { tail -n 20 $OUT/kv$i.err; exit 2; }
  tail -n 1 $OUT/kv$i.json | cut -c1-120; grep "bsdb" $OUT/kv$i.err
done
bash tools/gpu_gov_variants.sh "$@"
