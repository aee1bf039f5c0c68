#!/bin/bash
# Round 5, GPU call N: kv.db -> index with the partitions streamed into the
# builder in chunks (BSDB_KV_CHUNK records per add; 0 = one add a partition),
# alternated; then the kv.db parity tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5n; mkdir -p $OUT
for ch in 1048576 2097152 4194304 1048576 2097152 4194304; do
  BSDB_KV_CHUNK=$ch BSDB_BUILDER_PROFILE=1 timeout -k 10 300 python -u tools/e2e_legs.py --kv --reps 2 >> $OUT/kv_$ch.json 2>> $OUT/kv_$ch.err || { tail -n 20 $OUT/kv_$ch.err; exit 5; }
done
for ch in 1048576 2097152 4194304; do
  echo "chunk $ch: $(python3 -c 'import json,sys; print([round(json.loads(l)["keys_per_s"]/1e6,1) for l in open(sys.argv[1])])' $OUT/kv_$ch.json)"
  grep "records:" $OUT/kv_$ch.err | cut -c1-200
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_builder_gpu.py tests/test_writer_gpu.py -k "kv or writer" > $OUT/pytest.log 2>&1; rc=$?; tail -n 3 $OUT/pytest.log; exit $rc
