#!/bin/bash
# Round 5, GPU call H: kv.db -> index, files read through a window (default)
# vs mapped whole (BSDB_KV_MMAP=1), alternated; then the kv.db parity tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5h; mkdir -p $OUT
for mode in window mmap window mmap; do
  if [ $mode = mmap ]; then export BSDB_KV_MMAP=1; else unset BSDB_KV_MMAP; fi
  BSDB_BUILDER_PROFILE=1 timeout -k 10 300 python -u tools/e2e_legs.py --kv --reps 2 >> $OUT/kv_$mode.json 2>> $OUT/kv_$mode.err || { tail -n 20 $OUT/kv_$mode.err; exit 5; }
done
unset BSDB_KV_MMAP
for mode in window mmap; do
  echo "$mode: $(python3 -c 'import json,sys; print([round(json.loads(l)["keys_per_s"]/1e6,1) for l in open(sys.argv[1])])' $OUT/kv_$mode.json)"
  grep "records:" $OUT/kv_$mode.err | cut -c1-200
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_builder_gpu.py tests/test_writer_gpu.py -k "kv or writer" > $OUT/pytest.log 2>&1; rc=$?; tail -n 3 $OUT/pytest.log; exit $rc
