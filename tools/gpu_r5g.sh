#!/bin/bash
# Round 5, GPU call G: kv.db -> index with the partitions unmapped in
# 32 MiB steps (the finish's index mmap no longer waits behind a 1 GB munmap).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r5g}; mkdir -p $OUT
for i in 1 2 3; do
  BSDB_BUILDER_PROFILE=1 timeout -k 10 300 python -u tools/e2e_legs.py --kv --reps 2 > $OUT/kv_$i.json 2> $OUT/kv_$i.err || { tail -n 20 $OUT/kv_$i.err; exit 5; }
  echo "run $i: $(python3 -c 'import json,sys; print([round(json.loads(l)["keys_per_s"]/1e6,1) for l in open(sys.argv[1])])' $OUT/kv_$i.json)"; grep "created\|opened\|prefaulted\|released in\|release:\|records:" $OUT/kv_$i.err | cut -c1-200
done
