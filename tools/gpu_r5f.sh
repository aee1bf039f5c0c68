#!/bin/bash
# Round 5, GPU call F: kv.db -> index, the concurrent adds' copies through
# pinned pieces (default) vs the source registered in place, alternated.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r5f}; mkdir -p $OUT
for mode in bounce register bounce register; do
  BSDB_ADD_COPY=$mode BSDB_BUILDER_PROFILE=1 timeout -k 10 300 python -u tools/e2e_legs.py --kv --reps 2 > $OUT/kv_$mode.json 2> $OUT/kv_$mode.err || { tail -n 20 $OUT/kv_$mode.err; exit 5; }
  echo "$mode: $(python3 -c 'import json,sys; print([round(json.loads(l)["keys_per_s"]/1e6,1) for l in open(sys.argv[1])])' $OUT/kv_$mode.json)"; grep "adds:\|records:" $OUT/kv_$mode.err | cut -c1-200
done
