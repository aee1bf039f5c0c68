#!/bin/bash
# Round 5, GPU call I: kv.db -> index, the partitions' release held until
# the finish's files are open (default) vs for the whole finish, alternated.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5i; mkdir -p $OUT
for mode in open finish open finish; do
  BSDB_KV_REAP_HOLD=$mode BSDB_BUILDER_PROFILE=1 timeout -k 10 300 python -u tools/e2e_legs.py --kv --reps 2 >> $OUT/kv_$mode.json 2>> $OUT/kv_$mode.err || { tail -n 20 $OUT/kv_$mode.err; exit 5; }
done
for mode in open finish; do
  echo "$mode: $(python3 -c 'import json,sys; print([round(json.loads(l)["keys_per_s"]/1e6,1) for l in open(sys.argv[1])])' $OUT/kv_$mode.json)"
  grep "records:\|pass 0" $OUT/kv_$mode.err | cut -c1-200
done
