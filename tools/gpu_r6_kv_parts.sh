#!/bin/bash
# Round 6: the kv.db leg's phases at 8 partitions and at the reference writer's
# 2 x cores (BSDB_BUILDER_PROFILE=1), two reps each in one process.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r6/kv}; mkdir -p $OUT
for PT in "8 0" "0 0" "0 8" "0 4"; do
  set -- $PT; P=$1; T=$2
  BSDB_BUILDER_PROFILE=1 timeout -k 10 300 python -u tools/e2e_legs.py --kv --parts $P --threads $T --reps 2 > $OUT/kv_p${P}_t$T.json 2> $OUT/kv_p${P}_t$T.err || { tail -n 20 $OUT/kv_p${P}_t$T.err; exit 1; }
  echo "parts $P threads $T"; grep "bsdb kv\] 1\|adds:" $OUT/kv_p${P}_t$T.err
done
