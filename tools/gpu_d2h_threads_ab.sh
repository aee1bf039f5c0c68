#!/bin/bash
# C4 exact full build into a host index array: one runtime pageable copy per pass slice
# (BSDB_D2H_THREADS=1) against 8 threads each copying an eighth of it.  Alternated, 2 runs each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-d2h_threads}; mkdir -p $OUT
for rep in 1 2; do
  for t in 1 8; do
    BSDB_D2H_THREADS=$t timeout -k 10 200 python -u tools/c4_trace.py --host-index > $OUT/t${t}_$rep.json 2> $OUT/t${t}_$rep.err || { tail -5 $OUT/t${t}_$rep.err; exit 1; }
    echo "threads $t rep $rep: $(tail -1 $OUT/t${t}_$rep.json)"
  done
done
