#!/bin/bash
# Pass 1's memory-traffic limit at C4: the production kernel (BSDB_D13_VARIANT=0) against the
# same kernel with the hash replaced by a 2-instruction stand-in (VARIANT=12, results invalid):
# identical loads, LDS bins, cursor atomics and id write-out.  Alternated, 2 runs each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-mixlimit}; mkdir -p $OUT
for rep in 1 2; do
  for v in 0 12; do
    BSDB_D13_VARIANT=$v timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-full-build > $OUT/v${v}_$rep.json 2> $OUT/v${v}_$rep.err || { tail -5 $OUT/v${v}_$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/v${v}_$rep.json')); print('variant $v rep $rep', round(d['ms_per_step'],2), d['kernel_ms_per_step'], d['check'])"
  done
done
