#!/bin/bash
# Round 5, GPU call D: the kv.db leg with the release timing, then the
# narrow-row register Gauss-Jordan variants against production.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r5d}; mkdir -p $OUT
BSDB_BUILDER_PROFILE=1 timeout -k 10 300 python -u tools/e2e_legs.py --kv --reps 2 > $OUT/kv.json 2> $OUT/kv.err || { tail -n 20 $OUT/kv.err; exit 5; }
cut -c1-120 $OUT/kv.json; grep "bsdb kv\|adds:" $OUT/kv.err
bash tools/gpu_gov_variants.sh "$@"
