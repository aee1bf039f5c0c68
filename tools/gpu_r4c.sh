#!/bin/bash
# Round 4 measurement batch B: the end-to-end legs with phase prints (kv.db -> index at C2; C4 host keys ->
# index.db through mapped writes), the slice-copy threads A/B of the C4 exact build, then pass 1's PMC stalls.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-e2e}; mkdir -p $OUT
BSDB_BUILDER_PROFILE=1 timeout -k 10 300 python -u tools/e2e_legs.py --kv --c4 > $OUT/legs.json 2> $OUT/legs.err || { tail -20 $OUT/legs.err; exit 1; }
cat $OUT/legs.json; grep "bsdb" $OUT/legs.err | tail -20
TAG=${TAG1:-d2h_threads} bash tools/gpu_d2h_threads_ab.sh || exit 2
TAG=${TAG2:-pmc_stalls} bash tools/gpu_pmc_stalls.sh || exit 3
