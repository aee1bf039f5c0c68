#!/bin/bash
# Round 5, GPU call K: the third solver workgroup per CU at a mean bucket of
# 950 keys (state 52.9 KB: three fit), against the same library held to two.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5k; mkdir -p $OUT
run() {  # tag lib per_cu
  local tag=$1 lib=$2 k=$3
  BSDB_LIB=$PWD/$lib BSDB_GOV_PER_CU=$k timeout -k 10 200 python tools/full_build.py --n 100000000 --reps 3 > $OUT/$tag.c2.log 2>&1 || { tail -5 $OUT/$tag.c2.log; return 2; }
  echo "$tag: C2 gov ms: $(python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print([round(d[f"rep{i}"]["gov_build_ms"],1) for i in range(3)], [round(d[f"rep{i}"]["keys_per_s"]/1e6,1) for i in range(3)])' $OUT/$tag.c2.log)"
}
run b950_t256_p3 tools/variants/probe_b950_t256_p3.so 3 &&
run b950_t256_p3_at2 tools/variants/probe_b950_t256_p3.so 2 &&
run b950_t256_p3_again tools/variants/probe_b950_t256_p3.so 3 &&
run b950_t256_p3_at2_again tools/variants/probe_b950_t256_p3.so 2
