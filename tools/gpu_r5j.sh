#!/bin/bash
# Round 5, GPU call J: what a third / fourth solver workgroup per CU is worth
# (VERDICT r4 item 2's premise), priced on measurement builds with a smaller
# mean bucket so that the per-bucket LDS state fits 3 (4) workgroups:
# the same library run with its full count and with fewer (BSDB_GOV_PER_CU:
# grid + LDS padding).  C2-size key sets (1e8), ranks checked as a bijection.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5j; mkdir -p $OUT
run() {  # tag lib per_cu
  local tag=$1 lib=$2 k=$3
  BSDB_LIB=$PWD/$lib BSDB_GOV_PER_CU=$k BSDB_GOV_PROFILE=1 timeout -k 10 120 python tools/full_build.py --n 10000000 --reps 1 > $OUT/$tag.prof.log 2>&1 || { tail -5 $OUT/$tag.prof.log; return 1; }
  BSDB_LIB=$PWD/$lib BSDB_GOV_PER_CU=$k timeout -k 10 200 python tools/full_build.py --n 100000000 --reps 3 > $OUT/$tag.c2.log 2>&1 || { tail -5 $OUT/$tag.c2.log; return 2; }
  echo "$tag: $(grep 'workgroups per CU' $OUT/$tag.prof.log | cut -c1-120) | C2 gov ms: $(python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print([round(d[f"rep{i}"]["gov_build_ms"],1) for i in range(3)], [round(d[f"rep{i}"]["keys_per_s"]/1e6,1) for i in range(3)])' $OUT/$tag.c2.log)"
}
run prod_p2 bsdb_amd/libbsdb_mi355x.so 2 &&
run b1000_t512_p2 tools/variants/probe_b1000_t512_p2.so 2 &&
run b1000_t256_p3 tools/variants/probe_b1000_t256_p3.so 3 &&
run b1000_t256_p3_at2 tools/variants/probe_b1000_t256_p3.so 2 &&
run b750_t512_p2 tools/variants/probe_b750_t512_p2.so 2 &&
run b750_t256_p4 tools/variants/probe_b750_t256_p4.so 4 &&
run b750_t256_p4_at3 tools/variants/probe_b750_t256_p4.so 3 &&
run b750_t256_p4_at2 tools/variants/probe_b750_t256_p4.so 2
