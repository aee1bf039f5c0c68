#!/bin/bash
# Solver tunables on one box: the speculation cap (BSDB_GOV_SPEC, runtime) at
# C1 and C2 on the production library, then C2 for each variant library given
# (e.g. -DGOV_FVS_MIN / -DGOV_PICK_REPS builds under tools/variants/).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${TAG:-sweep}; mkdir -p $out
c2() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d["rep1"]["keys_per_s"]/1e6,1), "M keys/s, gov", round(d["rep1"]["gov_build_ms"],2), "ms")'; }
for spec in 1 2 3 4; do
  for n in 1000000 100000000; do
    BSDB_GOV_SPEC=$spec timeout -k 10 200 python tools/full_build.py --n $n --reps 2 > $out/spec$spec.$n.log 2>&1 || { tail -5 $out/spec$spec.$n.log; exit 1; }
    echo "spec $spec n $n: $(tail -1 $out/spec$spec.$n.log | c2)"
  done
done
for lib in "$@"; do
  tag=$(basename $lib .so)
  BSDB_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_build_gpu.py -m gpu -x -q -k "gov or oversized or fvs or range" --timeout 120 --timeout-method thread > $out/$tag.pytest.log 2>&1 || { echo "$tag tests failed"; tail -30 $out/$tag.pytest.log; exit 2; }
  BSDB_LIB=$PWD/$lib timeout -k 10 200 python tools/full_build.py --n 100000000 --reps 2 > $out/$tag.c2.log 2>&1 || { tail -5 $out/$tag.c2.log; exit 3; }
  echo "$tag: $(tail -1 $out/$tag.pytest.log) C2 $(tail -1 $out/$tag.c2.log | c2)"
done
