#!/bin/bash
# Solver variants (in-tree builds under tools/variants/): GOV parity tests,
# phase profile at 1e7 keys and the C2 full build for each library given.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/govv
for lib in "$@"; do
  tag=$(basename $lib .so)
  export BSDB_LIB=$PWD/$lib
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_build_gpu.py -m gpu -x -q -k "gov or oversized or fvs or range" --timeout 120 --timeout-method thread > gpurun_out/govv/$tag.pytest.log 2>&1 || { echo "$tag tests failed"; tail -30 gpurun_out/govv/$tag.pytest.log; exit 1; }
  echo "$tag: $(tail -1 gpurun_out/govv/$tag.pytest.log)"
  BSDB_GOV_PROFILE=1 timeout -k 10 120 python tools/full_build.py --n 10000000 --reps 1 > gpurun_out/govv/$tag.prof.log 2>&1 || { tail -5 gpurun_out/govv/$tag.prof.log; exit 2; }
  grep "gov-profile" gpurun_out/govv/$tag.prof.log | tail -2
  timeout -k 10 200 python tools/full_build.py --n 100000000 --reps 2 > gpurun_out/govv/$tag.c2.log 2>&1 || { tail -5 gpurun_out/govv/$tag.c2.log; exit 3; }
  echo "$tag C2: $(tail -1 gpurun_out/govv/$tag.c2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["rep1"]["keys_per_s"]/1e6,1), "M keys/s, gov", round(d["rep1"]["gov_build_ms"],1), "ms")')"
done
