#!/bin/bash
# GOV solver iteration: GOV parity tests, phase profile at 1e7 keys, C2 full build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gov_iter
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k gov --timeout 120 --timeout-method thread > gpurun_out/gov_iter/pytest_gov.log 2>&1 || { tail -30 gpurun_out/gov_iter/pytest_gov.log; exit 1; }
tail -1 gpurun_out/gov_iter/pytest_gov.log
BSDB_GOV_PROFILE=1 timeout -k 10 120 python tools/full_build.py --n 10000000 > gpurun_out/gov_iter/gov_prof_10m.log 2>&1 || { tail -20 gpurun_out/gov_iter/gov_prof_10m.log; exit 2; }
grep -v "^W2\|amdgpu.ids" gpurun_out/gov_iter/gov_prof_10m.log | tail -2
timeout -k 10 200 python tools/full_build.py --n 100000000 --reps 2 > gpurun_out/gov_iter/fb_100m.log 2>&1 || { tail -20 gpurun_out/gov_iter/fb_100m.log; exit 3; }
grep -v "^W2\|amdgpu.ids" gpurun_out/gov_iter/fb_100m.log | tail -1
