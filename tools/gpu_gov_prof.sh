#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export BSDB_GOV_PROFILE=1
cd $GRAFT_REPO_ROOT; timeout -k 10 120 python tools/full_build.py --n 10000000 > gpurun_out/gov_prof_10m.log 2>&1
rc=$?
grep -v "^W2\|amdgpu.ids" gpurun_out/gov_prof_10m.log | tail -5
exit $rc
