#!/bin/bash
# GOV evidence: phase profile at 1e7 keys, full builds at C2 (1e8) and C3 (1e9,
# approximate), rocprof kernel stats of the C2 build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gov
BSDB_GOV_PROFILE=1 timeout -k 10 120 python tools/full_build.py --n 10000000 > gpurun_out/gov/gov_prof_10m.log 2>&1 || { tail -20 gpurun_out/gov/gov_prof_10m.log; exit 1; }
grep -v "^W2\|amdgpu.ids" gpurun_out/gov/gov_prof_10m.log | tail -4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/gov/prof_fb -o fb --output-format csv -- python3 tools/full_build.py --n 100000000 --reps 2 > gpurun_out/gov/fb_100m.log 2>&1 || { tail -20 gpurun_out/gov/fb_100m.log; exit 2; }
grep -v "^W2\|amdgpu.ids" gpurun_out/gov/fb_100m.log | tail -3
timeout -k 10 300 python tools/full_build.py --n 1000000000 --approx --reps 1 > gpurun_out/gov/fb_1b.log 2>&1 || { tail -20 gpurun_out/gov/fb_1b.log; exit 3; }
grep -v "^W2\|amdgpu.ids" gpurun_out/gov/fb_1b.log | tail -3
