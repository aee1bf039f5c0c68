#!/bin/bash
# Register / scratch / LDS use of the solver kernels (device-only compile with
# the resource-usage remarks; nothing is built).  usage: tools/solver_resources.sh [-DFLAG ...]
HERE=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -c -o /dev/null "$@" \
  -Rpass-analysis=kernel-resource-usage "$HERE/bsdb_amd/csrc/bsdb_capi.hip" 2>&1 |
  grep -A11 "Function Name: _ZN4bsdb11k_gov_solveILb0EEEvNS_9SolveArgsE" | grep -E "VGPRs:|AGPRs|ScratchSize|Occupancy|LDS Size|SGPRs:"
