#!/bin/bash
# Round 4 measurement batch B: slice-copy threads A/B of the C4 exact build, then pass 1's PMC stall breakdown.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-d2h_threads} bash tools/gpu_d2h_threads_ab.sh || exit 1
TAG=${TAG2:-pmc_stalls} bash tools/gpu_pmc_stalls.sh || exit 2
