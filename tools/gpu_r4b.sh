#!/bin/bash
# Round 4 measurement batch A: the panel Gauss-Jordan A/B (parity + phase profile + C2), then pass 1's
# mix-limit A/B.  Each step under its own time limit; the first failure ends the call.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-gjpanel} bash tools/gpu_gj_panel_ab.sh || exit 1
TAG=${TAG2:-mixlimit} bash tools/gpu_mixlimit.sh || exit 2
