#!/bin/bash
# Pass-1 time at fewer persistent workgroups (BSDB_D13_GRID): how much of the
# chip pass 1 needs (tools/pass_split.py, C4 size).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/grid
for g in ${GRIDS:-256 240 224 192 128}; do
  BSDB_D13_GRID=$g timeout -k 10 150 python tools/pass_split.py --reps 4 >> gpurun_out/grid/sweep.jsonl 2> gpurun_out/grid/g$g.err || exit 1
done
cat gpurun_out/grid/sweep.jsonl
