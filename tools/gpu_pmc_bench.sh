#!/bin/bash
# HBM traffic of the headline's pass-1 kernel at the bench's own launch size:
# separate --pmc passes (FETCH_SIZE, WRITE_SIZE) over a 1-step bench, then
# tools/pmc_traffic.py (gfx950 corrections) -> gpurun_out/pmc_bench/pmc_pass1.json.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_bench; mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c -d $OUT/$c -o $c --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-full-build > $OUT/$c.log 2>&1 || { echo "pmc $c failed"; tail -n 5 $OUT/$c.log; exit 1; }
done
python3 tools/pmc_traffic.py $(find $OUT/FETCH_SIZE -name "*counter_collection.csv") $(find $OUT/WRITE_SIZE -name "*counter_collection.csv") $OUT/pmc_pass1.json ${ROUND:-6}
