#!/bin/bash
# pass-1 time of the var-len kernel's profiling variants (BSDB_D13_VARIANT).
set -o pipefail
TAG=${1:-varv}; shift
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/$TAG; export TMPDIR=/tmp
for v in "$@"; do
  BSDB_D13_VARIANT=$v timeout -k 10 100 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/v$v -o v$v --output-format csv -- python3 tools/varlen_bench.py --fe 0 --reps 2 > gpurun_out/$TAG/v$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/$TAG/v$v.log; exit 1; }
  python3 - "$TAG" "$v" <<'PY'
import csv, sys
tag, v = sys.argv[1], sys.argv[2]
for r in csv.DictReader(open(f"gpurun_out/{tag}/v{v}/v{v}_kernel_stats.csv")):
    if "vare" in r["Name"] or "pass2b" in r["Name"]:
        print(f"v{v}: {r['Name'][:28]} {float(r['AverageNs'])/1e6:.3f} ms")
PY
done
