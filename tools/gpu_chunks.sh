#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/chunks
for ch in ${1//,/ }; do
  timeout -k 10 300 python -u bench.py --no-cpu --steps 5 --warmup 2 --chunk $ch > gpurun_out/chunks/c$ch.log 2>&1 || { echo "chunk $ch failed"; tail -5 gpurun_out/chunks/c$ch.log; exit 1; }
  echo "chunk $ch: $(tail -1 gpurun_out/chunks/c$ch.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e9,1), d["kernel_ms_per_step"])')"
done
