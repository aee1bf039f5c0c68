#!/bin/bash
# Round 4: builder/kv GPU tests on the production library, then the
# 256-thread solver probe against production (tools/gpu_gov_variants.sh).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4d
timeout -k 10 400 python -u -m pytest tests/test_builder_gpu.py tests/test_writer_gpu.py tests/test_kv_scan.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4d/builder.log 2>&1 || { tail -30 gpurun_out/r4d/builder.log; exit 1; }
tail -1 gpurun_out/r4d/builder.log
bash tools/gpu_gov_variants.sh "$@"
