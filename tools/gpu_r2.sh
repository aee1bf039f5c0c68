#!/bin/bash
# Round-2 check: new GPU tests, then the bench line (one GPU call).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r2; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest ${TESTS:-tests/test_build_gpu.py tests/test_writer_gpu.py tests/test_distributed.py} -v --timeout 300 --timeout-method thread > gpurun_out/r2/tests.log 2>&1 || { tail -40 gpurun_out/r2/tests.log; exit 1; }
tail -3 gpurun_out/r2/tests.log
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r2/bench.json 2> gpurun_out/r2/bench.err || { tail -20 gpurun_out/r2/bench.err; exit 2; }
tail -1 gpurun_out/r2/bench.json
