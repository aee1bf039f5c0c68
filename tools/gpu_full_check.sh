#!/bin/bash
# Whole GPU suite (split in two pytest processes: the long config-size file
# second), then the bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/full
timeout -k 10 900 python -u -m pytest tests -m gpu --deselect tests/test_configs_gpu.py -q --timeout 300 --timeout-method thread --ignore=tests/test_configs_gpu.py > gpurun_out/full/tests_a.log 2>&1 || { tail -40 gpurun_out/full/tests_a.log; exit 1; }
tail -2 gpurun_out/full/tests_a.log
timeout -k 10 900 python -u -m pytest tests/test_configs_gpu.py -v --timeout 900 --timeout-method thread --durations=0 > gpurun_out/full/tests_b.log 2>&1 || { tail -40 gpurun_out/full/tests_b.log; exit 2; }
tail -8 gpurun_out/full/tests_b.log
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > gpurun_out/full/bench.json 2> gpurun_out/full/bench.err || { tail -20 gpurun_out/full/bench.err; exit 3; }
tail -1 gpurun_out/full/bench.json
