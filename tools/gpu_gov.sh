#!/bin/bash
# Device GOV build parity on the GPU box.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "gov_build" > gpurun_out/pytest_gov.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gov.log
exit $rc
