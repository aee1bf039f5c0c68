#!/bin/bash
# Round 5, GPU call Z: the leader-wave panel Gauss-Jordan (production now):
# GOV parity + C2 A/B against the previous form, then the config-size pins.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5z; mkdir -p $OUT
bash tools/gpu_gov_variants.sh tools/variants/lead5.so tools/variants/lead6.so tools/variants/base.so tools/variants/lead6.so || exit 1
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/test_configs_gpu.py -k "field_for_field or equals_oracle" > $OUT/pins.log 2>&1; rc=$?; tail -n 8 $OUT/pins.log; exit $rc
