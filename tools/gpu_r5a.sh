#!/bin/bash
# Round 5, GPU call A: the config-size solver pins, the
# builder suite after the concurrent-add / spill-mode changes (items 4, 6),
# the writer suite, smoke.  (The 1e9 C3-size builder test runs in call B.)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r5a}; mkdir -p $OUT
export BSDB_TEST_REPORT=$OUT/solver_report.jsonl
timeout -k 10 1080 python -u -m pytest tests/test_builder_gpu.py tests/test_configs_gpu.py -k "not c3_size_host_passes and (builder or spill or kv_ or host_passes or streamed or concurrent or field_for_field or 2e8_slice or empty or errors)" -x -v -s --timeout 900 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -n 40 $OUT/pytest.log; exit 1; }
tail -n 3 $OUT/pytest.log
