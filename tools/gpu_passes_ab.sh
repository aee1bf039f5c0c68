#!/bin/bash
# Pass builds after a change: pass tests, then the C4 exact full build at size (bench leg).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/passes
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_build_gpu.py -m gpu -x -q -k "passes" --timeout 150 --timeout-method thread > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
echo "tests: $(tail -1 $out/pytest.log)"
timeout -k 10 500 python -u -m pytest tests/test_configs_gpu.py -m gpu -x -q -k "c4_exact or c5_full" --timeout 400 --timeout-method thread > $out/pytest_cfg.log 2>&1 || { tail -40 $out/pytest_cfg.log; exit 2; }
echo "config tests: $(tail -1 $out/pytest_cfg.log)"
