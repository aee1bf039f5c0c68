#!/bin/bash
# C1 after a change: GOV parity tests, C1 timing (9 reps), C1 kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/c1ab
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_build_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
echo "tests: $(tail -1 $out/pytest.log)"
summ='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=[d[k]["gov_build_ms"] for k in d if k.startswith("rep")][1:]; t=[d[k]["total_ms"] for k in d if k.startswith("rep")][1:]; print("gov ms median %.3f min %.3f; total median %.3f" % (sorted(r)[len(r)//2], min(r), sorted(t)[len(t)//2]))'
for rep in 1 2; do
  timeout -k 10 120 python tools/full_build.py --n 1000000 --reps 9 > $out/c1.$rep.log 2>&1 || { tail -5 $out/c1.$rep.log; exit 2; }
  echo "C1 rep $rep: $(python3 -c "$summ" < $out/c1.$rep.log)"
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $out/rp -o c1 --output-format csv -- python tools/full_build.py --n 1000000 --reps 5 > $out/rp.log 2>&1 || { tail -5 $out/rp.log; exit 3; }
cut -d, -f1-4 $out/rp/c1_kernel_stats.csv | head -9
