#!/bin/bash
# After a GOV build change: build/parity tests, C1 and C2 timings, C2 kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/c2ab
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_build_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread --durations=5 > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
echo "tests: $(tail -1 $out/pytest.log)"
summ='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=[d[k]["gov_build_ms"] for k in d if k.startswith("rep")][1:]; t=[d[k]["total_ms"] for k in d if k.startswith("rep")][1:]; print("gov ms median %.3f min %.3f; total median %.3f -> %.1f M keys/s" % (sorted(r)[len(r)//2], min(r), sorted(t)[len(t)//2], d["n"]/sorted(t)[len(t)//2]/1e3))'
timeout -k 10 120 python tools/full_build.py --n 1000000 --reps 9 > $out/c1.log 2>&1 || { tail -5 $out/c1.log; exit 2; }
echo "C1: $(python3 -c "$summ" < $out/c1.log)"
timeout -k 10 200 python tools/full_build.py --n 100000000 --reps 4 > $out/c2.log 2>&1 || { tail -5 $out/c2.log; exit 3; }
echo "C2: $(python3 -c "$summ" < $out/c2.log)"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/rp -o c2 --output-format csv -- python tools/full_build.py --n 100000000 --reps 2 > $out/rp.log 2>&1 || { tail -5 $out/rp.log; exit 4; }
python3 -c "
import csv
for r in csv.DictReader(open('$out/rp/c2_kernel_stats.csv')):
    if float(r['AverageNs']) > 2e5: print(r['Name'][:48].ljust(48), r['Calls'], '%.3f ms' % (float(r['AverageNs'])/1e6))
"
