#!/bin/bash
# (Round 4: the panel Gauss-Jordan was not kept and its code is gone, DESIGN §4.3;
# this is the script that ran that A/B.)
# A/B of the heavy system's Gauss-Jordan: panels of 8 columns (default) against the column loop
# (BSDB_GOV_GJ_COLUMN=1), same library: GOV parity tests in both modes, the phase profile at 1e7
# keys and the C2 full build, alternated.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${TAG:-gjpanel}
mkdir -p $out
for mode in panel column; do
  if [ $mode = column ]; then export BSDB_GOV_GJ_COLUMN=1; else unset BSDB_GOV_GJ_COLUMN; fi
  timeout -k 10 400 python -u -m pytest tests/test_build_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/$mode.pytest.log 2>&1 || { echo "$mode tests failed"; tail -30 $out/$mode.pytest.log; exit 1; }
  echo "$mode: $(tail -1 $out/$mode.pytest.log)"
  BSDB_GOV_PROFILE=1 timeout -k 10 120 python tools/full_build.py --n 10000000 --reps 1 > $out/$mode.prof.log 2>&1 || { tail -5 $out/$mode.prof.log; exit 2; }
  grep "gov-profile\] m=" $out/$mode.prof.log | tr ' ' '\n' | grep -E "^(bfs|fvs_select|fvs_forms|fvs_gauss_jordan|dense|n_seeds)=" | tr '\n' ' '; echo
done
for rep in 1 2; do
  for mode in panel column; do
    if [ $mode = column ]; then export BSDB_GOV_GJ_COLUMN=1; else unset BSDB_GOV_GJ_COLUMN; fi
    timeout -k 10 200 python tools/full_build.py --n 100000000 --reps 2 > $out/$mode.c2.$rep.log 2>&1 || { tail -5 $out/$mode.c2.$rep.log; exit 3; }
    echo "$mode C2 rep $rep: $(tail -1 $out/$mode.c2.$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["rep1"]["keys_per_s"]/1e6,1), "M keys/s, gov", round(d["rep1"]["gov_build_ms"],1), "ms")')"
  done
done
