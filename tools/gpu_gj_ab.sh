#!/bin/bash
# A/B of the register-resident heavy Gauss-Jordan (default) against the
# workgroup form (BSDB_GOV_GJ_WG=1), same library: GOV parity tests in both
# modes, phase profile at 1e7 keys and the C2 full build, alternated.
# Then the headline ceiling probe (tools/ceiling_probe, built beforehand).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/gjab
mkdir -p $out
for mode in reg wg; do
  if [ $mode = wg ]; then export BSDB_GOV_GJ_WG=1; else unset BSDB_GOV_GJ_WG; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_build_gpu.py -m gpu -x -q -k "gov or oversized or fvs or range" --timeout 120 --timeout-method thread > $out/$mode.pytest.log 2>&1 || { echo "$mode tests failed"; tail -30 $out/$mode.pytest.log; exit 1; }
  echo "$mode: $(tail -1 $out/$mode.pytest.log)"
  BSDB_GOV_PROFILE=1 timeout -k 10 120 python tools/full_build.py --n 10000000 --reps 1 > $out/$mode.prof.log 2>&1 || { tail -5 $out/$mode.prof.log; exit 2; }
  grep "gov-profile\] m=" $out/$mode.prof.log | tr ' ' '\n' | grep -E "^(bfs|fvs_select|fvs_forms|fvs_gauss_jordan|dense|n_seeds)=" | tr '\n' ' '; echo
done
for rep in 1 2; do
  for mode in reg wg; do
    if [ $mode = wg ]; then export BSDB_GOV_GJ_WG=1; else unset BSDB_GOV_GJ_WG; fi
    timeout -k 10 200 python tools/full_build.py --n 100000000 --reps 2 > $out/$mode.c2.$rep.log 2>&1 || { tail -5 $out/$mode.c2.$rep.log; exit 3; }
    echo "$mode C2 rep $rep: $(tail -1 $out/$mode.c2.$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["rep1"]["keys_per_s"]/1e6,1), "M keys/s, gov", round(d["rep1"]["gov_build_ms"],1), "ms")')"
  done
done
unset BSDB_GOV_GJ_WG
if [ -x tools/ceiling_probe ]; then
  timeout -k 10 240 ./tools/ceiling_probe > $out/ceiling_probe_c4.json || exit 4
  cat $out/ceiling_probe_c4.json
fi
