#!/bin/bash
# Round 5, GPU call E: the early orientation count (solver) -- GOV parity,
# the config-size pins, profile + C2 against the previous solver -- and the
# kv.db leg with the partition reaper.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r5e}; mkdir -p $OUT
export BSDB_TEST_REPORT=$OUT/solver_report.jsonl
timeout -k 10 700 python -u -m pytest tests/test_build_gpu.py tests/test_gpu_parity.py tests/test_configs_gpu.py -k "gov or oversized or fvs or range or passes or field_for_field or 2e8_slice or varlen_passes or c5_checksum16" -x -q --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -n 40 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
BSDB_BUILDER_PROFILE=1 timeout -k 10 300 python -u tools/e2e_legs.py --kv --reps 2 > $OUT/kv.json 2> $OUT/kv.err || { tail -n 20 $OUT/kv.err; exit 5; }
cut -c1-120 $OUT/kv.json; grep "bsdb kv\|adds:" $OUT/kv.err
for lib in tools/variants/t512.so tools/variants/main_cnt.so tools/variants/t512.so tools/variants/main_cnt.so; do
  tag=$(basename $lib .so)
  BSDB_LIB=$PWD/$lib timeout -k 10 200 python tools/full_build.py --n 100000000 --reps 2 > $OUT/$tag.c2.log 2>&1 || { tail -5 $OUT/$tag.c2.log; exit 3; }
  echo "$tag C2: $(tail -1 $OUT/$tag.c2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["rep1"]["keys_per_s"]/1e6,1), "M keys/s, gov", round(d["rep1"]["gov_build_ms"],1), "ms")')"
done
BSDB_LIB=$PWD/tools/variants/main_cnt.so BSDB_GOV_PROFILE=1 timeout -k 10 120 python tools/full_build.py --n 10000000 --reps 1 > $OUT/main_cnt.prof.log 2>&1 || exit 4
grep "gov-profile" $OUT/main_cnt.prof.log | tail -1 | cut -c1-400
