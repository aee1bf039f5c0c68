#!/bin/bash
# One GPU call: the whole -m gpu suite, the bench line, the rocprofv3 kernel-trace summary
# of the headline alone (--no-full-build: its pass-1 launches are the bench's roofline launches).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-round}; mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 700 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -n 40 $OUT/pytest_gpu.log; exit 1; }
tail -n 2 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -n 20 $OUT/smoke.log; exit 4; }
tail -n 1 $OUT/smoke.log
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 700 python -u bench.py --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail -n 20 $OUT/bench.err; exit 2; }
tail -n 1 $OUT/bench.json | cut -c1-400
[ -n "$NOPROF" ] && exit 0
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-full-build > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { tail -n 20 $OUT/prof_bench.err; exit 3; }
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
head -n 12 $OUT/kernel_stats.csv | cut -c1-160
[ -n "$NOKV" ] && exit 0
BSDB_BUILDER_PROFILE=1 timeout -k 10 300 python -u tools/e2e_legs.py --kv --reps 2 > $OUT/kv.json 2> $OUT/kv.err || { tail -n 20 $OUT/kv.err; exit 5; }
grep "bsdb kv\|adds:" $OUT/kv.err
