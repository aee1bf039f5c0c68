#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
BSDB_D13_VARIANT=6 timeout -k 10 200 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "k13 or full_size" > gpurun_out/pytest_v6.log 2>&1 || { tail -30 gpurun_out/pytest_v6.log; exit 1; }
tail -2 gpurun_out/pytest_v6.log
for V in 0 6 0 6; do
  BSDB_D13_VARIANT=$V timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_v$V.json 2> gpurun_out/bench_v$V.err || { tail -20 gpurun_out/bench_v$V.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_v$V.json')); print('V=$V', round(d['value']/1e9,1), 'G keys/s', d['kernel_ms_per_step'], round(d['roofline']['frac'],4))"
done
