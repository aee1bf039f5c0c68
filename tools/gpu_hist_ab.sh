#!/bin/bash
# Headline A/B (pass-1 kernel change): parity tests + the full-size C4
# histogram test on the new library, then the headline bench alternated.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/hab
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
echo "parity: $(tail -1 $out/pytest.log)"
timeout -k 10 400 python -u -m pytest tests/test_configs_gpu.py -m gpu -x -q -k "c4_full_size_histogram" --timeout 300 --timeout-method thread > $out/pytest_c4.log 2>&1 || { tail -40 $out/pytest_c4.log; exit 2; }
echo "c4 histogram: $(tail -1 $out/pytest_c4.log)"
for rep in 1 2 3; do
  for lib in tools/variants/base.so bsdb_amd/libbsdb_mi355x.so; do
    tag=$(basename $lib .so)
    BSDB_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-full-build --no-cpu > $out/$tag.$rep.json 2> $out/$tag.$rep.err || { tail -5 $out/$tag.$rep.err; exit 3; }
    python3 -c "
import json; d=json.loads(open('$out/$tag.$rep.json').read().strip().splitlines()[-1])
print('$tag rep $rep: %.1f G  %.2f ms  p1 %.2f p2 %.2f' % (d['value']/1e9, d['ms_per_step'], d['kernel_ms_per_step']['pass1'], d['kernel_ms_per_step']['pass2']))"
  done
done
