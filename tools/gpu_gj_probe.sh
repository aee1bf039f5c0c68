#!/bin/bash
# Phase cycles (BSDB_GOV_PROFILE, 1e7 keys) of measurement builds whose
# results may be invalid (the run's own checks are not required to pass).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gjp
for lib in "$@"; do
  tag=$(basename $lib .so)
  BSDB_LIB=$PWD/$lib BSDB_GOV_PROFILE=1 timeout -k 10 120 python tools/full_build.py --n 10000000 --reps 1 > gpurun_out/gjp/$tag.log 2>&1
  rc=$?
  [ $rc -ge 124 ] && { echo "$tag: rc $rc"; exit 1; }
  echo "$tag (rc $rc): $(grep 'gov-profile\] m=' gpurun_out/gjp/$tag.log | grep -o 'fvs_gauss_jordan=[^ ]*\|gj_columns=[^ ]*' | tr '\n' ' ')"
done
