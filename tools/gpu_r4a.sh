#!/bin/bash
# Round 4, first call: box probe, the builder tests, the C4 per-pass trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r4a}; mkdir -p $OUT
[ -z "$NOPROBE" ] && {
  echo "== free"; free -g
  echo "== df"; df -h /tmp /dev/shm "$HOME" "$GRAFT_REPO_ROOT" 2>&1
  echo "== mounts"; grep -E " / | /tmp | /dev/shm " /proc/mounts
  echo "== cgroup"; cat /sys/fs/cgroup/memory.max /sys/fs/cgroup/cpu.max 2>&1
  echo "== cpus"; python3 -c "import os; print(len(os.sched_getaffinity(0)), os.cpu_count())"
  echo "== dd 8 GiB to /tmp (fdatasync)"; dd if=/dev/zero of=/tmp/bsdb_dd_probe bs=64M count=128 conv=fdatasync 2>&1 | tail -1
  rm -f /tmp/bsdb_dd_probe
} > $OUT/box_probe.txt 2>&1
[ -z "$NOPROBE" ] && cat $OUT/box_probe.txt
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_builder_gpu.py} ${KEXPR:+-k "$KEXPR"} -x -v --timeout 600 --timeout-method thread > $OUT/pytest_builder.log 2>&1 || { tail -n 40 $OUT/pytest_builder.log; exit 1; }
tail -n 3 $OUT/pytest_builder.log
[ -n "$NOTRACE" ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/rp -o c4 --output-format csv -- python3 tools/c4_trace.py --host-index > $OUT/c4.log 2>&1 || { tail -20 $OUT/c4.log; exit 3; }
tail -1 $OUT/c4.log
python3 tools/trace_passes.py $OUT/rp/c4_kernel_trace.csv --json $OUT/passes.json
cp $OUT/rp/c4_kernel_stats.csv $OUT/kernel_stats.csv
gzip -c $OUT/rp/c4_kernel_trace.csv > $OUT/kernel_trace.csv.gz
rm -rf $OUT/rp
