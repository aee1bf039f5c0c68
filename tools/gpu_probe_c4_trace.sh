#!/bin/bash
# Box probe (memory, file systems, write rate) + a kernel trace of the C4
# exact full build on one GPU (per-pass solve / oversized-bucket solve timing).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-c4trace}; mkdir -p $OUT
{
  echo "== free"; free -g
  echo "== df"; df -h /tmp /dev/shm "$HOME" "$GRAFT_REPO_ROOT" 2>&1
  echo "== mounts"; grep -E " / | /tmp | /dev/shm " /proc/mounts
  echo "== cgroup"; cat /sys/fs/cgroup/memory.max /sys/fs/cgroup/cpu.max 2>&1
  echo "== nproc"; nproc; python3 -c "import os; print(len(os.sched_getaffinity(0)))"
  echo "== dd 8 GiB to /tmp (fdatasync)"; dd if=/dev/zero of=/tmp/bsdb_dd_probe bs=64M count=128 conv=fdatasync 2>&1 | tail -1
  rm -f /tmp/bsdb_dd_probe
} > $OUT/box_probe.txt 2>&1
cat $OUT/box_probe.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/rp -o c4 --output-format csv -- python3 tools/c4_trace.py --host-index > $OUT/c4.log 2>&1 || { tail -20 $OUT/c4.log; exit 3; }
tail -1 $OUT/c4.log
python3 tools/trace_passes.py $OUT/rp/c4_kernel_trace.csv --json $OUT/passes.json
find $OUT/rp -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
find $OUT/rp -name "*kernel_trace.csv" -exec gzip -c {} \; > $OUT/kernel_trace.csv.gz
