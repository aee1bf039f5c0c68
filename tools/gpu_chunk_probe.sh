set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 150 python tools/chunk_probe.py 13193787549 2 > gpurun_out/chunk_probe_fe2.log 2>&1
echo "rc=$?" >> gpurun_out/chunk_probe_fe2.log
