cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python tools/mem_probe.py 13193787549 > gpurun_out/mem_probe.log 2>&1; echo "rc=$?" >> gpurun_out/mem_probe.log
