cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 100 python tools/kbench.py --n 2147483648 --m 8795859 --reps 1 --frontends 0,2 --chunks 0,1073741824 > gpurun_out/kb_big_m.log 2>&1; echo "rc=$?" >> gpurun_out/kb_big_m.log
