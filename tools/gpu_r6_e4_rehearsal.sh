#!/bin/bash
# Round 6: the N>1 bench legs rehearsed on a one-GPU box -- two ranks
# (torch.distributed.run) share cuda:0 over gloo (RCCL refuses two ranks on one
# device): the histogram stage and the E4 full build over the ranks (hash ->
# owner partition -> all-to-all -> window build -> index slots to host -> the
# windows assembled on rank 0), sized to fit two ranks on one GPU.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${TAG:-r6/e4_rehearsal}; mkdir -p $out
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo --num-keys 2000000000 --e4-keys 200000000 --e4-reps 2 \
  > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
tail -n 1 $out/bench.json | cut -c1-1500
