#!/bin/bash
# The N>1 bench path rehearsed on a one-GPU box: two ranks (torch.distributed.run)
# share cuda:0 with the gloo backend (RCCL refuses two ranks on one device), so
# the sharding, per-rank histograms, the all-reduce of the counts, the barriers
# and the max-over-ranks timing run as on a node; the in-ABI RCCL collective does not.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/two_rank; mkdir -p $out
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
tail -n 1 $out/bench.json | cut -c1-600
