#!/bin/bash
# Multi-rank rehearsal of bench.py on a one-GPU box: N ranks share cuda:0 over gloo
# (RCCL refuses two ranks on one device).  Exercises rendezvous, parameter broadcast,
# the bucketed all-reduce hooks, barrier + max-over-ranks timing and the rank-0 JSON line.
#   bash tools/ddp_rehearsal.sh [N]
set -e
cd "$GRAFT_REPO_ROOT"
N=${1:-2}
mkdir -p gpurun_out
VDIFF_DIST_BACKEND=gloo timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus $N \
  --steps 2 --warmup 1 --only train --no-cpu > gpurun_out/ddp_rehearsal.json 2> gpurun_out/ddp_rehearsal.err
tail -c 600 gpurun_out/ddp_rehearsal.json
