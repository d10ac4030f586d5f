#!/bin/bash
# 2-rank rehearsal of the ViViT config-5 bench leg on a one-GPU box (ranks share cuda:0 over
# gloo): eager steps, bucketed all-reduce hooks (the unused pooler parameters ride along as
# zeros), barrier + max-over-ranks timing.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
VDIFF_DIST_BACKEND=gloo timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 \
  --only vivit --vivit-steps 10 --no-cpu > gpurun_out/ddp_rehearsal_vivit.json 2> gpurun_out/ddp_rehearsal_vivit.err
tail -c 700 gpurun_out/ddp_rehearsal_vivit.json
