#!/bin/bash
# 2-rank rehearsal of the ViViT config-5 bench leg on a one-GPU box (ranks share cuda:0 over
# gloo): the graph-captured step (graph 1: fwd + bwd + flatten, one all-reduce, graph 2:
# average + AdamW), then the eager step with the bucketed all-reduce hooks (the unused
# pooler parameters ride along as zeros); barrier + max-over-ranks timing.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
VDIFF_DIST_BACKEND=gloo timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 \
  --only vivit --vivit-steps 10 --vivit-graph-ddp --no-cpu > gpurun_out/ddp_rehearsal_vivit.json 2> gpurun_out/ddp_rehearsal_vivit.err
tail -c 700 gpurun_out/ddp_rehearsal_vivit.json
VDIFF_DIST_BACKEND=gloo timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 2 \
  --only vivit --vivit-steps 10 --no-cpu > gpurun_out/ddp_rehearsal_vivit_eager.json 2> gpurun_out/ddp_rehearsal_vivit_eager.err
tail -c 700 gpurun_out/ddp_rehearsal_vivit_eager.json
VDIFF_DIST_BACKEND=gloo timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29543 tools/vivit_ddp_check.py \
  > gpurun_out/vivit_ddp_check.log 2>&1
tail -2 gpurun_out/vivit_ddp_check.log
