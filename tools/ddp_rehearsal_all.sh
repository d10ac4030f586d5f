#!/bin/bash
# Every bench leg over N ranks sharing cuda:0 (gloo), launched as the driver launches the
# multi-GPU bench (torch.distributed.run):  bash tools/ddp_rehearsal_all.sh [N]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
N=${1:-2}
VDIFF_DIST_BACKEND=gloo timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus $N \
  --steps 2 --warmup 1 --c4-steps ${C4:-1} --vivit-steps 3 --xattn-steps 1 --st-steps 1 --no-cpu $EXTRA \
  > gpurun_out/ddp_rehearsal_all.json 2> gpurun_out/ddp_rehearsal_all.err
rc=$?; tail -c 1500 gpurun_out/ddp_rehearsal_all.json; tail -5 gpurun_out/ddp_rehearsal_all.err; exit $rc
