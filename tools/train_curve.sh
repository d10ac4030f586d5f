#!/bin/bash
# Loss curves of the drop-in train.py on synthetic config-2 clips (GPU box), 8 epochs x 40
# steps per (attention mode, lr) pair given as arguments, e.g.
#   bash tools/train_curve.sh "joint 1e-3" "spatial_temporal 1e-3" "joint 1e-2"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TR=lipreading-video-generation_amd/video-generation/diffusion/train.py
COMMON="--dims 3 --frames 16 --image-size 128 --batch-size 1 --epochs 8 --steps-per-epoch 40 \
  --random-audio-encoder --reinit-nonzero --ckpt /tmp/curve.pth"
for spec in "$@"; do
  set -- $spec
  echo "== attention $1, lr $2" | tee -a gpurun_out/train_curve.txt
  timeout -k 10 400 python3 -u $TR $COMMON --attention-mode $1 --lr $2 >> gpurun_out/train_curve.txt 2>&1 \
    || { echo "rc=$?"; tail -5 gpurun_out/train_curve.txt; exit 1; }
done
grep -E "^==|Finished" gpurun_out/train_curve.txt
