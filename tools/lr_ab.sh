#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lr in 1e-3 1e-4 1e-3 1e-4; do
  timeout -k 10 300 python3 -u bench.py --only train --steps 20 --warmup 5 --no-cpu --xattn-steps 0 \
    --st-steps 0 --lr $lr > gpurun_out/lr_$lr.json 2>/dev/null || { echo "rc=$?"; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/lr_$lr.json').read().strip().splitlines()[-1])
print('lr $lr', d['value'], d['ms_per_step'], d['roofline']['frac'], d['train_losses'][0], d['train_losses'][-1])" | tee -a gpurun_out/lr_ab.txt
done
