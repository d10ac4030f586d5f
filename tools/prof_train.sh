#!/bin/bash
# rocprofv3 kernel summary of the timed config-2 train step alone (bench --only train).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -rf /tmp/prof_train
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_train -o run -- \
  python bench.py --only train --steps 4 --warmup 1 --no-cpu --xattn-steps 0 --st-steps 0 \
  > gpurun_out/prof_train.json 2> gpurun_out/prof_train.err || { tail gpurun_out/prof_train.err; exit 1; }
db=$(find /tmp/prof_train -name '*.db' | head -n 1)
python tools/prof_summary.py "$db" > gpurun_out/train_kernel_stats.md
python tools/prof_steps.py "$db" | tee gpurun_out/train_steps.txt
