#!/bin/bash
# Round 2: train-step breakdown, rocprofv3 kernel summary of the train step, attention A/B
# at head_dim 128 / 256.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/step_breakdown.py > gpurun_out/breakdown.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/step_breakdown.py --bf16-w2v >> gpurun_out/breakdown.txt 2>&1 || exit 1
cat gpurun_out/breakdown.txt | grep "{"
rm -rf /tmp/prof_train
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_train -o run -- \
  python bench.py --only train --steps 3 --warmup 1 --no-cpu --xattn-steps 0 \
  > gpurun_out/prof_train.json 2> gpurun_out/prof_train.err || exit 1
db=$(find /tmp/prof_train -name '*.db' | head -n 1)
python tools/prof_summary.py "$db" > gpurun_out/r02_train_kernel_stats.md
head -40 gpurun_out/r02_train_kernel_stats.md
for cfg in auto p4 w8 base; do
  echo "== d128 cfg=$cfg"
  VDIFF_ATTN_CFG=$cfg timeout -k 10 150 python -u tools/attn_bench.py --nocheck 3 --only 128 || exit 1
done
echo "== d256 auto"
timeout -k 10 150 python -u tools/attn_bench.py --nocheck 3 --only 256 || exit 1
