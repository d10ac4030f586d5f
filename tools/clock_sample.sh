#!/bin/bash
# Samples the GPU's current clocks and power (rocm-smi, read-only) while tools/step_gap.py
# trains at lr 0 and then lr 1e-2 (GPU box): bash tools/clock_sample.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lr in 0 1e-2; do
  timeout -k 10 200 python -u tools/step_gap.py --rounds 5 --lr $lr > gpurun_out/clock_step_$lr.txt 2>&1 &
  pid=$!
  sleep 25
  for i in 1 2 3 4 5; do
    echo "== lr $lr sample $i" >> gpurun_out/clock_samples.txt
    timeout -k 5 15 rocm-smi --showpower --showclocks >> gpurun_out/clock_samples.txt 2>&1
    sleep 4
  done
  wait $pid || exit 1
done
grep -E "==|sclk|Power|fclk|mclk" gpurun_out/clock_samples.txt | head -80
grep mean gpurun_out/clock_step_*.txt
