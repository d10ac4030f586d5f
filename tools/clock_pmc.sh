#!/bin/bash
# Effective clock of the train step's kernels with the weights at the benchmark init
# (lr 0) and after Adam updates (lr 1e-2): one GRBM_GUI_ACTIVE pass each (GPU box).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lr in 0 1e-2; do
  rm -rf /tmp/clk_$lr
  timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
    -d /tmp/clk_$lr -o clk -- python tools/step_gap.py --rounds 2 --steps 2 --lr $lr \
    > gpurun_out/clock_pmc_run_$lr.txt 2>&1 || { tail gpurun_out/clock_pmc_run_$lr.txt; exit 1; }
  echo "== lr $lr" | tee -a gpurun_out/clock_pmc.txt
  grep "mean period" gpurun_out/clock_pmc_run_$lr.txt | tee -a gpurun_out/clock_pmc.txt
  python tools/clock_pmc.py /tmp/clk_$lr | tee -a gpurun_out/clock_pmc.txt
done
