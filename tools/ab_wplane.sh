#!/bin/bash
# Nine-tap-plane conv weight gradient (VDIFF_CONV_WPLANE=1) vs the kw-strip kernel: conv GPU
# tests on the plane path, then per-shape conv times of the train step with and without it.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
VDIFF_CONV_WPLANE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_wplane.log 2>&1; rc=$?
echo "wplane tests: $(tail -1 gpurun_out/pytest_wplane.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_wplane.log | head -20; exit $rc; }
for v in 0 1; do
  VDIFF_CONV_WPLANE=$v timeout -k 10 300 python tools/conv_breakdown.py > gpurun_out/cbd_wp$v.txt 2>&1 || exit 1
done
grep -E "bwd_weight.*k3x3x3" gpurun_out/cbd_wp0.txt | head -12; echo; grep -E "bwd_weight.*k3x3x3" gpurun_out/cbd_wp1.txt | head -12
