#!/bin/bash
# conv GPU tests, then the 1x1 conv bench with the streaming kernel off / on (interleaved).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_conv.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_conv.log | head -20; exit $rc; }
for r in 1 2; do for pw in 0 1; do
  VDIFF_CONV_PW=$pw timeout -k 10 120 python -u tools/conv1x1_bench.py || exit 1
done; done > gpurun_out/ab_conv1x1.txt 2>&1; rc=$?
cat gpurun_out/ab_conv1x1.txt; exit $rc
