#!/bin/bash
# Halo conv with 32-channel steps (64-B LDS rows, 40 KiB, four workgroups per CU;
# VDIFF_CONV_HALO_KS=32) vs 64-channel steps: conv tests on the KS=32 path (every eligible
# shape), then per-shape conv times with the halo forced on for every eligible shape.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
VDIFF_CONV_HALO=1 VDIFF_CONV_HALO_KS=32 timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_halo32.log 2>&1; rc=$?
echo "halo ks32 tests: $(tail -1 gpurun_out/pytest_halo32.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_halo32.log | head -20; exit $rc; }
VDIFF_CONV_HALO=0 timeout -k 10 300 python tools/conv_breakdown.py > gpurun_out/cbd_k0.txt 2>&1 || exit 1
VDIFF_CONV_HALO=1 timeout -k 10 300 python tools/conv_breakdown.py > gpurun_out/cbd_k64.txt 2>&1 || exit 1
VDIFF_CONV_HALO=1 VDIFF_CONV_HALO_KS=32 timeout -k 10 300 python tools/conv_breakdown.py > gpurun_out/cbd_k32.txt 2>&1 || exit 1
echo ok
