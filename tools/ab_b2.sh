#!/bin/bash
# Deferred forward with one barrier per two tiles (VD_DEFER_B2 build) vs the default build:
# correctness (long ragged ring, lagged-max rescale, default shapes) then per-kernel times.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V=lipreading-video-generation_amd/vdiff
VDIFF_LIB=$V/libvdiff_b2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -k "auto or d8n or lagged or long_sequence" > gpurun_out/pytest_b2.log 2>&1; rc=$?
echo "b2: $(tail -1 gpurun_out/pytest_b2.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_b2.log | head; exit $rc; }
bash tools/attn_ab.sh "libvdiff libvdiff_b2 libvdiff libvdiff_b2" "auto" 64 > gpurun_out/ab_b2.txt 2>&1 || exit 1
grep -E "==|d= 64" gpurun_out/ab_b2.txt
