#!/bin/bash
# Deferred forward with the softmax of the first block interleaved into the next block's
# MFMAs (VD_DEFER_IGLP=NV builds) vs the default build.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V=lipreading-video-generation_amd/vdiff
VDIFF_LIB=$V/libvdiff_ig5.so timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -k "auto or d8n or lagged or long" > gpurun_out/pytest_ig.log 2>&1; rc=$?
echo "ig5: $(tail -1 gpurun_out/pytest_ig.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_ig.log | head; exit $rc; }
bash tools/attn_ab.sh "libvdiff libvdiff_ig4 libvdiff_ig5 libvdiff_ig6 libvdiff libvdiff_ig4 libvdiff_ig5 libvdiff_ig6" "auto" 64 > gpurun_out/ab_ig.txt 2>&1 || exit 1
grep -E "==|attn_fwd" gpurun_out/ab_ig.txt
