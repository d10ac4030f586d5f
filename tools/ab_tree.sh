#!/bin/bash
# Deferred forward with pairwise row sums (VD_DEFER_TREE build) vs the sequential chain;
# also the head_dim-128 forward shapes (d8n default vs nb2) on the default build.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V=lipreading-video-generation_amd/vdiff
VDIFF_LIB=$V/libvdiff_tree.so timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -k "auto or d8n or lagged or long" > gpurun_out/pytest_tree.log 2>&1; rc=$?
echo "tree: $(tail -1 gpurun_out/pytest_tree.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_tree.log | head; exit $rc; }
for D in 64 128; do
  bash tools/attn_ab.sh "libvdiff libvdiff_tree libvdiff libvdiff_tree" "auto" $D > gpurun_out/ab_tree_$D.txt 2>&1 || exit 1
  grep -E "==|attn_fwd" gpurun_out/ab_tree_$D.txt
done
bash tools/attn_ab.sh "libvdiff" "nb2 auto nb2" 128 > gpurun_out/ab_nb2_128.txt 2>&1 || exit 1
grep -E "==|attn_fwd" gpurun_out/ab_nb2_128.txt
