#!/bin/bash
# attention.hip built with -fno-slp-vectorize (no v_pk_add_f32 / v_pk_mul_f32 from SLP
# packing of the row sums and dS products) vs the default build: attention GPU tests on
# the variant, then per-kernel times at every head dim, alternating builds.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V=lipreading-video-generation_amd/vdiff
VDIFF_LIB=$V/libvdiff_noslp.so timeout -k 10 400 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_cross_attention.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_noslp.log 2>&1; rc=$?
echo "noslp: $(tail -1 gpurun_out/pytest_noslp.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_noslp.log | head; exit $rc; }
for D in 64 128 256; do
  bash tools/attn_ab.sh "libvdiff libvdiff_noslp libvdiff libvdiff_noslp" "auto" $D > gpurun_out/ab_noslp_$D.txt 2>&1 || exit 1
  grep -E "==|d=" gpurun_out/ab_noslp_$D.txt
done
