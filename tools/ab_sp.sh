#!/bin/bash
# Fragment-pipelined D=64 backward (cfg sp) vs the default pipelines: correctness of every
# built variant on the long ragged ring, then per-kernel times.  GPU box: bash tools/ab_sp.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V=lipreading-video-generation_amd/vdiff
for lib in libvdiff ${SP_LIBS:-libvdiff_sp41 libvdiff_sp42}; do
  VDIFF_LIB=$V/$lib.so timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -k "sp and (long_ragged or kernel_shapes or lagged)" \
    > gpurun_out/pytest_sp_$lib.log 2>&1; rc=$?
  echo "$lib: $(tail -1 gpurun_out/pytest_sp_$lib.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_sp_$lib.log | head; exit $rc; }
done
bash tools/attn_ab.sh "libvdiff" "auto sp" 64 > gpurun_out/ab_sp.txt 2>&1 || exit 1
bash tools/attn_ab.sh "${SP_LIBS:-libvdiff_sp41 libvdiff_sp42}" "sp" 64 >> gpurun_out/ab_sp.txt 2>&1
grep -E "==|d= 64" gpurun_out/ab_sp.txt
