#!/bin/bash
# conv GPU tests, then tools/conv_breakdown.py per library, interleaved:  bash tools/ab_conv_lib.sh "libvdiff libvdiff_x"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_conv.log; [ $rc -eq 0 ] || { grep -E "^E|FAIL" gpurun_out/pytest_conv.log | head; exit $rc; }
for r in 1 2; do for lib in $1; do
  echo "== $lib"
  VDIFF_LIB=lipreading-video-generation_amd/vdiff/$lib.so timeout -k 10 200 python -u tools/conv_breakdown.py 2>&1 | head -12 || exit 1
done; done > gpurun_out/ab_conv_lib.txt
grep -E "==|conv total" gpurun_out/ab_conv_lib.txt
