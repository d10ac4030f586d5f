#!/bin/bash
# conv GPU tests, then tools/conv_breakdown.py under env settings, interleaved:
#   bash tools/ab_conv_env.sh "VDIFF_CONV_N64=0 VDIFF_CONV_N64=1"   (libs: $LIBS, default libvdiff)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_modules.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_conv.log; [ $rc -eq 0 ] || { grep -E "^E|FAIL" gpurun_out/pytest_conv.log | head; exit $rc; }
for r in 1 2; do for lib in ${LIBS:-libvdiff}; do for e in $1; do
  echo "== $lib $e"
  env $e VDIFF_LIB=lipreading-video-generation_amd/vdiff/$lib.so timeout -k 10 200 python -u tools/conv_breakdown.py 2>&1 | cat || exit 1
done; done; done > gpurun_out/ab_conv_env.txt
grep -E "==|conv total" gpurun_out/ab_conv_env.txt
