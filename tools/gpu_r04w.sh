#!/bin/bash
# Round-4 GPU batch w: kw-strip tile width chosen per shape (cot 0 = auto) against fixed 64 /
# 128, then the conv GPU tests under the new defaults (split rule + tile width).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04w}
for v in 2,0,32 2,64,32 2,128,32 2,0,32; do
  VDIFF_WGRAD3=$v timeout -k 10 120 python3 -u tools/wgrad_ab.py > gpurun_out/${T}_w3_$v.log 2>&1
  rc=$?; echo "VDIFF_WGRAD3=$v: $(grep 'per train' gpurun_out/${T}_w3_$v.log)"
  [ $rc -eq 0 ] || { echo "rc=$rc: stopping"; tail -5 gpurun_out/${T}_w3_$v.log; exit $rc; }
  (echo "== VDIFF_WGRAD3=$v"; cat gpurun_out/${T}_w3_$v.log) >> gpurun_out/${T}_all.log
done
timeout -k 10 400 python3 -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_conv.py tests/test_gpu_modules.py > gpurun_out/${T}_conv_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_conv_tests.log; exit $rc
