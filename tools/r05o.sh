#!/bin/bash
# Round-5 batch o: the tap-shifted weight gradient -- conv tests (incl. the bit-identity test
# against VDIFF_WGRAD_SHIFT=0), then the per-shape A/B, interleaved, two passes each.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05o
timeout -k 10 800 python3 -u -m pytest -q --timeout 400 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_conv.py > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.log
case $rc in 0) ;; *) echo "pytest rc=$rc: stopping"; grep -E "Error|assert|FAIL" gpurun_out/${T}_tests.log | head; exit $rc;; esac
for sh in 0 1 0 1; do
  echo "== VDIFF_WGRAD_SHIFT=$sh" >> gpurun_out/${T}_ab.txt
  VDIFF_WGRAD_SHIFT=$sh timeout -k 10 300 python3 -u tools/wgrad_ab.py >> gpurun_out/${T}_ab.txt 2>&1 \
    || { echo "ab rc=$?"; tail -5 gpurun_out/${T}_ab.txt; exit 1; }
done
grep -E "^==|per train step" gpurun_out/${T}_ab.txt
