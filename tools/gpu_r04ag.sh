#!/bin/bash
# Round-4 GPU batch ag: GroupNorm rows in flight per thread (VDIFF_GN_UNROLL 1 / 2 / 4), GPU time
# of the C-ABI calls, then the GN tests under each setting.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04ag}
for u in 1 2 4 1 2 4; do
  VDIFF_GN_UNROLL=$u timeout -k 10 120 python3 -u tools/gn_bench.py --capi > gpurun_out/${T}_u$u.log 2>&1
  rc=$?; echo "== unroll $u"; grep -v amdgpu.ids gpurun_out/${T}_u$u.log
  [ $rc -eq 0 ] || { echo "rc=$rc: stopping"; exit $rc; }
done
for u in 2 4; do
  VDIFF_GN_UNROLL=$u timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider tests/test_gpu_groupnorm.py > gpurun_out/${T}_tests_u$u.log 2>&1
  rc=$?; echo "tests unroll $u: $(tail -1 gpurun_out/${T}_tests_u$u.log)"; [ $rc -eq 0 ] || exit $rc
done
