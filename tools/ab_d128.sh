#!/bin/bash
# D=128 dK/dV: parity of the paired kernel, then base vs pair timing (same box).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_attn.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_attn.log; [ $rc -eq 0 ] || exit $rc
VDIFF_ATTN_CFG=pair timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -q \
  -k "attention and 128" --timeout 120 --timeout-method thread > gpurun_out/pytest_fs.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_fs.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for cfg in base pair; do
  echo "== d128 cfg=$cfg"
  VDIFF_ATTN_CFG=$cfg timeout -k 10 150 python -u tools/attn_bench.py --nocheck 5 --only 128 | grep dkdv || exit 1
done
done
