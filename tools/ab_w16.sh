#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -x -q --timeout 120 \
  --timeout-method thread -k "w16 or pair or auto" > gpurun_out/pytest_attn.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_attn.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for cfg in auto w16; do
  echo "== d64 cfg=$cfg"
  VDIFF_ATTN_CFG=$cfg timeout -k 10 150 python -u tools/attn_bench.py --nocheck 3 --only 64 | grep -v dkdv || exit 1
done
done
