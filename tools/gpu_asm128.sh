#!/bin/bash
# Hand-scheduled head_dim-128 dK/dV (asm/gen_d128.py) on the GPU box: parity tests, then
# per-launch A/B timing against the paired default.  Usage: bash tools/gpu_asm128.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-asm128}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_attention_asm128.py > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|passed|failed|Error|error|assert" gpurun_out/${TAG}_tests.log | tail -20
# a fault, abort or time limit ends the call; an ordinary test failure does not
case $rc in 0|1) ;; *) exit $rc ;; esac
for cfg in pair asm pair asm; do
  echo "== cfg=$cfg"
  VDIFF_ATTN_CFG=$cfg timeout -k 10 150 python -u tools/attn_bench.py --nocheck 3 --only 128 \
    2>&1 | tee -a gpurun_out/${TAG}_bench.log | grep -E "attn_fwd|attn_bwd_dq|attn_bwd_dkdv" || exit 1
done
exit $rc
