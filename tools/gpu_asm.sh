#!/bin/bash
# Hand-scheduled attention kernels on the GPU box: parity tests first, then per-launch A/B
# timing against the compiler-scheduled kernels.  Usage: bash tools/gpu_asm.sh TAG "cfgs"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-asm}; CFGS=${2:-"p8 asm"}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_attention_asm.py > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|passed|failed|Error|error" gpurun_out/${TAG}_tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
for cfg in $CFGS; do
  echo "== cfg=$cfg"
  VDIFF_ATTN_CFG=$cfg timeout -k 10 150 python -u tools/attn_bench.py --nocheck 3 --only 64 \
    2>&1 | tee -a gpurun_out/${TAG}_bench.log | grep -E "attn_fwd|attn_bwd_dq|attn_bwd_dkdv"
done
