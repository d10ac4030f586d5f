#!/bin/bash
# A/B of hand-scheduled forward variants (tools/asm_ab.py) on the GPU box.
#   bash tools/gpu_asm_ab.sh TAG 'name:K=v' ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 400 python -u tools/asm_ab.py "$@" > gpurun_out/ab_${TAG}.txt 2>&1
rc=$?
cat gpurun_out/ab_${TAG}.txt | tail -30
exit $rc
