#!/bin/bash
# D=64 backward: 8-wave single-block pipelined kernels (p8, default) vs 4 waves x 2 blocks
# (p4n2), after the attention GPU tests.  GPU box: bash tools/ab_p4n2.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_attention.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_attn.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pytest_attn.log | head; exit $rc; }
bash tools/attn_ab.sh libvdiff "auto p4n2 auto p4n2" 64 > gpurun_out/ab_p4n2.txt 2>&1; rc=$?
grep -E "==|d= 64" gpurun_out/ab_p4n2.txt; exit $rc
