#!/bin/bash
# head_dim 256 dK/dV: role-split pairs (auto; 4 waves, or the 8-wave build) vs the
# output-column split (cfg base), after the attention GPU tests.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_attn.log; [ $rc -eq 0 ] || { grep -E "^E|FAIL" gpurun_out/pytest_attn.log | head -20; exit $rc; }
bash tools/attn_ab.sh "libvdiff libvdiff_role8" "auto base auto base" 256 > gpurun_out/ab_role.txt 2>&1; rc=$?
grep -E "==|d=256" gpurun_out/ab_role.txt; exit $rc
