cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_attn.log; [ $rc -eq 0 ] || exit $rc
bash tools/attn_ab.sh "libvdiff_u0 libvdiff libvdiff_u0 libvdiff" auto 64 > gpurun_out/ab_unroll.txt 2>&1; rc=$?
grep -E "==|d=64|fwd|dq|dkdv" gpurun_out/ab_unroll.txt | head -60; exit $rc
