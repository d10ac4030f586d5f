#!/bin/bash
# Round-4 GPU batch a: the whole -m gpu suite WITHOUT -x (every failure, not the first),
# then round 3's already-written localisation batch (full-size DDIM graph vs eager; graph-
# replayed train step without dropout at config 2 and with dropout at 64x64).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04a}
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?
tail -15 gpurun_out/${T}_gpu_tests.log
grep -E "FAILED|ERROR" gpurun_out/${T}_gpu_tests.log | head -30
# 124/137 = time limit, 134/139 = abort/segv: stop here
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
bash tools/gpu_r03t.sh ${T}t
