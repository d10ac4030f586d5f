#!/bin/bash
# Round-3 GPU check: the new / changed tests with their printed metrics (-s), then the whole
# GPU suite.  Usage (GPU box): bash tools/gpu_r03.sh [tag]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-r03}
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_trajectory.py tests/test_gpu_bench_spawn.py tests/test_gpu_ddim_graph.py \
  tests/test_gpu_data.py "tests/test_gpu_fullsize.py::test_attention_full_length" \
  > gpurun_out/${TAG}_new_tests.log 2>&1
rc=$?
grep -E "TRAJ|FULLSIZE|passed|failed|Error" gpurun_out/${TAG}_new_tests.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gpu_tests.log
