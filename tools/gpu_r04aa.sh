#!/bin/bash
# Round-4 GPU batch aa: the round-4 weight-gradient launch-choice tests.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_conv.py -k "round4 or config2" > gpurun_out/r04aa_wgrad_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/r04aa_wgrad_tests.log | tail -15; exit $rc
