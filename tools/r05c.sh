#!/bin/bash
# Round-5 batch c: the bf16 five-step parity test (with its autocast-bf16 oracle peer), then
# the pure-HIP graph reproducer (tools/graph_memset_repro.hip): semaphore reset by
# hipMemsetAsync or by a kernel, host work between replays 0 / 1 / 2, HIP graph packet
# capture on (default) / off.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05c
VDIFF_TEST_METRICS=gpurun_out/${T}_metrics.jsonl timeout -k 10 600 python3 -u -m pytest -v \
  --timeout 400 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_modules.py::test_trainer_five_steps_bf16_match_reference" \
  > gpurun_out/${T}_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed|autocast" gpurun_out/${T}_tests.log | tail -6
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
for reset in 0 1; do for hw in 0 1 2; do
  timeout -k 10 120 tools/graph_memset_repro.bin 1000 $hw $reset >> gpurun_out/${T}_hiprepro.txt 2>&1 \
    || { echo "repro rc=$?"; tail -3 gpurun_out/${T}_hiprepro.txt; exit 1; }
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 120 tools/graph_memset_repro.bin 1000 $hw $reset \
    >> gpurun_out/${T}_hiprepro.txt 2>&1 || { echo "repro rc=$?"; tail -3 gpurun_out/${T}_hiprepro.txt; exit 1; }
done; done
cat gpurun_out/${T}_hiprepro.txt
