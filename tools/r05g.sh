#!/bin/bash
# Round-5 batch g: vd_mse_loss (kernel tests), the graph-replayed train step returning its
# in-graph loss (no memset nodes), the ViViT graph step vs eager, the bf16 five-step pin,
# then the torch-only reproducer with the semaphore probe.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05g
VDIFF_TEST_METRICS=gpurun_out/${T}_metrics.jsonl timeout -k 10 900 python3 -u -m pytest -v \
  --timeout 400 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_elementwise.py::test_mse_loss tests/test_gpu_elementwise.py::test_mse_loss_mixed_dtype_and_layout \
  tests/test_gpu_train_graph.py tests/test_vivit.py \
  tests/test_gpu_modules.py::test_trainer_five_steps_bf16_match_reference \
  tests/test_gpu_modules.py::test_trainer_five_steps_match_reference \
  > gpurun_out/${T}_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed" gpurun_out/${T}_tests.log | tail -40
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 200 python3 -u tools/graph_reduce_repro.py --check-grads --host-ops 3 --probe-sem \
  > gpurun_out/${T}_repro.txt 2>&1 || { echo "repro rc=$?"; tail -5 gpurun_out/${T}_repro.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_repro.txt | cut -c1-3000
