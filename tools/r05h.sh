#!/bin/bash
# Round-5 batch h: vd_mse_loss, the graph step's in-graph loss (no memset nodes), the ViViT
# graph vs eager, the short-sequence attention kernels, the existing attention suite (its
# bf16 temporal cases now take the short kernels), the bf16 five-step pin; then a short bench
# with the spatial_temporal leg.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05h
VDIFF_TEST_METRICS=gpurun_out/${T}_metrics.jsonl timeout -k 10 900 python3 -u -m pytest -v \
  --timeout 400 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_elementwise.py::test_mse_loss tests/test_gpu_elementwise.py::test_mse_loss_mixed_dtype_and_layout \
  tests/test_gpu_attention_short.py tests/test_gpu_attention.py \
  tests/test_gpu_train_graph.py tests/test_vivit.py \
  tests/test_gpu_modules.py::test_trainer_five_steps_bf16_match_reference \
  tests/test_gpu_modules.py::test_trainer_five_steps_match_reference \
  > gpurun_out/${T}_tests.log 2>&1
rc=$?; grep -E "FAIL|passed|failed" gpurun_out/${T}_tests.log | tail -30
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 600 python3 -u bench.py --steps 5 --warmup 2 --c4-steps 1 --vivit-steps 5 --no-cpu \
  > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
grep -E "spatial_temporal|temporal|train:" gpurun_out/${T}_bench.err | cut -c1-400
timeout -k 10 200 python3 -u tools/graph_reduce_repro.py --check-grads --host-ops 3 --probe-sem \
  > gpurun_out/${T}_repro_sem.txt 2>&1 || { echo "repro rc=$?"; tail -5 gpurun_out/${T}_repro_sem.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_repro_sem.txt | cut -c1-2500
