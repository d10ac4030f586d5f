#!/bin/bash
# Round-5 batch b: re-run of batch a (tools/r05a.sh) after the bar changes:
# then the graph-reduction experiments (torch-only reproducer; the real-model probe with
# and without HIP's graph packet capture).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05b
VDIFF_TEST_METRICS=gpurun_out/${T}_metrics.jsonl timeout -k 10 900 python3 -u -m pytest -v \
  --timeout 400 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_fullsize.py::test_attention_full_length[config4-1638400-64]" \
  "tests/test_gpu_modules.py::test_trainer_five_steps_bf16_match_reference" \
  > gpurun_out/${T}_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed" gpurun_out/${T}_tests.log | tail -12
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
for v in "" "--quiet-host" "--impl twostage"; do
  timeout -k 10 120 python3 -u tools/graph_reduce_repro.py $v >> gpurun_out/${T}_repro.txt 2>&1 \
    || { echo "repro rc=$?"; tail -5 gpurun_out/${T}_repro.txt; exit 1; }
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 120 python3 -u tools/graph_reduce_repro.py $v \
    >> gpurun_out/${T}_repro.txt 2>&1 || { echo "repro rc=$?"; tail -5 gpurun_out/${T}_repro.txt; exit 1; }
done
grep impl gpurun_out/${T}_repro.txt
for pc in 1 0; do
  echo "# DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc" >> gpurun_out/${T}_probe.txt
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc timeout -k 10 300 python3 -u tools/graph_loss_probe.py \
    --twin --compare-weights --snap --steps 8 >> gpurun_out/${T}_probe.txt 2>&1 \
    || { echo "probe rc=$?"; tail -5 gpurun_out/${T}_probe.txt; exit 1; }
done
grep -E "^#|returned" gpurun_out/${T}_probe.txt | cut -c1-200
