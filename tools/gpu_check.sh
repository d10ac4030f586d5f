#!/bin/bash
# GPU test suite + a short bench line.  Usage (GPU box): bash tools/gpu_check.sh [pytest -k expr]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
K=${1:-}
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
VDIFF_TEST_METRICS=gpurun_out/test_metrics.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  "${KARG[@]}" > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "FAIL|Error|error" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --c4-steps 1 --vivit-steps 5 \
    > gpurun_out/bench_short.json 2> gpurun_out/bench_short.err
  rc=$?
  tail -c 3000 gpurun_out/bench_short.json
  exit $rc
fi
