#!/bin/bash
# conv kernels: GPU parity tests, then the train-step bench with the tap-outer bf16 kernel and
# with the legacy kernel (VDIFF_CONV_LEGACY=1); per-shape conv times go to the .err logs
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/conv_t.log 2>&1 || { tail -30 gpurun_out/conv_t.log; exit 1; }
timeout -k 10 300 python bench.py --only train --no-cpu > gpurun_out/conv_new.json 2> gpurun_out/conv_new.err
VDIFF_CONV_LEGACY=1 timeout -k 10 300 python bench.py --only train --no-cpu > gpurun_out/conv_old.json 2> gpurun_out/conv_old.err
