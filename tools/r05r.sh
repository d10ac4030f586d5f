#!/bin/bash
# Round-5 batch r: short-sequence backward with dQ / dK / dV staged through LDS (whole-row
# stores); short + flash attention tests, then the temporal kernel timings.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -q --timeout 200 -p no:cacheprovider \
  tests/test_gpu_attention_short.py tests/test_gpu_attention.py \
  > gpurun_out/r05r_tests.txt 2>&1 || { tail -20 gpurun_out/r05r_tests.txt; exit 1; }
tail -1 gpurun_out/r05r_tests.txt
timeout -k 10 200 python3 -u tools/attn_bench.py 20 --temporal --nocheck \
  > gpurun_out/r05r_temporal.txt 2>&1 || { echo "rc=$?"; tail -3 gpurun_out/r05r_temporal.txt; exit 1; }
cat gpurun_out/r05r_temporal.txt
