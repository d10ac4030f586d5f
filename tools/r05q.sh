#!/bin/bash
# Round-5 batch q: short-sequence forward with 1 / 2 / 4 sequences per wave (prefetch), A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -q --timeout 200 -p no:cacheprovider tests/test_gpu_attention_short.py \
  > gpurun_out/r05q_tests.txt 2>&1 || { tail -20 gpurun_out/r05q_tests.txt; exit 1; }
tail -1 gpurun_out/r05q_tests.txt
for spw in 1 2 4; do
  echo "== SPW $spw" >> gpurun_out/r05q_ab.txt
  VDIFF_SHORT_SPW=$spw timeout -k 10 200 python3 -u tools/attn_bench.py 20 --temporal --nocheck \
    >> gpurun_out/r05q_ab.txt 2>&1 || { echo "rc=$?"; tail -3 gpurun_out/r05q_ab.txt; exit 1; }
done
grep -E "^==|attn_fwd" gpurun_out/r05q_ab.txt
