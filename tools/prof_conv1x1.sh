#!/bin/bash
# Kernel durations of tools/conv1x1_bench.py under rocprofv3, streaming 1x1 kernel off / on.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for pw in 0 1; do
  rm -rf /tmp/prof_pw$pw
  VDIFF_CONV_PW=$pw timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/prof_pw$pw -o run -- \
    python -u tools/conv1x1_bench.py > gpurun_out/pw$pw.log 2>&1 || { tail gpurun_out/pw$pw.log; exit 1; }
  db=$(find /tmp/prof_pw$pw -name '*.db' | head -n 1)
  echo "== VDIFF_CONV_PW=$pw"
  python tools/prof_dispatch.py "$db" gemm
done > gpurun_out/prof_conv1x1.md
cat gpurun_out/prof_conv1x1.md
