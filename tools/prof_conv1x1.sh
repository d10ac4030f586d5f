#!/bin/bash
# Kernel durations of tools/conv1x1_bench.py under rocprofv3 for each VDIFF_PW_AB value given
# (default: 0), per (kernel, grid, LDS) shape.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for ab in ${@:-0}; do
  rm -rf /tmp/prof_pw$ab
  VDIFF_PW_AB=$ab timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/prof_pw$ab -o run -- \
    python -u tools/conv1x1_bench.py > gpurun_out/pw$ab.log 2>&1 || { tail gpurun_out/pw$ab.log; exit 1; }
  db=$(find /tmp/prof_pw$ab -name '*.db' | head -n 1)
  echo "== VDIFF_PW_AB=$ab"
  python tools/prof_dispatch.py "$db" gemm
done > gpurun_out/prof_conv1x1.md
cat gpurun_out/prof_conv1x1.md
