#!/bin/bash
# Kernel durations of tools/conv1x1_bench.py under rocprofv3, per (kernel, grid, LDS) shape,
# for each library given (default: the product build), e.g.
#   bash tools/prof_conv1x1.sh libvdiff libvdiff_variant
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lib in ${@:-libvdiff}; do
  rm -rf /tmp/prof_pw_$lib
  VDIFF_LIB=lipreading-video-generation_amd/vdiff/$lib.so timeout -k 10 200 rocprofv3 --kernel-trace \
    -d /tmp/prof_pw_$lib -o run -- python -u tools/conv1x1_bench.py > gpurun_out/pw_$lib.log 2>&1 \
    || { tail gpurun_out/pw_$lib.log; exit 1; }
  db=$(find /tmp/prof_pw_$lib -name '*.db' | head -n 1)
  echo "== $lib"
  python tools/prof_dispatch.py "$db" gemm
done > gpurun_out/prof_conv1x1.md
cat gpurun_out/prof_conv1x1.md
