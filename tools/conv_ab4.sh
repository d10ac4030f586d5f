#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$PWD/lipreading-video-generation_amd/vdiff
for v in "" s2; do
  lib=$L/libvdiff.so; [ -n "$v" ] && lib=$L/libvdiff_$v.so
  VDIFF_LIB=$lib timeout -k 10 300 python bench.py --only train --no-cpu > gpurun_out/cab4_$v.json 2> gpurun_out/cab4_$v.err
done
VDIFF_CONV_DMA=0 timeout -k 10 300 python bench.py --only train --no-cpu > gpurun_out/cab4_reg.json 2> gpurun_out/cab4_reg.err
