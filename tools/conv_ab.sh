#!/bin/bash
# A/B of conv.hip variants (tools/build_conv_variant.sh NAME ...): train bench per library.
#   tools/conv_ab.sh NAME... ("" = the default build, "reg" = VDIFF_CONV_DMA=0)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$PWD/lipreading-video-generation_amd/vdiff
for v in "$@"; do
  if [ "$v" = reg ]; then
    VDIFF_CONV_DMA=0 timeout -k 10 300 python bench.py --only train --no-cpu > gpurun_out/cab_reg.json 2> gpurun_out/cab_reg.err
  else
    lib=$L/libvdiff.so; [ -n "$v" ] && lib=$L/libvdiff_$v.so
    VDIFF_LIB=$lib timeout -k 10 300 python bench.py --only train --no-cpu > gpurun_out/cab_$v.json 2> gpurun_out/cab_$v.err
  fi
done
