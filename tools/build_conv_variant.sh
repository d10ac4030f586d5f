#!/bin/bash
# A/B build of libvdiff.so with extra flags for conv.hip only -> vdiff/libvdiff_NAME.so
set -e
cd "$(dirname "$0")/../lipreading-video-generation_amd/csrc"
make -s -j8 >/dev/null
NAME=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function \
  -munsafe-fp-atomics -I../../include $@ -c conv.hip -o build/conv_$NAME.o
OBJS=$(ls build/*.o | grep -v -e "/conv" -e "/attention_")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../vdiff/libvdiff_$NAME.so $OBJS build/conv_$NAME.o
echo ../vdiff/libvdiff_$NAME.so
