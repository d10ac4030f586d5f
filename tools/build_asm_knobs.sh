#!/bin/bash
# Build an A/B variant of libvdiff.so whose hand-scheduled attention kernels are generated with other knob values
# (gen_attn_asm.py --knob=module.NAME=value):
#   tools/build_asm_knobs.sh NAME gen_fwd.CHAINS=4 ...  ->  vdiff/libvdiff_NAME.so
# Run it with VDIFF_LIB=<that path>.  Experiments only; the product build is make.
set -e
cd "$(dirname "$0")/../lipreading-video-generation_amd/csrc"
make -s -j8 >/dev/null
NAME=$1; shift; KN=""; for k in "$@"; do KN="$KN --knob=$k"; done
T=$(mktemp -d)
mkdir -p $T/build
python3 asm/gen_attn_asm.py $T/attn_asm.s $KN
/opt/rocm/llvm/bin/clang -x assembler -target amdgcn-amd-amdhsa -mcpu=gfx950 -c $T/attn_asm.s -o $T/attn_asm.co.o
/opt/rocm/llvm/bin/ld.lld -shared $T/attn_asm.co.o -o $T/attn_asm.hsaco
python3 asm/blob.py $T/attn_asm.hsaco $T/build/attn_asm_blob.inc vd_attn_asm_hsaco
cp asm_kernels.cpp $T/
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function \
  -munsafe-fp-atomics -I../../include -I. -x hip -c $T/asm_kernels.cpp -o build/asm_kernels_$NAME.o
OBJS=$(ls build/*.o | grep -v -e "asm_kernels" -e "attention_" -e "/conv_" -e "attn_asm")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../vdiff/libvdiff_$NAME.so $OBJS build/asm_kernels_$NAME.o
rm -rf $T
echo ../vdiff/libvdiff_$NAME.so
