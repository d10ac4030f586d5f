#!/bin/bash
# Round-4 GPU batch aj: code placement of the hand-scheduled attention kernels -- every asm
# kernel shifted by 4 bytes (libvdiff_ph1.so, tools/build_asm_phase.sh) against the product
# library, interleaved, all head dims (tools/attn_bench.py, 3 reps per launch kind).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lib in libvdiff libvdiff_ph1 libvdiff libvdiff_ph1; do
  echo "== $lib"
  VDIFF_LIB=lipreading-video-generation_amd/vdiff/$lib.so timeout -k 10 200 \
    python3 -u tools/attn_bench.py 3 2>&1 | grep -v amdgpu.ids
  rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || { echo "rc=$rc: stopping"; exit $rc; }
done
