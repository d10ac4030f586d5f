#!/bin/bash
# Round-4 GPU batch af: conv bias / emb-add channel sums, stage-1 blocks per sample and loads in
# flight per thread (VDIFF_CSUM_BLOCKS, VDIFF_CSUM_UNROLL).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04af}
run() {
  env $2 timeout -k 10 120 python3 -u tools/csum_bench.py > gpurun_out/${T}_$1.log 2>&1
  rc=$?; echo "== $1 ($2)"; grep -v amdgpu.ids gpurun_out/${T}_$1.log
  [ $rc -eq 0 ] || { echo "rc=$rc: stopping"; exit $rc; }
}
run base VDIFF_X=0
run u4 VDIFF_CSUM_UNROLL=4
run b512 VDIFF_CSUM_BLOCKS=512
run b512u4 "VDIFF_CSUM_BLOCKS=512 VDIFF_CSUM_UNROLL=4"
run b1024u4 "VDIFF_CSUM_BLOCKS=1024 VDIFF_CSUM_UNROLL=4"
run b1024 VDIFF_CSUM_BLOCKS=1024
run base2 VDIFF_X=0
