#!/bin/bash
# Round-3 GPU batch j: 3x3x3 weight-gradient variants with the pixels-per-split knob
# (VDIFF_WGRAD3=nst,cot,steps), alternating with the default.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03j}
for v in 2,64,32 2,64,16 2,128,16 2,128,8 3,128,16 2,64,32 2,64,24 2,128,24; do
  VDIFF_WGRAD3=$v timeout -k 10 200 python -u tools/wgrad3_bench.py \
    >> gpurun_out/${T}_wgrad3.txt 2>&1; rc=$?
  grep "per train step" gpurun_out/${T}_wgrad3.txt | tail -1
  case $rc in 0|1) ;; *) exit $rc ;; esac
done
timeout -k 10 300 python -u tools/gn_bench.py > gpurun_out/${T}_gn.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/${T}_gn.txt | tail -10
exit $rc
