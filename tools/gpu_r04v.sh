#!/bin/bash
# Round-4 GPU batch v: kw-strip weight-gradient ring depth / tile width / minimum steps per
# split (VDIFF_WGRAD3=nst,cot,msteps) under the occupancy-round split rule.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04v}
for v in 2,64,32 3,64,32 2,128,32 3,128,32 2,64,16 2,64,64 2,64,32; do
  VDIFF_WGRAD3=$v timeout -k 10 120 python3 -u tools/wgrad_ab.py > gpurun_out/${T}_w3_$v.log 2>&1
  rc=$?; echo "VDIFF_WGRAD3=$v: $(grep 'per train' gpurun_out/${T}_w3_$v.log)"
  [ $rc -eq 0 ] || { echo "rc=$rc: stopping"; tail -5 gpurun_out/${T}_w3_$v.log; exit $rc; }
  (echo "== VDIFF_WGRAD3=$v"; cat gpurun_out/${T}_w3_$v.log) >> gpurun_out/${T}_all.log
done
