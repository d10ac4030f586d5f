#!/bin/bash
# Round-4 GPU batch u: the occupancy-round split rule for the weight gradients
# (VDIFF_WGRAD_QRULE=c, applied where the default rule gives <= c splits) against the default.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04u}
for q in 0 32 64 256 0 32 64 256; do
  VDIFF_WGRAD_QRULE=$q timeout -k 10 120 python3 -u tools/wgrad_ab.py > gpurun_out/${T}_q$q.log 2>&1
  rc=$?; echo "qrule $q: $(grep 'per train' gpurun_out/${T}_q$q.log)"
  [ $rc -eq 0 ] || { echo "rc=$rc: stopping"; tail -5 gpurun_out/${T}_q$q.log; exit $rc; }
  cat gpurun_out/${T}_q$q.log >> gpurun_out/${T}_all.log
done
