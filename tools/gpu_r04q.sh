#!/bin/bash
# Round-4 GPU batch q: weight-gradient pixel-split counts (VDIFF_WGRAD_SPLITS, diagnostic
# override; 0 = the default rule) over every conv shape of the train step (tools/wgrad_ab.py).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04q}
for s in 0 3 4 5 6 7 8 10 12 14 16 20 24 32 48; do
  VDIFF_WGRAD_SPLITS=$s timeout -k 10 120 python3 -u tools/wgrad_ab.py > gpurun_out/${T}_splits$s.log 2>&1
  rc=$?; grep "per train" gpurun_out/${T}_splits$s.log
  [ $rc -eq 0 ] || { echo "rc=$rc at s=$s: stopping"; tail -5 gpurun_out/${T}_splits$s.log; exit $rc; }
done
