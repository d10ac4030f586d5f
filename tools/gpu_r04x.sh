#!/bin/bash
# Round-4 GPU batch x: weight-gradient knobs under the occupancy-round split rule: 1x1 ring /
# tile width (VDIFF_WGRAD1=nst,cot), kw-strip minimum steps per split (VDIFF_WGRAD3=2,0,m),
# the XCD-aware grid (VDIFF_WGRAD_XCD=0).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04x}
run() {  # name, env assignment
  env $2 timeout -k 10 120 python3 -u tools/wgrad_ab.py > gpurun_out/${T}_$1.log 2>&1
  rc=$?; echo "$1 ($2): $(grep 'per train' gpurun_out/${T}_$1.log)"
  [ $rc -eq 0 ] || { echo "rc=$rc: stopping"; tail -5 gpurun_out/${T}_$1.log; exit $rc; }
  (echo "== $1 $2"; cat gpurun_out/${T}_$1.log) >> gpurun_out/${T}_all.log
}
run base VDIFF_X=0
run w1_2_128 VDIFF_WGRAD1=2,128
run w1_4_64 VDIFF_WGRAD1=4,64
run w1_6_64 VDIFF_WGRAD1=6,64
run w1_4_192 VDIFF_WGRAD1=4,192
run w1_2_192 VDIFF_WGRAD1=2,192
run w3_m16 VDIFF_WGRAD3=2,0,16
run w3_m24 VDIFF_WGRAD3=2,0,24
run w3_m48 VDIFF_WGRAD3=2,0,48
run xcd0 VDIFF_WGRAD_XCD=0
run base2 VDIFF_X=0
