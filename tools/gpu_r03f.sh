#!/bin/bash
# Round-3 GPU batch f: 3x3x3 weight-gradient variants (VDIFF_WGRAD3), cycle attribution of
# the head_dim-64 forward body (in-kernel stamps with one instruction class dropped at a time,
# rare path off so every variant runs the same bodies), train.py --data vs synthetic.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03f}
ok() { case $1 in 0|1) return 0 ;; *) echo "stopping: rc $1"; exit $1 ;; esac; }
for v in 2,64 3,64 2,128 3,128 2,64; do
  VDIFF_WGRAD3=$v timeout -k 10 200 python -u tools/wgrad3_bench.py \
    >> gpurun_out/${T}_wgrad3.txt 2>&1; rc=$?; ok $rc
  grep "per train step" gpurun_out/${T}_wgrad3.txt | tail -1
done
timeout -k 10 300 python -u tools/asm_ab.py 'nr:NORARE=1,STAMP=1' \
  'nr_dexp:NORARE=1,STAMP=1,DROP=1' 'nr_dadd:NORARE=1,STAMP=1,DROP=2' \
  'nr_dcvt:NORARE=1,STAMP=1,DROP=4' 'nr_dread:NORARE=1,STAMP=1,DROP=8' \
  'nr_ddma:NORARE=1,STAMP=1,DROP=16' 'nr_c4:NORARE=1,STAMP=1,CHAINS=4' 'nr2:NORARE=1,STAMP=1' \
  > gpurun_out/${T}_fwd_cycles.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/${T}_fwd_cycles.txt | tail -9; ok $rc
timeout -k 10 700 python -u tools/data_vs_synth.py > gpurun_out/${T}_data_vs_synth.json \
  2> gpurun_out/${T}_data_vs_synth.err; rc=$?
tail -c 500 gpurun_out/${T}_data_vs_synth.json; tail -3 gpurun_out/${T}_data_vs_synth.err; ok $rc
