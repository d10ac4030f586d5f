#!/bin/bash
# Round-3 GPU batch h: generator-knob A/B of the hand-scheduled forwards (tools/asm_ab.py):
# head_dim 64 (row-sum chains through the lagged list, LDS-DMA slots) and head_dim 128
# (chains, DMA slots, K-read gap, prefetch distance).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03h}
timeout -k 10 400 python -u tools/asm_ab.py base: lag1:LAG1=1 c2:CHAINS=2 dmas1:DMAS=1 \
  dmas2:DMAS=2 dmas3:DMAS=3 base2: lag1b:LAG1=1 c2b:CHAINS=2 base3: \
  > gpurun_out/${T}_fwd64_ab.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/${T}_fwd64_ab.txt | tail -11
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 400 python -u tools/asm_ab.py --d128 base: c1:CHAINS=1 c2:CHAINS=2 dmas1:DMAS=1 \
  dmas2:DMAS=2 ks4:KSLOT=4 pd3:PD=3 pd5:PD=5 base2: c2b:CHAINS=2 \
  > gpurun_out/${T}_fwd128_ab.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/${T}_fwd128_ab.txt | tail -11
exit $rc
