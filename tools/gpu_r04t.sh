#!/bin/bash
# Round-4 GPU batch t: the K-split-wave weight-gradient kernel (wgrad_ks_body, VDIFF_WGRAD_KS=1)
# at two workgroups per CU (launch bounds 2: 254 VGPRs, no spills at COT = 64) against the
# default kw-strip kernel, both checked against the fp32 parity-mode kernel.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04t}
for ks in 1 0 1; do
  VDIFF_WGRAD_KS=$ks timeout -k 10 120 python3 -u tools/wgrad_ab.py > gpurun_out/${T}_ks$ks.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/${T}_ks$ks.log | grep -E "k3|per train"
  [ $rc -eq 0 ] || { echo "rc=$rc: stopping"; tail -5 gpurun_out/${T}_ks$ks.log; exit $rc; }
done
