#!/bin/bash
# Round-4 GPU batch f: the D = 256 asm backward tests (tolerance per split-count grouping),
# the D = 256 micro-benchmark compiled vs asm, the graph-step loss probe, and the K-split-wave
# conv weight gradient (VDIFF_WGRAD_KS=1) against the default, each checked against the fp32
# parity-mode kernel.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04f}
timeout -k 10 300 python3 -u -m pytest -v -s --timeout 120 --timeout-method thread \
  -p no:cacheprovider tests/test_gpu_attention_asm256.py > gpurun_out/${T}_asm256_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_asm256_tests.log
[ $rc -eq 0 ] || { grep -E "rel-L2|FAILED" gpurun_out/${T}_asm256_tests.log | head; echo "rc=$rc: stopping"; exit $rc; }
for a in 0 1; do
  VDIFF_ASM256=$a timeout -k 10 200 python3 -u tools/attn_bench.py 20 --only 256 \
    > gpurun_out/${T}_bench256_a$a.log 2>&1 || { echo "attn_bench rc=$?"; tail -5 gpurun_out/${T}_bench256_a$a.log; exit 1; }
  echo "VDIFF_ASM256=$a"; grep -v amdgpu.ids gpurun_out/${T}_bench256_a$a.log
done
for tw in "" "--twin"; do
  timeout -k 10 300 python3 -u tools/graph_loss_probe.py --steps 7 $tw > gpurun_out/${T}_loss_probe$tw.log 2>&1
  prc=$?; echo "loss probe $tw"; grep -v amdgpu.ids gpurun_out/${T}_loss_probe$tw.log
  [ $prc -eq 0 ] || { echo "probe rc=$prc: stopping"; exit $prc; }
done
for ks in 0 1; do
  VDIFF_WGRAD_KS=$ks timeout -k 10 300 python3 -u tools/wgrad_ab.py > gpurun_out/${T}_wgrad_ks$ks.log 2>&1
  wrc=$?; grep -v amdgpu.ids gpurun_out/${T}_wgrad_ks$ks.log
  [ $wrc -eq 0 ] || { echo "wgrad_ab rc=$wrc: stopping"; exit $wrc; }
done
