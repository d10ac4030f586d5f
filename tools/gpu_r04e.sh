#!/bin/bash
# Round-4 GPU batch e: (1) the head_dim-256 asm backward after the store-data hazard fix
# (asmgen STORE_DATA: a VALU write of the data VGPRs of a 128-bit store 1 instruction after
# it clobbered the fp32 partials of lanes 12-15 of every 16): its tests, then the D = 256
# micro-benchmark compiled vs asm; (2) where the graph step's wrong loss comes from.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04e}
VDIFF_ASM256=1 timeout -k 10 300 python3 -u -m pytest -v -s --timeout 120 --timeout-method thread \
  -p no:cacheprovider tests/test_gpu_attention_asm256.py > gpurun_out/${T}_asm256_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_asm256_tests.log; grep -E "rel-L2|FAILED" gpurun_out/${T}_asm256_tests.log | head -30
if [ $rc -ne 0 ]; then
  VDIFF_ASM256_DQ_L=1 timeout -k 10 200 python3 -u tools/asm256_dump.py 1024 > gpurun_out/${T}_asm256_dump.log 2>&1
  grep -v amdgpu.ids gpurun_out/${T}_asm256_dump.log | head -60
  echo "asm256 tests rc=$rc: stopping"; exit $rc
fi
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
