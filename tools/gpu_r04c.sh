#!/bin/bash
# Round-4 GPU batch c: the hand-scheduled head_dim-256 dQ (asm/gen_d256.py): parity tests, then
# the D = 256 micro-benchmark with the compiled dQ (default) and the asm dQ (VDIFF_ASM256=1).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04c}
VDIFF_ASM256=1 timeout -k 10 300 python3 -u -m pytest -v -s --timeout 120 --timeout-method thread \
  -p no:cacheprovider tests/test_gpu_attention_asm256.py > gpurun_out/${T}_asm256_tests.log 2>&1
rc=$?; tail -4 gpurun_out/${T}_asm256_tests.log; grep -E "rel-L2|FAILED|Error" gpurun_out/${T}_asm256_tests.log | head -20
[ $rc -eq 0 ] || { echo "asm256 tests rc=$rc: stopping"; exit $rc; }
for a in 0 1; do
  VDIFF_ASM256=$a timeout -k 10 200 python3 -u tools/attn_bench.py 20 --only 256 \
    > gpurun_out/${T}_bench256_a$a.log 2>&1 || { echo "attn_bench rc=$?"; tail -5 gpurun_out/${T}_bench256_a$a.log; exit 1; }
  echo "VDIFF_ASM256=$a"; cat gpurun_out/${T}_bench256_a$a.log
done
