#!/bin/bash
# Round-4 GPU batch p: first run of the hand-scheduled head_dim-256 forward
# (csrc/asm/gen_fwd256.py): its parity tests against the compiled forward and an fp32
# reference, then the timing A/B at N = 16384 / 4096.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04p}
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_attention_asm256.py -k "fwd" -rP > gpurun_out/${T}_fwd256_tests.log 2>&1
rc=$?; grep -E "passed|failed|Error|error" gpurun_out/${T}_fwd256_tests.log | tail -5
[ $rc -eq 0 ] || { echo "tests rc=$rc: stopping"; grep -E "rel-L2|assert" gpurun_out/${T}_fwd256_tests.log | tail -20; exit $rc; }
timeout -k 10 200 python3 -u tools/fwd256_ab.py > gpurun_out/${T}_fwd256_ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${T}_fwd256_ab.log
[ $rc -eq 0 ] || exit $rc
# generator variants: LDS read distances ahead of the MFMAs
timeout -k 10 300 python3 -u tools/asm_ab256.py 'base:' 'rd3:RD_AHEAD=3' 'rd4:RD_AHEAD=4' \
  'rd5:RD_AHEAD=5' 'tr3:TR_AHEAD=3' 'tr6:TR_AHEAD=6' 'rd4tr6:RD_AHEAD=4,TR_AHEAD=6' 'ch1:CHAINS=1' \
  'base2:' > gpurun_out/${T}_asm_ab256.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${T}_asm_ab256.log
exit $rc
