#!/bin/bash
# Round-4 GPU batch r: (1) the head_dim-256 forward now the default: its test file; (2) its
# generator variants (LDS read distances); (3) the weight-gradient pixel-split sweep
# (tools/gpu_r04q.sh).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04r}
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_attention_asm256.py > gpurun_out/${T}_asm256_tests.log 2>&1
rc=$?; tail -1 gpurun_out/${T}_asm256_tests.log
[ $rc -eq 0 ] || { echo "tests rc=$rc: stopping"; grep -E "Error|assert" gpurun_out/${T}_asm256_tests.log | tail -10; exit $rc; }
timeout -k 10 300 python3 -u tools/asm_ab256.py 'base:' 'rd3:RD_AHEAD=3' 'rd4:RD_AHEAD=4' \
  'rd5:RD_AHEAD=5' 'tr3:TR_AHEAD=3' 'tr6:TR_AHEAD=6' 'rd4tr6:RD_AHEAD=4,TR_AHEAD=6' 'ch1:CHAINS=1' \
  'base2:' > gpurun_out/${T}_asm_ab256.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${T}_asm_ab256.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r04q.sh ${T}q
