#!/bin/bash
# Round-4 GPU batch o: the 128 x 128-tile weight gradient (wgrad_wide_kernel, 8 waves, half
# the LDS-DMA bytes per MAC; VDIFF_WGRAD_WIDE=1) against the default, both checked against
# the fp32 parity-mode kernel.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04o}
for w in 1 2 0; do
  VDIFF_WGRAD_WIDE=$w timeout -k 10 300 python3 -u tools/wgrad_ab.py > gpurun_out/${T}_wgrad_wide$w.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/${T}_wgrad_wide$w.log | grep -E "k3|per train"
  [ $rc -eq 0 ] || { echo "rc=$rc: stopping"; tail -5 gpurun_out/${T}_wgrad_wide$w.log; exit $rc; }
done
# the D = 256 asm backward after the store-data padding went from 1 to 2 wait states
timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_attention_asm256.py > gpurun_out/${T}_asm256_tests.log 2>&1
rc=$?; tail -1 gpurun_out/${T}_asm256_tests.log
exit $rc
