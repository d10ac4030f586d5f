#!/bin/bash
# Halo-tile 3x3x3 conv (VDIFF_CONV_HALO=1) vs the gathered-tile kernel: conv GPU tests with
# the halo path on, then the train bench's per-direction conv times with and without it.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
VDIFF_CONV_HALO=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_halo.log 2>&1; rc=$?
echo "halo tests: $(tail -1 gpurun_out/pytest_halo.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_halo.log | head -20; exit $rc; }
for v in 0 1 0 1; do
  VDIFF_CONV_HALO=$v timeout -k 10 300 python bench.py --only train --no-cpu --steps 3 > gpurun_out/halo_$v.json 2> gpurun_out/halo_$v.err || { tail -5 gpurun_out/halo_$v.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('halo=$v', d['ms_per_step'], json.dumps(d['conv_kernels']))" gpurun_out/halo_$v.json
done
