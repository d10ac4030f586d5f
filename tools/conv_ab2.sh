#!/bin/bash
# conv A/B: tests, then the train-step bench with libvdiff.so and with libvdiff_base.so
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$PWD/lipreading-video-generation_amd/vdiff
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_modules.py -x -q --timeout 120 --timeout-method thread > gpurun_out/cab_t.log 2>&1 || { tail -30 gpurun_out/cab_t.log; exit 1; }
timeout -k 10 300 python bench.py --only train --no-cpu > gpurun_out/cab_new.json 2> gpurun_out/cab_new.err
VDIFF_LIB=$L/libvdiff_base.so timeout -k 10 300 python bench.py --only train --no-cpu > gpurun_out/cab_old.json 2> gpurun_out/cab_old.err
