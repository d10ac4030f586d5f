#!/bin/bash
# Round-5 batch m: the LDS-tiled batched weight pack -- equality tests, then rocprof of a
# short train-only bench (pack_weights_kernel time per step).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05m
timeout -k 10 600 python3 -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_modules.py -k "pack or five_steps" tests/test_gpu_elementwise.py -k pack \
  > gpurun_out/${T}_tests.log 2>&1
rc=$?; grep -E "FAIL|passed|failed" gpurun_out/${T}_tests.log | tail -8
case $rc in 0) ;; *) echo "pytest rc=$rc: stopping"; grep -E "Error|assert" gpurun_out/${T}_tests.log | head; exit $rc;; esac
rm -rf /tmp/prof_${T}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_${T} -o run -- \
  python3 -u bench.py --steps 5 --warmup 2 --only train --xattn-steps 0 --st-steps 0 --no-cpu \
  > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "rocprof rc=$?"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
db=$(find /tmp/prof_${T} -name '*.db' | head -n 1)
python3 tools/prof_summary.py "$db" > gpurun_out/${T}_kernel_stats.md
grep -E "pack_weight|unit \(grids" gpurun_out/${T}_kernel_stats.md
