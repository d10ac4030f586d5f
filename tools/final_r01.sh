#!/bin/bash
# Round-end measurement: full bench.py line + rocprofv3 kernel summary of the same workload.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python bench.py > gpurun_out/bench_r01.json 2> gpurun_out/bench_r01.err
rm -rf /tmp/prof_r01
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_r01 -o run -- \
  python bench.py --no-cpu --c4-steps 0 > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err
db=$(find /tmp/prof_r01 -name '*.db' | head -n 1)
python tools/prof_summary.py "$db" > gpurun_out/r01_kernel_stats.md
