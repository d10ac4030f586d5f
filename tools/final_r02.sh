#!/bin/bash
# Round-2 measurement set (GPU box): PMC passes over the head_dim-64 attention kernels
# (traffic + MFMA-busy; the table bench.py reads), the default bench.py line, then
# rocprofv3 --kernel-trace --stats of the very same bench.py invocation.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
[ -n "$NO_PMC" ] || bash tools/pmc_attn.sh --only 64 > gpurun_out/pmc_run.log 2>&1 || { tail -20 gpurun_out/pmc_run.log; exit 1; }
[ -n "$NO_PMC" ] || cp gpurun_out/pmc/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 900 python -u bench.py > gpurun_out/r02_bench.json 2> gpurun_out/r02_bench.err || { tail -20 gpurun_out/r02_bench.err; exit 1; }
tail -c 600 gpurun_out/r02_bench.json
rm -rf /tmp/prof_r02
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/prof_r02 -o run -- \
  python -u bench.py > gpurun_out/r02_bench_profiled.json 2> gpurun_out/r02_bench_profiled.err || { tail -20 gpurun_out/r02_bench_profiled.err; exit 1; }
db=$(find /tmp/prof_r02 -name '*.db' | head -n 1)
python tools/prof_summary.py "$db" > gpurun_out/r02_kernel_stats.md
head -12 gpurun_out/r02_kernel_stats.md
