#!/bin/bash
# End-of-round measurement set (GPU box): PMC passes over the head_dim-64 attention kernels
# (HBM traffic + MFMA-busy; the table bench.py reads), the full GPU test suite, smoke, the
# default bench.py line, then rocprofv3 --kernel-trace --stats of the very same invocation.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
true
true
true
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_final.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_final.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_final.log
timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/r02e_bench.json 2> gpurun_out/r02e_bench.err || { tail -20 gpurun_out/r02e_bench.err; exit 1; }
tail -c 300 gpurun_out/r02e_bench.json
rm -rf /tmp/prof_r02e
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/prof_r02e -o run -- \
  python -u bench.py > gpurun_out/r02e_bench_profiled.json 2> gpurun_out/r02e_bench_profiled.err || { tail -20 gpurun_out/r02e_bench_profiled.err; exit 1; }
db=$(find /tmp/prof_r02e -name '*.db' | head -n 1)
python tools/prof_summary.py "$db" > gpurun_out/r02e_kernel_stats.md
head -10 gpurun_out/r02e_kernel_stats.md
