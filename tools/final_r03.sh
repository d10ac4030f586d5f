#!/bin/bash
# Round-3 measurement set (GPU box): PMC passes over the head_dim-64 attention kernels with
# the hand-scheduled backward (default) and the pipelined backward (p8, before), the full
# GPU test suite, smoke, the default bench.py line, then rocprofv3 --kernel-trace --stats of
# the very same invocation.   bash tools/final_r03.sh [tag] [skip-pmc]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03}
if [ -z "$2" ]; then
  PMC_OUT=gpurun_out/pmc_${T}_asm timeout -k 10 600 bash tools/pmc_attn.sh --only 64 || exit 1
  PMC_OUT=gpurun_out/pmc_${T}_p8 VDIFF_ATTN_CFG=p8 timeout -k 10 600 bash tools/pmc_attn.sh --only 64 || exit 1
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.log
timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
tail -c 400 gpurun_out/${T}_bench.json
rm -rf /tmp/prof_${T}
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/prof_${T} -o run -- \
  python -u bench.py > gpurun_out/${T}_bench_profiled.json 2> gpurun_out/${T}_bench_profiled.err || { tail -20 gpurun_out/${T}_bench_profiled.err; exit 1; }
db=$(find /tmp/prof_${T} -name '*.db' | head -n 1)
python tools/prof_summary.py "$db" > gpurun_out/${T}_kernel_stats.md
head -14 gpurun_out/${T}_kernel_stats.md
