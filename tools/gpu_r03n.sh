#!/bin/bash
# Round-3 GPU batch n (end of round): the GPU suite and smoke, the default bench line (with
# the graph-replayed train-step leg) and the rocprofv3 summary of the same invocation.
#   bash tools/gpu_r03n.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03n}
ok() { case $1 in 0|1) return 0 ;; *) echo "stopping: rc $1"; exit $1 ;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${T}_gpu_tests.log; ok $rc
timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err \
  || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
tail -c 300 gpurun_out/${T}_bench.json
rm -rf /tmp/prof_${T}
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/prof_${T} -o run -- \
  python -u bench.py > gpurun_out/${T}_bench_profiled.json 2> gpurun_out/${T}_bench_profiled.err \
  || { tail -20 gpurun_out/${T}_bench_profiled.err; exit 1; }
db=$(find /tmp/prof_${T} -name '*.db' | head -n 1)
python tools/prof_summary.py "$db" > gpurun_out/${T}_kernel_stats.md
head -16 gpurun_out/${T}_kernel_stats.md
