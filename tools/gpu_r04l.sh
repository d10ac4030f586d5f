#!/bin/bash
# Round-4 measurement part 2: rocprofv3 --kernel-trace --stats of exactly the driver's bench
# command (`python3 bench.py --steps 20 --warmup 5`), summarised per kernel, then the PMC
# passes of the D = 64 and D = 256 attention kernels (HBM bytes per launch).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04l}
rm -rf /tmp/prof_${T}
timeout -k 10 1000 rocprofv3 --kernel-trace --stats -d /tmp/prof_${T} -o run -- \
  python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench_profiled.json \
  2> gpurun_out/${T}_bench_profiled.err || { echo "rocprof rc=$?"; tail -20 gpurun_out/${T}_bench_profiled.err; exit 1; }
db=$(find /tmp/prof_${T} -name '*.db' | head -n 1)
python3 tools/prof_summary.py "$db" > gpurun_out/${T}_kernel_stats.md || { echo "summary failed"; exit 1; }
head -14 gpurun_out/${T}_kernel_stats.md
tail -c 300 gpurun_out/${T}_bench_profiled.json; echo
if [ -z "$2" ]; then
  PMC_OUT=gpurun_out/${T}_pmc64 timeout -k 10 500 bash tools/pmc_attn.sh --only 64 > gpurun_out/${T}_pmc64.log 2>&1 \
    || { echo "pmc64 rc=$?"; tail -5 gpurun_out/${T}_pmc64.log; exit 1; }
  PMC_OUT=gpurun_out/${T}_pmc256 timeout -k 10 500 bash tools/pmc_attn.sh --only 256 > gpurun_out/${T}_pmc256.log 2>&1 \
    || { echo "pmc256 rc=$?"; tail -5 gpurun_out/${T}_pmc256.log; exit 1; }
  echo pmc done
fi
