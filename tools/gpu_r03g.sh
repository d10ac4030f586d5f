#!/bin/bash
# Round-3 GPU batch g: the cost of per-launch conv events inside the timed train step
# (bench.py --timer-convs, the round-2 measurement) against the attention-only timer, two
# alternations on one box; then the default bench line and its rocprofv3 summary.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03g}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_modules.py -k pack > gpurun_out/${T}_pack_tests.log 2>&1; rc=$?
tail -1 gpurun_out/${T}_pack_tests.log; case $rc in 0|1) ;; *) exit $rc ;; esac
for i in 1 2; do
  for f in "" "--timer-convs"; do
    timeout -k 10 300 python -u bench.py --only train --no-cpu --steps 5 --warmup 2 $f \
      > gpurun_out/${T}_ab$i${f:+_tc}.json 2> gpurun_out/${T}_ab$i${f:+_tc}.err \
      || { tail -5 gpurun_out/${T}_ab$i${f:+_tc}.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d['roofline']['avg_unit_ms'])" gpurun_out/${T}_ab$i${f:+_tc}.json
  done
done
timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err \
  || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
tail -c 300 gpurun_out/${T}_bench.json
rm -rf /tmp/prof_${T}
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/prof_${T} -o run -- \
  python -u bench.py > gpurun_out/${T}_bench_profiled.json 2> gpurun_out/${T}_bench_profiled.err \
  || { tail -20 gpurun_out/${T}_bench_profiled.err; exit 1; }
db=$(find /tmp/prof_${T} -name '*.db' | head -n 1)
python tools/prof_summary.py "$db" > gpurun_out/${T}_kernel_stats.md
head -12 gpurun_out/${T}_kernel_stats.md
