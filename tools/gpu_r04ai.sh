#!/bin/bash
# Round-4 GPU batch ai: the benchmark with no flags (the driver's default invocation), timed.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
s=$(date +%s)
timeout -k 10 900 python3 -u bench.py > gpurun_out/r04ai_bench_default.json 2> gpurun_out/r04ai_bench_default.err
rc=$?; e=$(date +%s); echo "bench (no flags) rc=$rc wall $((e - s)) s"; tail -c 400 gpurun_out/r04ai_bench_default.json; echo
exit $rc
