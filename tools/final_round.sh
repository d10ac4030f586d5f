#!/bin/bash
# End-of-round measurement set (GPU box), every step under its own time limit and chained:
#   the whole -m gpu suite (no -x: every failure is listed), smoke(), the driver's bench
#   command `python bench.py --steps 20 --warmup 5`, then rocprofv3 --kernel-trace --stats of
#   that very command (its dQ + dK/dV averages reproduce roofline.frac), then the PMC passes
#   of the attention kernels (HBM traffic per launch, D = 64 and D = 256).
#   bash tools/final_round.sh [tag] [skip-pmc]
#   PHASE=a: the suite, smoke() and the bench only; PHASE=b: the profiled bench and the PMC
#   passes only (two gpurun calls under the 20-minute limit); default both.
#   The suite's measured parity errors go to gpurun_out/<tag>_parity_metrics.jsonl.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r05}
PHASE=${PHASE:-ab}
if [[ $PHASE == *a* ]]; then
VDIFF_TEST_METRICS=gpurun_out/${T}_parity_metrics.jsonl timeout -k 10 1100 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/${T}_gpu_tests.log | tail -2; grep FAILED gpurun_out/${T}_gpu_tests.log | head
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 600 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 \
  || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 900 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json \
  2> gpurun_out/${T}_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
tail -c 300 gpurun_out/${T}_bench.json; echo
fi
[[ $PHASE == *b* ]] || exit 0
rm -rf /tmp/prof_${T}
timeout -k 10 1000 rocprofv3 --kernel-trace --stats -d /tmp/prof_${T} -o run -- \
  python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench_profiled.json \
  2> gpurun_out/${T}_bench_profiled.err || { echo "rocprof rc=$?"; tail -20 gpurun_out/${T}_bench_profiled.err; exit 1; }
db=$(find /tmp/prof_${T} -name '*.db' | head -n 1)
python3 tools/prof_summary.py "$db" > gpurun_out/${T}_kernel_stats.md
head -12 gpurun_out/${T}_kernel_stats.md
if [ -z "$2" ]; then
  PMC_OUT=gpurun_out/${T}_pmc64 timeout -k 10 600 bash tools/pmc_attn.sh --only 64 > gpurun_out/${T}_pmc64.log 2>&1 \
    || { echo "pmc64 rc=$?"; tail -5 gpurun_out/${T}_pmc64.log; exit 1; }
  PMC_OUT=gpurun_out/${T}_pmc256 timeout -k 10 600 bash tools/pmc_attn.sh --only 256 > gpurun_out/${T}_pmc256.log 2>&1 \
    || { echo "pmc256 rc=$?"; tail -5 gpurun_out/${T}_pmc256.log; exit 1; }
  echo pmc done
fi
