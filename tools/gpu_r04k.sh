#!/bin/bash
# Round-4 GPU batch k: the graph-step loss fix (engine.TrainStepGraph reports the eager MSE of
# the replayed prediction): its tests and the reproducer, then the round-4 measurement part 1
# (whole -m gpu suite, smoke, the driver's bench command) -- tools/final_r04.sh without the
# profiler passes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04k}
timeout -k 10 400 python3 -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_train_graph.py > gpurun_out/${T}_graph_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed" gpurun_out/${T}_graph_tests.log | tail -14
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 300 python3 -u tools/graph_localize.py --size 64 --steps 6 --lr 1e-2 \
  > gpurun_out/${T}_graphloc.log 2>&1
grc=$?; tail -2 gpurun_out/${T}_graphloc.log
case $grc in 0|1) ;; *) echo "rc=$grc: stopping"; exit $grc;; esac
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/${T}_gpu_tests.log | tail -2; grep FAILED gpurun_out/${T}_gpu_tests.log | head
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 600 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 \
  || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 900 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json \
  2> gpurun_out/${T}_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
tail -c 300 gpurun_out/${T}_bench.json; echo
