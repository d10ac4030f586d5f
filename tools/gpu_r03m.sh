#!/bin/bash
# Round-3 GPU batch m: graph-replayed train step (Trainer(graph=True)) tests, the GPU idle
# time inside the eager step (batch l), and the graph leg against the eager step in bench.py.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03m}
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_train_graph.py > gpurun_out/${T}_graph_tests.txt 2>&1; rc=$?
tail -12 gpurun_out/${T}_graph_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --only train --steps 5 --warmup 3 --no-cpu --xattn-steps 0 \
  > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
grep -E 'train|graph' gpurun_out/${T}_bench.err | tail -5
bash tools/gpu_r03l.sh ${T}l
