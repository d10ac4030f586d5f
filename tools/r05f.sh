#!/bin/bash
# Round-5 batch f: the torch-only graph reproducer with the graph's memset nodes listed and
# their destinations (the reduction's semaphore) read after every replay.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05f
for v in "--check-grads --host-ops 3 --probe-sem" "--check-grads --host-ops 3 --probe-sem"; do
  timeout -k 10 200 python3 -u tools/graph_reduce_repro.py $v >> gpurun_out/${T}_repro.txt 2>&1 \
    || { echo "repro rc=$?"; tail -5 gpurun_out/${T}_repro.txt; exit 1; }
done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 200 python3 -u tools/graph_reduce_repro.py \
  --check-grads --host-ops 3 --probe-sem >> gpurun_out/${T}_repro.txt 2>&1 \
  || { echo "repro rc=$?"; tail -5 gpurun_out/${T}_repro.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_repro.txt
