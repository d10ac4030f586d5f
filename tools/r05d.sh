#!/bin/bash
# Round-5 batch d: graph reproducers.  Pure HIP with ~1 KiB kernel arguments (reduction node
# and eager launches between replays), then the torch-only reproducer with the graph's
# gradients checked against an eager recompute and 1x / 3x the host work between replays.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05d
for pc in unset 0; do
  for args in "2000 3 2" "2000 3 0" "2000 2 2"; do
    if [ $pc = unset ]; then E=(); else E=(env DEBUG_CLR_GRAPH_PACKET_CAPTURE=0); fi
    timeout -k 10 120 "${E[@]}" tools/graph_memset_repro.bin $args >> gpurun_out/${T}_hiprepro.txt 2>&1 \
      || { echo "repro rc=$?"; tail -3 gpurun_out/${T}_hiprepro.txt; exit 1; }
  done
done
cat gpurun_out/${T}_hiprepro.txt
for v in "--check-grads" "--check-grads --host-ops 3" "--check-grads --quiet-host"; do
  timeout -k 10 200 python3 -u tools/graph_reduce_repro.py $v >> gpurun_out/${T}_repro.txt 2>&1 \
    || { echo "repro rc=$?"; tail -5 gpurun_out/${T}_repro.txt; exit 1; }
done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 200 python3 -u tools/graph_reduce_repro.py --check-grads \
  --host-ops 3 >> gpurun_out/${T}_repro.txt 2>&1 || { echo "repro rc=$?"; tail -5 gpurun_out/${T}_repro.txt; exit 1; }
cat gpurun_out/${T}_repro.txt
