#!/bin/bash
# Round-5 batch e: the pure-HIP graph reproducer with torch's one-int semaphore memset.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05e
for pc in unset 0; do
  for args in "2000 1 3" "2000 2 3" "2000 3 3" "2000 0 3"; do
    if [ $pc = unset ]; then E=(); else E=(env DEBUG_CLR_GRAPH_PACKET_CAPTURE=0); fi
    timeout -k 10 120 "${E[@]}" tools/graph_memset_repro.bin $args >> gpurun_out/${T}_hiprepro.txt 2>&1 \
      || { echo "repro rc=$?"; tail -3 gpurun_out/${T}_hiprepro.txt; exit 1; }
  done
done
cat gpurun_out/${T}_hiprepro.txt
