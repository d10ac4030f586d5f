#!/bin/bash
# Round-3 GPU batch t: the full-size DDIM graph vs eager check, then batch s (graph-replayed
# train-step defect localisation).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03t}
timeout -k 10 300 python3 -u tools/ddim_graph_check.py --steps 3 > gpurun_out/${T}_ddim_graph.json \
  2> gpurun_out/${T}_ddim_graph.err || { tail -20 gpurun_out/${T}_ddim_graph.err; exit 1; }
cat gpurun_out/${T}_ddim_graph.json
bash tools/gpu_r03s.sh ${T}s
