#!/bin/bash
# Round-3 GPU batch q: loss sequences of the paired graph / eager trainers at the config-2
# shape (lr 1e-2, the same clip each step), and of two eager trainers (the run-to-run spread).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03q}
timeout -k 10 400 python3 -u bench.py --only train --steps 5 --warmup 3 --no-cpu --xattn-steps 0 \
  --train-graph > gpurun_out/${T}_graph.json 2> gpurun_out/${T}_graph.err || { tail -20 gpurun_out/${T}_graph.err; exit 1; }
python3 -c "import json,sys; print(json.dumps(json.load(open(sys.argv[1]))['train_graph']))" gpurun_out/${T}_graph.json
VDIFF_GRAPH_LEG_EAGER=1 timeout -k 10 400 python3 -u bench.py --only train --steps 5 --warmup 3 --no-cpu \
  --xattn-steps 0 --train-graph > gpurun_out/${T}_eager2.json 2> gpurun_out/${T}_eager2.err || { tail -20 gpurun_out/${T}_eager2.err; exit 1; }
python3 -c "import json,sys; print(json.dumps(json.load(open(sys.argv[1]))['train_graph']))" gpurun_out/${T}_eager2.json
