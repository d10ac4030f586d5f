#!/bin/bash
# Round-3 GPU batch s: localise the graph-replay loss defect -- paired graph / eager loss
# sequences (a) without ResBlock dropout at config 2, (b) with dropout at 64x64x16.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03s}
VDIFF_BENCH_DROPOUT=0 timeout -k 10 400 python3 -u bench.py --only train --steps 5 --warmup 3 \
  --no-cpu --xattn-steps 0 --train-graph > gpurun_out/${T}_nodrop.json 2> gpurun_out/${T}_nodrop.err \
  || { tail -20 gpurun_out/${T}_nodrop.err; exit 1; }
python3 -c "import json,sys; print(json.dumps(json.load(open(sys.argv[1]))['train_graph']))" gpurun_out/${T}_nodrop.json
timeout -k 10 400 python3 -u bench.py --only train --steps 5 --warmup 3 --size 64 \
  --no-cpu --xattn-steps 0 --train-graph > gpurun_out/${T}_s64.json 2> gpurun_out/${T}_s64.err \
  || { tail -20 gpurun_out/${T}_s64.err; exit 1; }
python3 -c "import json,sys; print(json.dumps(json.load(open(sys.argv[1]))['train_graph']))" gpurun_out/${T}_s64.json
