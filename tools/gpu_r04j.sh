#!/bin/bash
# Round-4 GPU batch j: the graph step's wrong loss (reproduced by comparing the weights after
# each step, batch r04i): the MSE copied inside the graph before the backward, and the loss
# output cloned right after the replay (before Adam).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04j}
for v in "--compare-weights --snap" "--compare-weights"; do
  tag=$(echo "$v" | tr -d ' -')
  timeout -k 10 300 python3 -u tools/graph_loss_probe.py --steps 8 --twin --keep-pred 0 --sync 0 $v \
    > gpurun_out/${T}_probe_$tag.log 2>&1
  prc=$?; echo "variant '$v'"; grep -v amdgpu.ids gpurun_out/${T}_probe_$tag.log | python3 -c "
import json,sys
for l in sys.stdin:
    try: d=json.loads(l)
    except Exception: print(l.strip()); continue
    print(d['step'], d['graph'], d['returned'], d['eager_twin'], d.get('snap'), d.get('pre'), d.get('n_weights_differ'))"
  [ $prc -eq 0 ] || { echo "probe rc=$prc: stopping"; exit $prc; }
done
