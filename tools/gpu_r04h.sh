#!/bin/bash
# Round-4 GPU batch h: which part of tools/graph_localize.py makes the graph step's returned
# loss wrong (batch r04d) when tools/graph_loss_probe.py never sees it (r04g): the gradient
# copies (eager hooks + clones of the replayed gradients) on / off, the loss read before them.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04h}
for v in "" "--loss-first" "--no-grads"; do
  timeout -k 10 300 python3 -u tools/graph_localize.py --size 64 --steps 6 --lr 1e-2 $v \
    > gpurun_out/${T}_gl$v.log 2>&1
  grc=$?; echo "variant '$v'"; grep -v amdgpu.ids gpurun_out/${T}_gl$v.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l)
    print({k: d[k] for k in d if k in ('step','loss_eager','loss_graph','n_differ','n_weights_differ','steps_bad','trainer','loss_changed_after_copies')})"
  case $grc in 0|1) ;; *) echo "rc=$grc: stopping"; exit $grc;; esac
done
