#!/bin/bash
# Round-4 GPU batch i: the product's graph step (no syncs, no extra references) with the eager
# twin, (a) re-seeding torch / numpy / random before each step, (b) comparing the weights after
# each step, (c) both -- the two things graph_localize.py does that graph_loss_probe.py did not.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04i}
for v in "--seed-each-step" "--compare-weights" "--seed-each-step --compare-weights"; do
  tag=$(echo "$v" | tr -d ' -')
  timeout -k 10 300 python3 -u tools/graph_loss_probe.py --steps 7 --twin --keep-pred 0 --sync 0 $v \
    > gpurun_out/${T}_probe_$tag.log 2>&1
  prc=$?; echo "variant '$v'"; grep -v amdgpu.ids gpurun_out/${T}_probe_$tag.log | python3 -c "
import json,sys
for l in sys.stdin:
    try: d=json.loads(l)
    except Exception: print(l.strip()); continue
    print(d['step'], d['graph'], d['returned'], d['eager_twin'], d.get('n_weights_differ'))"
  [ $prc -eq 0 ] || { echo "probe rc=$prc: stopping"; exit $prc; }
done
