#!/bin/bash
# Round-4 GPU batch g: the graph-step loss probe matrix (prediction buffer kept alive x
# synchronised reads, with the eager twin), then the whole -m gpu suite and the default bench
# line with the D = 256 hand-scheduled backward as the default.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04g}
for kp in 1 0; do for sy in 1 0; do
  timeout -k 10 300 python3 -u tools/graph_loss_probe.py --steps 7 --twin --keep-pred $kp --sync $sy \
    > gpurun_out/${T}_probe_k${kp}_s${sy}.log 2>&1
  prc=$?; echo "keep-pred $kp sync $sy"; grep -v amdgpu.ids gpurun_out/${T}_probe_k${kp}_s${sy}.log | python3 -c "
import json,sys
for l in sys.stdin:
    try: d=json.loads(l)
    except Exception: print(l.strip()); continue
    print(d['step'], d['graph'], d['returned'], d['eager_twin'], d.get('loss_out'), d.get('loss_after'))"
  [ $prc -eq 0 ] || { echo "probe rc=$prc: stopping"; exit $prc; }
done; done
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?; tail -15 gpurun_out/${T}_gpu_tests.log | grep -E "passed|failed|FAILED|Error" 
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 900 python3 -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
brc=$?; tail -c 600 gpurun_out/${T}_bench.json; echo; tail -3 gpurun_out/${T}_bench.err
exit $brc
