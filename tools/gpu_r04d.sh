#!/bin/bash
# Round-4 GPU batch d: (1) the whole-model config-2 check against the oracle (deselected by
# batch b's -k filter); (2) the graph-replayed train step vs eager with the weights moving
# (lr 1e-2), bit for bit, without and with the wav2vec2 encoder; (3) the fixed-order weight
# gradient with the parallel finish; (4) the head_dim-256 asm backward per split count;
# (5) head_dim-64 forward row sums on the matrix pipe (gen_fwd.py MSUM=2) vs the 62-add body.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04d}
VDIFF_TEST_METRICS=gpurun_out/${T}_metrics.jsonl timeout -k 10 400 python3 -u -m pytest -v -s \
  --timeout 300 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_fullsize.py::test_config2_model_vs_oracle_spatial_temporal" \
  > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.log; cat gpurun_out/${T}_metrics.jsonl 2>/dev/null | tail -2
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
for spec in "64 6" "128 5"; do
  set -- $spec
  timeout -k 10 400 python3 -u tools/graph_localize.py --size $1 --steps $2 --lr 1e-2 \
    > gpurun_out/${T}_graphloc_lr_$1.log 2>&1
  grc=$?; cat gpurun_out/${T}_graphloc_lr_$1.log | grep -v amdgpu.ids
  case $grc in 0|1) ;; *) echo "graph_localize rc=$grc: stopping"; exit $grc;; esac
done
timeout -k 10 400 python3 -u tools/graph_localize.py --size 64 --steps 6 --lr 1e-2 --audio \
  > gpurun_out/${T}_graphloc_audio_64.log 2>&1
grc=$?; cat gpurun_out/${T}_graphloc_audio_64.log | grep -v amdgpu.ids
case $grc in 0|1) ;; *) echo "graph_localize rc=$grc: stopping"; exit $grc;; esac
timeout -k 10 300 python3 -u tools/wgrad_ab.py > gpurun_out/${T}_wgrad_det.log 2>&1 \
  || { echo "wgrad_ab rc=$?"; tail -5 gpurun_out/${T}_wgrad_det.log; exit 1; }
grep -E "k1|per train" gpurun_out/${T}_wgrad_det.log
timeout -k 10 300 python3 -u tools/asm256_debug.py > gpurun_out/${T}_asm256_debug.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${T}_asm256_debug.log | tail -40
[ $rc -eq 0 ] || { echo "asm256_debug rc=$rc: stopping"; exit $rc; }
timeout -k 10 300 python3 -u tools/asm_ab.py base: msum2:MSUM=2 base_st:STAMP=1 \
  msum2_st:MSUM=2,STAMP=1 base2: msum2b:MSUM=2 > gpurun_out/${T}_fwd_msum.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${T}_fwd_msum.log
exit $rc
