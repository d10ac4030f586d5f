#!/bin/bash
# Round-4 GPU batch n: the kw-strip weight gradient's tile / ring / split-size knobs
# (VDIFF_WGRAD3=nst,cot,msteps) re-measured in the fixed-order mode, where the split-K epilogue
# is a plain partial store plus one finish pass instead of fp32 atomics (round 3's sweep,
# profiles/r03_ab_wgrad3*.txt, ran with atomics).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04n}
for v in 2,64,32 2,64,64 2,64,128 2,128,32 2,128,64 3,128,32 3,64,64 2,64,16; do
  VDIFF_WGRAD3=$v timeout -k 10 300 python3 -u tools/wgrad_ab.py > gpurun_out/${T}_wgrad_$v.log 2>&1
  rc=$?; echo "VDIFF_WGRAD3=$v: $(grep 'per train step' gpurun_out/${T}_wgrad_$v.log)"
  [ $rc -eq 0 ] || { echo "rc=$rc: stopping"; tail -5 gpurun_out/${T}_wgrad_$v.log; exit $rc; }
done
# the headline train leg twice (default lr 1e-3, host RNGs seeded): identical loss sequences?
for k in 1 2; do
  timeout -k 10 400 python3 -u bench.py --only train --steps 20 --warmup 5 --no-cpu \
    --xattn-steps 0 --vivit-steps 0 > gpurun_out/${T}_train_rep$k.json 2> gpurun_out/${T}_train_rep$k.err \
    || { echo "bench rc=$?"; tail -5 gpurun_out/${T}_train_rep$k.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['roofline']['frac'], d['train_losses'])" gpurun_out/${T}_train_rep$k.json
done
