#!/bin/bash
# Round-4 GPU batch m: the headline's train leg (driver's --steps 20 --warmup 5) from both
# inits at the reference lr and at 1e-3: loss sequences (finite?) and ms/step; then the
# two-rank bench spawn tests.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04m}
for v in "nonzero 1e-2" "reference 1e-2" "nonzero 1e-3" "reference 1e-3"; do
  set -- $v
  timeout -k 10 400 python3 -u bench.py --only train --steps 20 --warmup 5 --no-cpu \
    --xattn-steps 0 --vivit-steps 0 --init $1 --lr $2 > gpurun_out/${T}_train_$1_$2.json \
    2> gpurun_out/${T}_train_$1_$2.err
  brc=$?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['roofline']['frac'], d['train_losses'])" gpurun_out/${T}_train_$1_$2.json "$1 lr $2 rc $brc"
  case $brc in 0|3) ;; *) echo "bench rc=$brc: stopping"; tail -5 gpurun_out/${T}_train_$1_$2.err; exit $brc;; esac
done
timeout -k 10 600 python3 -u -m pytest -v --timeout 500 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_bench_spawn.py > gpurun_out/${T}_spawn_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed" gpurun_out/${T}_spawn_tests.log | tail -6
exit $rc
