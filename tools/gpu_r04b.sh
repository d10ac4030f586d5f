#!/bin/bash
# Round-4 GPU batch b.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04b}
# (0) the tests that failed in batch a (test bugs, fixed)
VDIFF_TEST_METRICS=gpurun_out/${T}_metrics.jsonl timeout -k 10 400 python3 -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_elementwise.py -k cond_concat_bwd tests/test_gpu_fullsize.py::test_config2_model_vs_oracle_spatial_temporal \
  -s > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -4 gpurun_out/${T}_tests.log; grep -E "config2_spatial|FAILED" gpurun_out/${T}_tests.log | head
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
cat gpurun_out/${T}_metrics.jsonl 2>/dev/null | tail -2
# (1) graph-replayed train step vs eager at lr 0, bit for bit (64x64 and 128x128)
for s in 64 128; do
  timeout -k 10 400 python3 -u tools/graph_localize.py --size $s --steps 4 \
    > gpurun_out/${T}_graphloc_$s.log 2>&1
  grc=$?
  cat gpurun_out/${T}_graphloc_$s.log | tail -6
  case $grc in 0|1) ;; *) echo "graph_localize rc=$grc: stopping"; exit $grc;; esac
done
# (2) out-of-bounds write check of the config-2 eager train step
timeout -k 10 900 python3 -u tools/guard_check.py --steps 2 > gpurun_out/${T}_guard.json \
  2> gpurun_out/${T}_guard.err
rc=$?
tail -5 gpurun_out/${T}_guard.err; cat gpurun_out/${T}_guard.json
case $rc in 0|1) ;; *) echo "guard check rc=$rc: stopping"; exit $rc;; esac
# (3) the bench train leg from both inits at the reference lr (losses + ms/step)
for init in nonzero reference; do
  timeout -k 10 400 python3 -u bench.py --only train --steps 20 --warmup 5 --no-cpu \
    --xattn-steps 0 --vivit-steps 0 --init $init > gpurun_out/${T}_bench_${init}.json \
    2> gpurun_out/${T}_bench_${init}.err
  brc=$?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['roofline']['frac'], d['train_losses'], d['conv_kernels'])" gpurun_out/${T}_bench_${init}.json $init
  case $brc in 0|3) ;; *) echo "bench rc=$brc: stopping"; tail -5 gpurun_out/${T}_bench_${init}.err; exit $brc;; esac
done
# (4) conv weight-gradient A/B: XCD-aware grid on/off x fixed-order / atomic split-K
for v in "1 0" "0 0" "1 1" "0 1"; do
  set -- $v
  VDIFF_WGRAD_XCD=$1 VDIFF_WGRAD_ATOMIC=$2 timeout -k 10 300 python3 -u tools/wgrad_ab.py \
    > gpurun_out/${T}_wgrad_x$1_a$2.log 2>&1 || { echo "wgrad_ab rc=$?"; tail -5 gpurun_out/${T}_wgrad_x$1_a$2.log; exit 1; }
  tail -1 gpurun_out/${T}_wgrad_x$1_a$2.log
done
# (5) PMC passes over the head_dim-256 attention kernels
PMC_OUT=gpurun_out/${T}_pmc256 timeout -k 10 900 bash tools/pmc_attn.sh --only 256 \
  > gpurun_out/${T}_pmc256.log 2>&1 || { echo "pmc rc=$?"; tail -5 gpurun_out/${T}_pmc256.log; exit 1; }
cat gpurun_out/${T}_pmc256/pmc_attn.md
# (6) the hand-scheduled head_dim-256 backward kernels (new; last, each step time-limited)
bash tools/gpu_r04c.sh ${T}c
