#!/bin/bash
# Round-3 GPU batch: head_dim-128 hand-scheduled kernels (parity + A/B), forward generator
# knob sweep, the batched-pack test, then the default bench line and the rocprofv3 summary
# of the same invocation, then the whole GPU suite + smoke.   bash tools/gpu_r03c.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03c}
ok() { case $1 in 0|1) return 0 ;; *) echo "stopping: rc $1"; exit $1 ;; esac; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_attention_asm128.py > gpurun_out/${T}_asm128_tests.log 2>&1; rc=$?
grep -E "passed|failed|Error|assert" gpurun_out/${T}_asm128_tests.log | tail -8; ok $rc
for cfg in auto asm auto asm; do
  echo "== cfg=$cfg"
  VDIFF_ATTN_CFG=$cfg timeout -k 10 150 python -u tools/attn_bench.py --nocheck 3 --only 128 \
    2>&1 | tee -a gpurun_out/${T}_asm128_bench.log | grep -E "attn_fwd|attn_bwd_dq|attn_bwd_dkdv"
  ok $?
done
timeout -k 10 400 python -u tools/asm_ab.py 'base:' 'chains1:CHAINS=1' 'gsgs:GSGS=1' 'pd3:PD=3' \
  'pd5:PD=5' 'pd6:PD=6' 'bar2:BAR2=1' 'nop1:CHECK_NOP=1' 'dexp:DROP=1' 'dadd:DROP=2' \
  'dcvt:DROP=4' 'dread:DROP=8' 'norare:NORARE=1' 'stamp:STAMP=1' 'base2:' \
  > gpurun_out/${T}_fwd_knobs.txt 2>&1; rc=$?; tail -16 gpurun_out/${T}_fwd_knobs.txt; ok $rc
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_modules.py -k batched_pack > gpurun_out/${T}_pack_test.log 2>&1; rc=$?
tail -1 gpurun_out/${T}_pack_test.log; ok $rc
timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err \
  || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
tail -c 300 gpurun_out/${T}_bench.json
rm -rf /tmp/prof_${T}
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/prof_${T} -o run -- \
  python -u bench.py > gpurun_out/${T}_bench_profiled.json 2> gpurun_out/${T}_bench_profiled.err \
  || { tail -20 gpurun_out/${T}_bench_profiled.err; exit 1; }
db=$(find /tmp/prof_${T} -name '*.db' | head -n 1)
python tools/prof_summary.py "$db" > gpurun_out/${T}_kernel_stats.md
head -14 gpurun_out/${T}_kernel_stats.md
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${T}_gpu_tests.log; ok $rc
timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
tail -1 gpurun_out/${T}_smoke.log
