#!/bin/bash
# Round-3 GPU batch o: the small-kernel changes (channel-sum finish, GroupNorm backward without
# the memset) through their tests, the graph / pack / module suites, then the paired graph vs
# eager train step and the per-kernel summary of a short train-only bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03o}
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_gpu_elementwise.py tests/test_gpu_groupnorm.py tests/test_gpu_train_graph.py \
  tests/test_gpu_modules.py tests/test_vivit.py > gpurun_out/${T}_tests.txt 2>&1; rc=$?
tail -3 gpurun_out/${T}_tests.txt
[ $rc -eq 0 ] || exit $rc
rm -rf /tmp/prof_${T}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_${T} -o run -- \
  python3 -u bench.py --only train --steps 5 --warmup 3 --no-cpu --xattn-steps 0 \
  > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
grep -E 'train' gpurun_out/${T}_bench.err | tail -3
db=$(find /tmp/prof_${T} -name '*.db' | head -n 1)
python3 tools/prof_summary.py "$db" > gpurun_out/${T}_kernel_stats.md
grep -E 'channel_sums|gn_bwd|fillBuffer' gpurun_out/${T}_kernel_stats.md
