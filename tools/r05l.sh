#!/bin/bash
# Round-5 batch l: the vectorised batched weight pack (tests + rocprof of a short train-only
# bench), then the PMC passes of the head_dim-128 attention kernels.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05l
timeout -k 10 600 python3 -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_modules.py -k "pack or five_steps" tests/test_gpu_elementwise.py::test_conv_pack_weight \
  > gpurun_out/${T}_tests.log 2>&1
rc=$?; grep -E "FAIL|passed|failed" gpurun_out/${T}_tests.log | tail -8
case $rc in 0) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
rm -rf /tmp/prof_${T}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_${T} -o run -- \
  python3 -u bench.py --steps 5 --warmup 2 --only train --xattn-steps 0 --st-steps 0 --no-cpu \
  > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "rocprof rc=$?"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
db=$(find /tmp/prof_${T} -name '*.db' | head -n 1)
python3 tools/prof_summary.py "$db" > gpurun_out/${T}_kernel_stats.md
grep -E "pack_weight|unit \(grids" gpurun_out/${T}_kernel_stats.md
PMC_OUT=gpurun_out/${T}_pmc128 timeout -k 10 600 bash tools/pmc_attn.sh --only 128 > gpurun_out/${T}_pmc128.log 2>&1 \
  || { echo "pmc128 rc=$?"; tail -5 gpurun_out/${T}_pmc128.log; exit 1; }
python3 tools/pmc_derive.py gpurun_out/${T}_pmc128/pmc_attn.md | head -20
