#!/bin/bash
# Round-5 batch k: the short-sequence (temporal) attention kernels -- timing at the three
# config-2 levels, then the PMC passes (HBM bytes per launch, MFMA / VALU / LDS counters).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python3 -u tools/attn_bench.py 20 --temporal > gpurun_out/r05k_temporal_timing.txt 2>&1 \
  || { echo "bench rc=$?"; tail -5 gpurun_out/r05k_temporal_timing.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r05k_temporal_timing.txt
PMC_OUT=gpurun_out/r05k_pmc_temporal timeout -k 10 700 bash tools/pmc_attn.sh --temporal > gpurun_out/r05k_pmc.log 2>&1 \
  || { echo "pmc rc=$?"; tail -5 gpurun_out/r05k_pmc.log; exit 1; }
cat gpurun_out/r05k_pmc_temporal/pmc_attn.md | head -40
