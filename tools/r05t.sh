#!/bin/bash
# Round-5 batch t: 1x1 streaming-kernel variants (VDIFF_PW_AB): nontemporal stores, workgroups
# per CU, persistent vs one tile per wave.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for ab in 0 1 64 65 256 257 0 1; do
  echo "== VDIFF_PW_AB=$ab" >> gpurun_out/r05t_pw.txt
  VDIFF_PW_AB=$ab timeout -k 10 120 python3 -u tools/conv1x1_bench.py >> gpurun_out/r05t_pw.txt 2>&1 \
    || { tail -5 gpurun_out/r05t_pw.txt; exit 1; }
done
grep -E "^==|->" gpurun_out/r05t_pw.txt | cut -c1-60
