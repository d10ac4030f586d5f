#!/bin/bash
# PMC passes (two SQ groups) over the D=64 forward for the configs given: tools/pmc_fwd.sh w8 pp
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
G1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU"
G2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC SQ_INSTS_SALU GRBM_GUI_ACTIVE"
for c in "$@"; do
  i=0
  for G in "$G1" "$G2"; do
    i=$((i+1))
    VDIFF_ATTN_CFG=$c timeout -s KILL 120 rocprofv3 --pmc $G --output-format csv -d gpurun_out/pmcf/$c$i -o pmc -- python tools/attn_bench.py 1 --only 64 --nocheck > gpurun_out/pmcf_$c$i.log 2>&1
  done
done
python tools/pmc_table.py gpurun_out/pmcf > gpurun_out/pmcf.md
