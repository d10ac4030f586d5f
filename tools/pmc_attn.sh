#!/bin/bash
# PMC passes over the attention micro-benchmark (one counter group per rocprofv3 run).
#   bash tools/pmc_attn.sh [extra attn_bench args, e.g. --only 64]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${PMC_OUT:-gpurun_out/pmc}
mkdir -p $OUT
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
G2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
G3="FETCH_SIZE"
G4="WRITE_SIZE"
G5="SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_SMEM SQ_IFETCH"
i=0
for G in "$G1" "$G2" "$G3" "$G4" "$G5"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $G --output-format csv -d $OUT/p$i -o pmc -- python tools/attn_bench.py 1 --calib --nocheck "$@" > $OUT/p$i.log 2>&1
done
python tools/pmc_traffic.py $OUT $OUT/pmc_traffic.json $OUT/pmc_attn.md
