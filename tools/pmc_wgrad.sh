#!/bin/bash
# PMC passes over tools/wgrad3_bench.py --det for one shape:
#   bash tools/pmc_wgrad.sh OUTDIR CI,CO,H [MODES]   (MODES: vd_conv_set_wgrad values, e.g. 0,1;
#   the two kernels have different names, so one pass counts both)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$1
MODES=${3:-1}
mkdir -p $OUT
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
G2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
G3="SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_SMEM SQ_IFETCH"
i=0
for G in "$G1" "$G2" "$G3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G --output-format csv -d $OUT/p$i -o pmc -- python tools/wgrad3_bench.py --det --only $2 --modes $MODES > $OUT/p$i.log 2>&1
done
