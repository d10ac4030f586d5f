#!/bin/bash
# PMC passes over the head_dim-64 attention kernels (default config) + derived MFMA-busy.
#   bash tools/pmc_fwd_asm.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-pmc}
PMC_OUT=gpurun_out/pmc_$T timeout -k 10 600 bash tools/pmc_attn.sh --only 64 || exit 1
python3 tools/pmc_derive.py gpurun_out/pmc_$T/pmc_attn.md
