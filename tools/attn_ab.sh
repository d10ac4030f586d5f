#!/bin/bash
# A/B timing of attention builds and kernel shapes on the GPU box:
#   bash tools/attn_ab.sh "libvdiff libvdiff_noslp" "auto o3" [head_dim]
# Each (library, VDIFF_ATTN_CFG) pair runs tools/attn_bench.py (3 reps) under its own time limit.
set -e
cd "$GRAFT_REPO_ROOT"
LIBS=${1:-libvdiff}; CFGS=${2:-auto}; ONLY=${3:-64}
for lib in $LIBS; do
  for cfg in $CFGS; do
    echo "== $lib cfg=$cfg"
    VDIFF_LIB=lipreading-video-generation_amd/vdiff/$lib.so VDIFF_ATTN_CFG=$cfg \
      timeout -k 10 150 python -u tools/attn_bench.py --nocheck 3 --only $ONLY
  done
done
