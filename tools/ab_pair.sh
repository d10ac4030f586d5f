#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
for lib in libvdiff libvdiff_prio; do
  echo "== $lib"
  VDIFF_LIB=lipreading-video-generation_amd/vdiff/$lib.so VDIFF_ATTN_CFG=pair timeout -k 10 150 \
    python -u tools/attn_bench.py --nocheck 5 --only 128 | grep dkdv || exit 1
done
done
