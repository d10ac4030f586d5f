#!/bin/bash
# Round-5 batch p: the driver's bench command after the clip bank and the tiled weight pack.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05p
timeout -k 10 900 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json \
  2> gpurun_out/${T}_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
grep -E "train:|ddim|spatial_temporal:|vivit:|xattn" gpurun_out/${T}_bench.err | cut -c1-200
