#!/bin/bash
# Round-5 batch i: localise the ViViT graph-vs-eager weight difference.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/vivit_graph_diff.py > gpurun_out/r05i_vivit_diff.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r05i_vivit_diff.txt | cut -c1-600; exit $rc
