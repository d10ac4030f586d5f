#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/asm_rare_count.py 65536 1.3 > gpurun_out/rare.txt 2>&1
rc=$?; cat gpurun_out/rare.txt | tail -8; exit $rc
