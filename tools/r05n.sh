#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -q --timeout 200 -p no:cacheprovider tests/test_gpu_elementwise.py -k pack > gpurun_out/r05n_tests.txt 2>&1 || { tail -20 gpurun_out/r05n_tests.txt; exit 1; }
tail -1 gpurun_out/r05n_tests.txt
timeout -k 10 300 python3 -u tools/pack_probe.py --no-cpu > gpurun_out/r05n_pack.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r05n_pack.txt | tail -8; exit $rc
