#!/bin/bash
# Round-4 GPU batch ac: GroupNorm launch shape (VDIFF_GN_CHUNKS workgroups per launch,
# VDIFF_GN_SUMPER chunk partials per backward-sum workgroup) A/B, then the GN tests.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r04ac}
run() {
  env $2 timeout -k 10 120 python3 -u tools/gn_bench.py --capi > gpurun_out/${T}_$1.log 2>&1
  rc=$?; echo "== $1 ($2)"; grep -v amdgpu.ids gpurun_out/${T}_$1.log
  [ $rc -eq 0 ] || { echo "rc=$rc: stopping"; exit $rc; }
}
run base VDIFF_X=0
run c1024 VDIFF_GN_CHUNKS=1024
run c512 VDIFF_GN_CHUNKS=512
run s256 VDIFF_GN_SUMPER=256
run c1024s256 "VDIFF_GN_CHUNKS=1024 VDIFF_GN_SUMPER=256"
run c512s256 "VDIFF_GN_CHUNKS=512 VDIFF_GN_SUMPER=256"
run base2 VDIFF_X=0
timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_groupnorm.py > gpurun_out/${T}_gn_tests.log 2>&1
rc=$?; tail -1 gpurun_out/${T}_gn_tests.log; exit $rc
