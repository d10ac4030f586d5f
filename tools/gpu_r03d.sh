#!/bin/bash
# Round-3 GPU batch d: forward row sums on the matrix pipe (gen_fwd MSUM) A/B, 1x1 weight-
# gradient variants (VDIFF_WGRAD1), train.py --data vs synthetic, the GPU suite on the new
# defaults.   bash tools/gpu_r03d.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03d}
ok() { case $1 in 0|1) return 0 ;; *) echo "stopping: rc $1"; exit $1 ;; esac; }
timeout -k 10 300 python -u tools/asm_ab.py 'base:' 'msum:MSUM=1' 'msum_st:MSUM=1,STAMP=1' \
  'base_st:STAMP=1' 'base2:' 'msum2:MSUM=1' > gpurun_out/${T}_msum.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/${T}_msum.txt | tail -8; ok $rc
for v in 2,64 4,64 6,64 2,128 4,128 2,192 4,192 2,64; do
  VDIFF_WGRAD1=$v timeout -k 10 120 python -u tools/wgrad1x1_bench.py \
    >> gpurun_out/${T}_wgrad1x1.txt 2>&1; rc=$?; ok $rc
  grep "per train step" gpurun_out/${T}_wgrad1x1.txt | tail -1
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${T}_gpu_tests.log; ok $rc
timeout -k 10 600 python -u tools/data_vs_synth.py > gpurun_out/${T}_data_vs_synth.json \
  2> gpurun_out/${T}_data_vs_synth.err; rc=$?
tail -c 600 gpurun_out/${T}_data_vs_synth.json; tail -3 gpurun_out/${T}_data_vs_synth.err; ok $rc
