#!/bin/bash
# Round-5 batch s: packed-f32 softmax VALU (v_pk_add_f32 row sums in the forwards,
# v_pk_mul_f32 P * dP in the backwards) -- parity of the product build, then A/B against the
# knob-off build (libvdiff_pk0.so) interleaved on one box; the 1x1 conv kernel with whole
# 64-B store segments against the previous mapping (libvdiff_pwold.so).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -q --timeout 300 -p no:cacheprovider \
  tests/test_gpu_attention.py tests/test_gpu_attention_asm.py tests/test_gpu_attention_asm128.py \
  tests/test_gpu_conv.py \
  > gpurun_out/r05s_tests.txt 2>&1 || { tail -30 gpurun_out/r05s_tests.txt; exit 1; }
tail -1 gpurun_out/r05s_tests.txt
for lib in libvdiff_pwold libvdiff libvdiff_pwold libvdiff; do
  echo "== $lib" >> gpurun_out/r05s_pw_ab.txt
  VDIFF_LIB=lipreading-video-generation_amd/vdiff/$lib.so timeout -k 10 120 python3 -u \
    tools/conv1x1_bench.py >> gpurun_out/r05s_pw_ab.txt 2>&1 || { tail -5 gpurun_out/r05s_pw_ab.txt; exit 1; }
done
grep -E "^==|->" gpurun_out/r05s_pw_ab.txt
timeout -k 10 200 python3 -u tools/asm_ab.py 'pk0:PKSUM=0,STAMP=1' 'pk1:PKSUM=1,STAMP=1' \
  'pk0:PKSUM=0' 'pk1:PKSUM=1' 'pk0:PKSUM=0' 'pk1:PKSUM=1' > gpurun_out/r05s_fwd_ab.txt 2>&1 \
  || { tail -5 gpurun_out/r05s_fwd_ab.txt; exit 1; }
cat gpurun_out/r05s_fwd_ab.txt
for d in 64 128; do
  timeout -k 10 500 bash tools/attn_ab.sh "libvdiff_pk0 libvdiff libvdiff_pk0 libvdiff" auto $d \
    > gpurun_out/r05s_ab_d$d.txt 2>&1 || { tail -5 gpurun_out/r05s_ab_d$d.txt; exit 1; }
  grep -E "^==|attn_" gpurun_out/r05s_ab_d$d.txt
done
