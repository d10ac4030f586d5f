#!/bin/bash
# Round-3 GPU batch l: GPU idle time inside the config-2 train step (what a HIP-graph replay
# of the step could recover at most) -- kernel trace of tools/step_gap.py without the
# per-launch events, summarised by tools/idle_gaps.py.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03l}
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_trace \
  -o run -- python3 -u tools/step_gap.py --no-timer --steps 4 --rounds 1 --lr 1e-3 \
  > gpurun_out/${T}_step_gap.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/${T}_step_gap.txt | tail -3
python3 tools/idle_gaps.py "gpurun_out/${T}_trace/**/*kernel_trace.csv" --top 20 --steps 4 \
  > gpurun_out/${T}_idle.txt 2>&1; rc=$?
cat gpurun_out/${T}_idle.txt
find gpurun_out/${T}_trace -name '*.csv' -size +20M -delete
exit $rc
