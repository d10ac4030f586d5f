#!/bin/bash
# Round-4 GPU batch ab: HIP API trace of the config-2 train step (where does the host wait?):
# synchronising API calls per step and their durations.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -rf /tmp/prof_hip
timeout -k 10 500 rocprofv3 --hip-trace --kernel-trace -d /tmp/prof_hip -o run -- \
  python3 bench.py --only train --steps 3 --warmup 1 --no-cpu --xattn-steps 0 \
  > gpurun_out/r04ab_train.json 2> gpurun_out/r04ab_train.err || { tail gpurun_out/r04ab_train.err; exit 1; }
db=$(find /tmp/prof_hip -name '*.db' | head -n 1)
timeout -k 10 120 python3 tools/host_waits.py "$db" > gpurun_out/r04ab_host_waits.txt 2>&1 && timeout -k 10 120 python3 tools/host_waits.py "$db" --lead 2 >> gpurun_out/r04ab_host_waits.txt 2>&1
rc=$?; tail -45 gpurun_out/r04ab_host_waits.txt; exit $rc
