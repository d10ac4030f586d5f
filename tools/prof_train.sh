#!/bin/bash
# rocprofv3 kernel summary of the timed config-2 train step alone (bench --only train);
# extra arguments go to bench.py (e.g. --mode spatial_temporal).  Output tag: $TAG (default train).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-train}
rm -rf /tmp/prof_$TAG
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o run -- \
  python bench.py --only train --steps 4 --warmup 1 --no-cpu --xattn-steps 0 --st-steps 0 "$@" \
  > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.err || { tail gpurun_out/prof_$TAG.err; exit 1; }
db=$(find /tmp/prof_$TAG -name '*.db' | head -n 1)
python tools/prof_summary.py "$db" > gpurun_out/${TAG}_kernel_stats.md
python tools/prof_steps.py "$db" | tee gpurun_out/${TAG}_steps.txt
