cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
VDIFF_DIST_BACKEND=gloo timeout -k 10 700 python -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 \
  --steps 2 --warmup 1 --c4-steps 1 --vivit-steps 3 --xattn-steps 1 --no-cpu > gpurun_out/ddp_rehearsal_all.json 2> gpurun_out/ddp_rehearsal_all.err
rc=$?; tail -c 1500 gpurun_out/ddp_rehearsal_all.json; tail -5 gpurun_out/ddp_rehearsal_all.err; exit $rc
