"""bench.py --gpus N starts its N ranks itself: no external launcher, the
JSON line reports n_gpus = N and the process-group size the ranks saw, and the gradient
exchange report (exposed / standalone all-reduce time).  On the one-GPU box the ranks share
the card over gloo (VDIFF_DIST_BACKEND=gloo); the driver's multi-GPU run uses RCCL.
Small shapes (32x32x4 clip) keep it to seconds; the ViViT leg runs its DDP graph path."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _run(extra, timeout=300):
    env = dict(os.environ, VDIFF_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--no-cpu"] + extra
    p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=timeout)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]  # rank 0 prints one line
    return json.loads(lines[0]), p.stderr


def test_bench_spawns_two_ranks_train():
    r, err = _run(["--only", "train", "--steps", "2", "--warmup", "1", "--size", "32",
                   "--frames", "4", "--xattn-steps", "0", "--vivit-steps", "0"])
    assert "spawning 2 ranks" in err
    assert r["n_gpus"] == 2
    assert r["config"]["parallelism"] == "dp2"
    ar = r["allreduce"]
    assert ar["world_size"] == 2 and ar["backend"] == "gloo"
    assert ar["steps"] == 2 and ar["standalone_ms_per_step"] > 0
    assert ar["grad_mbytes"] > 500  # UNet3D + wav2vec2-base fp32 gradients (+ flags)
    assert r["value"] > 0
    st = r["spatial_temporal"]  # the auxiliary leg over both ranks (short temporal kernels)
    assert st.get("error") is None and st["value"] > 0, st
    assert st["roofline_temporal"]["achieved"] > 0


def test_bench_spawns_two_ranks_vivit_ddp():
    """N > 1 ViViT: eager with the bucketed all-reduce by default (advisor r03: the graph
    form has not run over RCCL yet), graph replays around one all-reduce with
    --vivit-graph-ddp."""
    r, _ = _run(["--only", "vivit", "--vivit-steps", "3", "--vivit-batch", "4"])
    v = r["vivit"]
    assert v.get("error") is None, v
    assert v["hip_graph"] is False and v["parallelism"] == "dp2"
    r, _ = _run(["--only", "vivit", "--vivit-steps", "3", "--vivit-batch", "4",
                 "--vivit-graph-ddp"])
    v = r["vivit"]
    assert v.get("error") is None, v
    assert v["hip_graph"] is True and v["parallelism"] == "dp2"


def test_bench_rejects_mismatched_world():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--no-cpu", "--only", "train"], env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=300)
    assert p.returncode == 2
    assert "WORLD_SIZE 1" in p.stderr
