"""SURVEY 8e parity test on the real model, on the one GPU of the box: two processes train
the tiny audio-conditioned UNet3D (fp32 parity mode) on disjoint halves of a 2-clip batch,
with gradients averaged by vdiff.ddp.GradBucketer over gloo (tests/_ddp_worker.py).  The
averaged gradients must equal one process's gradients on the concatenated batch (rel-L2
<= 1e-5; GroupNorm is per-sample, so data parallelism is exact), and every bucket's
all-reduce must have been launched from the gradient hooks before backward() returned
(overlap with the backward).  RCCL itself is exercised by the driver's multi-GPU bench."""
import os
import socket
import subprocess
import sys

import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _two_ranks(out):
    port = _port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), VDIFF_DIST_BACKEND="gloo")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "_ddp_worker.py"),
                                       out], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    logs = [p.communicate(timeout=240)[0] for p in procs]
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-3000:]
    return [torch.load(f"{out}.rank{r}.pt", weights_only=True) for r in range(2)]


def test_two_rank_gradients_match_single_process(tmp_path):
    """Since round 4 every reduction of the step is fixed-order: the
    averaged gradients are bit-identical on both ranks AND across two launches of the
    2-rank job; against one process on the whole batch they agree to fp32 summation order
    (the pixel splits of the batched kernels straddle the two clips, so the sums are
    associated differently: rel-L2 <= 1e-5)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _ddp_worker as w
    res = _two_ranks(str(tmp_path / "ddp"))
    again = _two_ranks(str(tmp_path / "ddp2"))
    for name in res[0]["grads"]:
        assert torch.equal(res[0]["grads"][name], res[1]["grads"][name]), name
        assert torch.equal(res[0]["grads"][name], again[0]["grads"][name]), name
    # single process, whole batch
    dev = torch.device("cuda", 0)
    from vdiff.schedulers import LinearNoiseScheduler
    m = w.build(dev)
    w.loss_of(m, LinearNoiseScheduler(100, 0.00085, 0.012), *w.batch(dev)).backward()
    for r in res:
        assert r["buckets"] >= 3
        assert r["launched_in_backward"] == r["buckets"]
    for name, p in m.named_parameters():
        ref = p.grad.detach().cpu().double()
        for r in res:
            g = r["grads"][name].double()
            err = float((g - ref).norm() / ref.norm().clamp_min(1e-30))
            assert err <= 1e-5, (name, err)
