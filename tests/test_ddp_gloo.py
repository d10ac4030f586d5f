"""Data-parallel gradient averaging (vdiff.ddp.GradBucketer) with world_size 2 over gloo on
CPU: the bucketed, hook-launched all-reduce gives the same gradients as one process on the
concatenated batch (GroupNorm is per-sample, so DP is exact for the denoiser too)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG  # noqa: F401  (puts vdiff on sys.path)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(16, 64), torch.nn.GroupNorm(8, 64),
                               torch.nn.SiLU(), torch.nn.Linear(64, 64), torch.nn.SiLU(),
                               torch.nn.Linear(64, 4))


def _data():
    g = torch.Generator().manual_seed(1)
    return torch.randn(8, 16, generator=g), torch.randn(8, 4, generator=g)


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from vdiff.ddp import GradBucketer, broadcast_parameters, init_from_env
    init_from_env("gloo")
    m = _model()
    broadcast_parameters(m)
    bk = GradBucketer(list(m.parameters()), bucket_mb=0.01)  # several buckets
    x, y = _data()
    n = x.shape[0] // world
    for step in range(2):  # twice: the buckets re-arm after zero_grad
        loss = torch.nn.functional.mse_loss(m(x[rank * n:(rank + 1) * n]),
                                            y[rank * n:(rank + 1) * n])
        loss.backward()
        bk.finish()
        if step == 0:
            bk.zero_grad()
    if rank == 0:
        out.put([p.grad.clone() for p in m.parameters()] + [torch.tensor(len(bk.buckets))])
    dist.barrier()
    dist.destroy_process_group()


def test_bucketed_allreduce_matches_single_process():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    nb = int(got.pop())
    assert nb >= 2
    m = _model()
    x, y = _data()
    torch.nn.functional.mse_loss(m(x), y).backward()
    for g, p in zip(got, m.parameters()):
        torch.testing.assert_close(g, p.grad, atol=1e-6, rtol=1e-5)


class _Skippy(torch.nn.Module):
    """A trunk with blocks a rank may skip (as wav2vec2's LayerDrop does in train mode)."""

    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.inp = torch.nn.Linear(16, 32)
        self.blocks = torch.nn.ModuleList(torch.nn.Linear(32, 32) for _ in range(3))
        self.out = torch.nn.Linear(32, 4)

    def forward(self, x, skip):
        h = torch.tanh(self.inp(x))
        for i, b in enumerate(self.blocks):
            if i not in skip:
                h = h + torch.tanh(b(h))
        return self.out(h)


_SKIPS = {0: (1,), 1: ()}  # rank 0 drops block 1: its bucket completes on rank 1 only


def _skippy_loss(m, rank, world):
    x, y = _data()
    n = x.shape[0] // world
    return torch.nn.functional.mse_loss(m(x[rank * n:(rank + 1) * n], _SKIPS[rank]),
                                        y[rank * n:(rank + 1) * n])


def _skip_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from vdiff.ddp import GradBucketer, init_from_env
    init_from_env("gloo")
    m = _Skippy()
    bk = GradBucketer(list(m.parameters()), bucket_mb=0.003)  # one bucket per layer or less
    for step in range(2):
        _skippy_loss(m, rank, world).backward()
        bk.finish()
        if step == 0:
            bk.zero_grad()
    if rank == 0:
        out.put([p.grad.clone() for p in m.parameters()] + [torch.tensor(len(bk.buckets))])
    dist.barrier()
    dist.destroy_process_group()


def test_bucket_order_survives_rank_dependent_unused_params():
    """Rank-dependent unused parameters must not reorder the collectives: buckets launch in
    bucket order on every rank, and a skipped parameter contributes zeros to the average."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_skip_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert int(got.pop()) >= 4
    grads = []
    for r in range(world):
        m = _Skippy()
        _skippy_loss(m, r, world).backward()
        grads.append([p.grad if p.grad is not None else torch.zeros_like(p)
                      for p in m.parameters()])
    for i, g in enumerate(got):
        torch.testing.assert_close(g, sum(gr[i] for gr in grads) / world, atol=1e-6, rtol=1e-5)


def _global_skip_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from vdiff.ddp import GradBucketer, init_from_env
    init_from_env("gloo")
    m = _Skippy()
    bk = GradBucketer(list(m.parameters()), bucket_mb=0.003)
    skips = {0: (1, 2), 1: (2,)}  # block 2 unused on every rank, block 1 on rank 0 only
    x, y = _data()
    n = x.shape[0] // world
    state = []
    for step in range(2):
        loss = torch.nn.functional.mse_loss(m(x[rank * n:(rank + 1) * n], skips[rank]),
                                            y[rank * n:(rank + 1) * n])
        loss.backward()
        bk.finish()
        state.append([p.grad is None for p in m.parameters()])
        bk.zero_grad()
    if rank == 0:
        out.put(state + [[p.grad is None for p in m.parameters()]])
    dist.barrier()
    dist.destroy_process_group()


def test_globally_unused_params_get_no_grad():
    """A parameter no rank produced a gradient for gets .grad = None for the optimizer step
    (as in one process: AdamW's weight decay must not touch it); zero_grad() re-arms the
    bucket views.  A parameter unused on one rank only keeps its (averaged) gradient."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_global_skip_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    names = [n for n, _ in _Skippy().named_parameters()]
    for step_state in got[:2]:
        none = {n for n, is_none in zip(names, step_state) if is_none}
        assert none == {"blocks.2.weight", "blocks.2.bias"}, none
    assert not any(got[2])  # after zero_grad every parameter has its bucket view again
