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
    # the gradient hooks hold the bucketer weakly: dropping it frees it (and its pinned flag
    # buffer) at once, without the cyclic collector
    import gc
    import weakref
    nb, ref = len(bk.buckets), weakref.ref(bk)
    gc.disable()
    del bk
    freed = ref() is None
    gc.enable()
    if rank == 0:
        # numpy arrays travel by value: a tensor would travel as a shared-memory fd whose
        # sharer thread dies with this process, racing the parent's get()
        out.put([p.grad.detach().numpy().copy() for p in m.parameters()] + [freed, nb])
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
    freed, nb = got[-2], int(got[-1])
    got = [torch.from_numpy(a) for a in got[:-2]]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert nb >= 2
    assert freed, "GradBucketer was kept alive by a reference cycle"
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
    # the gradient hooks hold the bucketer weakly: dropping it frees it (and its pinned flag
    # buffer) at once, without the cyclic collector
    import gc
    import weakref
    nb, ref = len(bk.buckets), weakref.ref(bk)
    gc.disable()
    del bk
    freed = ref() is None
    gc.enable()
    if rank == 0:
        # numpy arrays travel by value: a tensor would travel as a shared-memory fd whose
        # sharer thread dies with this process, racing the parent's get()
        out.put([p.grad.detach().numpy().copy() for p in m.parameters()] + [freed, nb])
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
    freed, nb = got[-2], int(got[-1])
    got = [torch.from_numpy(a) for a in got[:-2]]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert nb >= 4 and freed
    grads = []
    for r in range(world):
        m = _Skippy()
        _skippy_loss(m, r, world).backward()
        grads.append([p.grad if p.grad is not None else torch.zeros_like(p)
                      for p in m.parameters()])
    for i, g in enumerate(got):
        torch.testing.assert_close(g, sum(gr[i] for gr in grads) / world, atol=1e-6, rtol=1e-5)


_GSKIPS = {0: (1, 2), 1: (2,)}  # block 2 unused on every rank, block 1 on rank 0 only


def _global_skip_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from vdiff.ddp import GradBucketer, init_from_env
    init_from_env("gloo")
    m = _Skippy()
    bk = GradBucketer(list(m.parameters()), bucket_mb=0.003)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-2, weight_decay=0.1)
    x, y = _data()
    n = x.shape[0] // world
    unused = []
    for step in range(3):
        loss = torch.nn.functional.mse_loss(m(x[rank * n:(rank + 1) * n], _GSKIPS[rank]),
                                            y[rank * n:(rank + 1) * n])
        loss.backward()
        bk.finish()
        names = {id(p): k for k, p in m.named_parameters()}
        unused.append(sorted(names[id(bk.views[i][0])] for i in bk.globally_unused()))
        bk.step(opt)
        bk.zero_grad()
    if rank == 0:
        out.put({"params": [p.detach().numpy().copy() for p in m.parameters()],
                 "unused": unused,
                 "grads_are_views": all(p.grad is not None for p in m.parameters())})
    dist.barrier()
    dist.destroy_process_group()


def test_globally_unused_params_keep_weights_and_state():
    """A parameter no rank produced a gradient for is left alone by the optimizer step (as
    with .grad = None in one process: AdamW's weight decay and moments must not touch it),
    decided on the device from the used-flags carried by the last bucket -- no host sync.
    A parameter unused on one rank only is updated with its averaged gradient.  The result
    equals a single process that averages the ranks' gradients by hand."""
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
    assert got["unused"] == [["blocks.2.bias", "blocks.2.weight"]] * 3
    assert got["grads_are_views"]
    m = _Skippy()
    init = {k: v.detach().clone() for k, v in m.named_parameters()}
    opt = torch.optim.AdamW(m.parameters(), lr=1e-2, weight_decay=0.1)
    x, y = _data()
    n = x.shape[0] // world
    for _ in range(3):
        per_rank = []
        for r in range(world):
            m.zero_grad(set_to_none=True)
            torch.nn.functional.mse_loss(m(x[r * n:(r + 1) * n], _GSKIPS[r]),
                                         y[r * n:(r + 1) * n]).backward()
            per_rank.append([None if p.grad is None else p.grad.clone() for p in m.parameters()])
        for i, p in enumerate(m.parameters()):
            gs = [g[i] for g in per_rank]
            p.grad = (None if all(g is None for g in gs) else
                      sum(g if g is not None else torch.zeros_like(p) for g in gs) / world)
        opt.step()
    for (name, p), g in zip(m.named_parameters(), got["params"]):
        g = torch.from_numpy(g)
        torch.testing.assert_close(g, p.detach(), atol=1e-6, rtol=1e-5)
        if name.startswith("blocks.2."):
            torch.testing.assert_close(g, init[name], atol=0, rtol=0)
