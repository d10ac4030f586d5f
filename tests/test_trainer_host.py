"""Trainer host logic on CPU with stand-in model / scheduler (plain torch, no kernels): the
loss finiteness record is kept on the device and read only every check_every steps or by
check_finite(), and it names the first bad step (SURVEY 5 failure detection)."""
import pytest
import torch
import torch.nn.functional as F

from vdiff.engine import Clip, Trainer


class _Sched:
    def add_noise(self, x0, eps, t):
        return x0 + eps


class _Model(torch.nn.Module):
    def __init__(self, bad_calls):
        super().__init__()
        self.lin = torch.nn.Linear(4, 4)
        self.calls, self.bad = 0, set(bad_calls)

    def forward(self, xt, cond, audio, t):
        y = self.lin(xt)
        self.calls += 1
        return y * float("nan") if self.calls - 1 in self.bad else y


def _clip():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 4, generator=g)
    return Clip(x, x, {}, torch.randn(2, 4, generator=g), torch.zeros(2, dtype=torch.int64))


def test_nonfinite_loss_raises_with_first_step():
    tr = Trainer(_Model({3, 5}), _Sched(), lr=1e-3, loss_fn=F.mse_loss, check_every=4)
    c = _clip()
    for _ in range(3):
        tr.step(c)
    with pytest.raises(FloatingPointError, match="step 3 "):
        tr.step(c)  # the 4th step reads the record


def test_check_finite_between_reads_and_disabled():
    tr = Trainer(_Model({1}), _Sched(), lr=1e-3, loss_fn=F.mse_loss, check_every=100)
    c = _clip()
    tr.step(c)
    tr.check_finite()  # finite so far
    tr.step(c)         # NaN at step 1: not read yet (no host sync per step)
    with pytest.raises(FloatingPointError, match="step 1 "):
        tr.check_finite()
    off = Trainer(_Model({0}), _Sched(), lr=1e-3, loss_fn=F.mse_loss, check_every=0)
    off.step(c)
    off.check_finite()


def _ddp_worker(rank, world, port, q):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from vdiff.ddp import broadcast_parameters, init_from_env
    init_from_env("gloo")
    torch.manual_seed(0)
    m = _Model({2} if rank == 1 else set())  # rank 1 alone goes non-finite at step 2
    broadcast_parameters(m)
    tr = Trainer(m, _Sched(), lr=1e-3, loss_fn=F.mse_loss, check_every=4)
    c = _clip()
    res = "no raise"
    try:
        for _ in range(6):
            tr.step(c)
    except FloatingPointError as e:
        res = f"raised after {tr.steps_done} steps: {e}"
    q.put((rank, res))
    torch.distributed.destroy_process_group()


def test_ddp_nonfinite_loss_raises_on_every_rank():
    """Advisor r03: a loss that goes non-finite on ONE rank makes every rank raise at the same
    read (the first bad step is MIN-all-reduced), so no rank is left waiting in the next
    gradient all-reduce.  world_size 2 over gloo."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for r in (0, 1):
        assert got[r].startswith("raised after 4 steps") and "step 2 " in got[r], got


def test_graph_trainer_is_gated(monkeypatch):
    """Advisor r03: Trainer(graph=True) stays opt-in (it measured no gain over the eager step,
    DESIGN section 9 item 3): it raises unless VDIFF_TRAIN_GRAPH_EXPERIMENTAL=1."""
    monkeypatch.delenv("VDIFF_TRAIN_GRAPH_EXPERIMENTAL", raising=False)
    with pytest.raises(RuntimeError, match="VDIFF_TRAIN_GRAPH_EXPERIMENTAL"):
        Trainer(_Model(set()), _Sched(), lr=1e-3, graph=True)
