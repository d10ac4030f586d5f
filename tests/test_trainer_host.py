"""Trainer host logic on CPU with stand-in model / scheduler (plain torch, no kernels): the
loss finiteness record is kept on the device and read only every check_every steps or by
check_finite(), and it names the first bad step (SURVEY 5 failure detection)."""
import pytest
import torch

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
    tr = Trainer(_Model({3, 5}), _Sched(), lr=1e-3, check_every=4)
    c = _clip()
    for _ in range(3):
        tr.step(c)
    with pytest.raises(FloatingPointError, match="step 3 "):
        tr.step(c)  # the 4th step reads the record


def test_check_finite_between_reads_and_disabled():
    tr = Trainer(_Model({1}), _Sched(), lr=1e-3, check_every=100)
    c = _clip()
    tr.step(c)
    tr.check_finite()  # finite so far
    tr.step(c)         # NaN at step 1: not read yet (no host sync per step)
    with pytest.raises(FloatingPointError, match="step 1 "):
        tr.check_finite()
    off = Trainer(_Model({0}), _Sched(), lr=1e-3, check_every=0)
    off.step(c)
    off.check_finite()
