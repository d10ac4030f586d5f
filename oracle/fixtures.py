"""Seeded synthetic tensors shared by the golden generator, the tests and bench.py's
CPU baseline (so large inputs never need to be committed)."""
from __future__ import annotations

import torch


def seeded(shape, seed: int, dist: str = "normal") -> torch.Tensor:
    """CPU fp32 tensor from its own torch.Generator (deterministic for a torch version)."""
    g = torch.Generator().manual_seed(int(seed))
    if dist == "normal":
        return torch.randn(tuple(shape), generator=g)
    if dist == "uniform":  # U[-1, 1): the Normalize(0.5, 0.5) image range (train.py:70-75)
        return torch.rand(tuple(shape), generator=g) * 2 - 1
    raise ValueError(dist)


def seeded_timesteps(n: int, num_timesteps: int, seed: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(int(seed))
    return torch.randint(0, num_timesteps, (n,), generator=g)


def rel_l2(a: torch.Tensor, b: torch.Tensor) -> float:
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


# Model configurations used by the fixtures (also the bench's CPU baseline sample).
TINY3D = dict(in_channels=35, model_channels=32, out_channels=3, num_res_blocks=1,
              attention_resolutions=(2,), channel_mult=(1, 2), dims=3)
TINY3D_SHAPE = (1, 35, 8, 64, 64)

FULL2D = dict(in_channels=195, model_channels=64, out_channels=3, num_res_blocks=2,
              attention_resolutions=(1, 2, 4), channel_mult=(1, 2, 4), dims=2)
FULL2D_SHAPE = (2, 195, 32, 32)

# train.py:88-97 / BASELINE config 2: the full-width 3-D model
FULL3D = dict(in_channels=195, model_channels=64, out_channels=3, num_res_blocks=2,
              attention_resolutions=(1, 2, 4), channel_mult=(1, 2, 4), dims=3)


def train_step_inputs(T=8, S=64):
    """Seeded inputs of the one-train-step fixture (tests/golden/train_step_tiny3d.npz):
    x0, cond image, pooled audio features [T, 64], eps."""
    return (seeded((1, 3, T, S, S), 70, "uniform"), seeded((1, 3, 32, 32), 71, "uniform"),
            seeded((T, 64), 72), seeded((1, 3, T, S, S), 73))


TRAIN5_T = (37, 5, 80, 62, 19)  # injected timesteps of the five-step fixture (train.py:125)


def train5_inputs(k, T=8, S=64):
    """Seeded inputs of step k of the five-step fixture (tests/golden/train_steps5_tiny3d.npz):
    x0, cond image, pooled audio features [T, 64], eps."""
    return (seeded((1, 3, T, S, S), 500 + 10 * k, "uniform"),
            seeded((1, 3, 32, 32), 501 + 10 * k, "uniform"),
            seeded((T, 64), 502 + 10 * k), seeded((1, 3, T, S, S), 503 + 10 * k))


def adam_delta_close(delta, delta_ref, grad_ref, lr=1e-2):
    """One Adam step from zero state moves each parameter by -lr * g / (|g| + 1e-8), i.e.
    ~ -lr * sign(g): compare where that is insensitive to the gradient's own rounding
    (|g| above 1e-2 of its RMS: d(delta)/dg = lr * 1e-8 / (|g| + 1e-8)^2 is then <~ 1, so a
    fp32-level gradient difference moves delta by as little), bound the rest by lr.
    Returns the max abs deviation on the mask."""
    delta, delta_ref, grad_ref = (u.detach().double().cpu() for u in (delta, delta_ref, grad_ref))
    mask = grad_ref.abs() > 1e-2 * grad_ref.pow(2).mean().sqrt()
    assert mask.float().mean() > 0.9
    assert float(delta.abs().max()) <= lr * (1 + 1e-5)
    return float((delta - delta_ref)[mask].abs().max())
