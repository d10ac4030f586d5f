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
