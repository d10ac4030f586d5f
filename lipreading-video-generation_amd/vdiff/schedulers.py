"""DDPM schedulers with the reference API (linear_noise_scheduler.py, noise_scheduler.py)
plus a DDIM sampler, all running on the HIP scheduler kernels.

The schedule tables are built on the host exactly as the reference builds them (same
torch CPU ops, so they are bit-identical and keep the reference attribute names);
the per-step math runs on the GPU with per-sample timesteps.  Noise `z` may be
injected (tests) or is drawn with torch.randn_like on the tensor's device.
"""
from __future__ import annotations

import math

import torch

from . import ops


class _Tables:
    _dev_cache: dict

    def _dev(self, name, device):
        key = (name, str(device))
        cache = self.__dict__.setdefault("_dev_cache", {})
        if key not in cache:
            cache[key] = getattr(self, name).to(device=device, dtype=torch.float32).contiguous()
        return cache[key]


class LinearNoiseScheduler(_Tables):
    """linear_noise_scheduler.py:6-76 (DDPM, standard posterior variance)."""

    def __init__(self, num_timesteps, beta_start, beta_end):
        self.num_timesteps = num_timesteps
        self.beta_start = beta_start
        self.beta_end = beta_end
        self.betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, num_timesteps) ** 2
        self.alphas = 1. - self.betas
        self.alpha_cum_prod = torch.cumprod(self.alphas, dim=0)
        self.sqrt_alpha_cum_prod = torch.sqrt(self.alpha_cum_prod)
        self.sqrt_one_minus_alpha_cum_prod = torch.sqrt(1 - self.alpha_cum_prod)

    def add_noise(self, original, noise, t):
        """q_sample (linear_noise_scheduler.py:24-46)."""
        d = original.device
        return ops.q_sample(original.contiguous(), noise.contiguous(), t,
                            self._dev("sqrt_alpha_cum_prod", d),
                            self._dev("sqrt_one_minus_alpha_cum_prod", d))

    def sample_prev_timestep(self, xt, noise_pred, t, z=None):
        """p_sample (linear_noise_scheduler.py:48-76); per-sample t, no noise where t == 0."""
        d = xt.device
        xt = xt.contiguous()
        if z is None:
            z = torch.randn_like(xt)
        return ops.p_sample_v1(xt, noise_pred.contiguous().to(xt.dtype), z.contiguous(), t,
                               self._dev("betas", d), self._dev("alphas", d),
                               self._dev("alpha_cum_prod", d),
                               self._dev("sqrt_one_minus_alpha_cum_prod", d))


class LinearNoiseSchedulerV2(LinearNoiseScheduler):
    """linear_noise_scheduler.py:79-101: the sampling schedule used by test.py; keeps the
    reference's non-standard mean xt - sqrt(1-acp) eps / sqrt(alpha) and adds noise at
    every step (also t == 0)."""

    def __init__(self, num_timesteps, beta_start=0.0001, beta_end=0.01):
        super().__init__(num_timesteps, beta_start, beta_end)

    def sample_prev_timestep(self, xt, noise_pred, t, z=None):
        d = xt.device
        xt = xt.contiguous()
        if z is None:
            z = torch.randn_like(xt)
        return ops.p_sample_v2(xt, noise_pred.contiguous().to(xt.dtype), z.contiguous(), t,
                               self._dev("betas", d), self._dev("alphas", d),
                               self._dev("alpha_cum_prod", d), self._dev("sqrt_alpha_cum_prod", d),
                               self._dev("sqrt_one_minus_alpha_cum_prod", d))


class CosineNoiseScheduler(_Tables):
    """noise_scheduler.py:4-29; returns (sampled, mean)."""

    def __init__(self, num_timesteps, s=0.008):
        self.num_timesteps = num_timesteps
        self.s = s
        self.timesteps = torch.arange(num_timesteps, dtype=torch.float32) / num_timesteps
        self.alphas_cumprod = torch.cos(((self.timesteps + self.s) / (1 + self.s)) * math.pi * 0.5) ** 2
        self.sqrt_alphas_cumprod = torch.sqrt(self.alphas_cumprod)
        self.sqrt_one_minus_alphas_cumprod = torch.sqrt(1 - self.alphas_cumprod)

    def sample_prev_timestep(self, xt, noise_pred, t, z=None):
        d = xt.device
        xt = xt.contiguous()
        if z is None:
            z = torch.randn_like(xt)
        return ops.p_sample_cosine(xt, noise_pred.contiguous().to(xt.dtype), z.contiguous(), t,
                                   self._dev("alphas_cumprod", d),
                                   self._dev("sqrt_alphas_cumprod", d),
                                   self._dev("sqrt_one_minus_alphas_cumprod", d))


class DDIMSampler:
    """DDIM (eta = 0: deterministic) over a subsequence of a DDPM schedule's acp table
    (build extension: the reference samples with 500-step DDPM V2, test.py:111).

    steps: number of denoising steps; timesteps = linspace(T-1, 0, steps) rounded.
    """

    def __init__(self, scheduler, steps=50, eta=0.0, clip_x0=False):
        acp = getattr(scheduler, "alpha_cum_prod", None)
        if acp is None:
            acp = scheduler.alphas_cumprod
        self.acp = acp.float()
        self.num_train_timesteps = acp.numel()
        self.steps = steps
        self.eta = eta
        self.clip_x0 = clip_x0
        ts = torch.linspace(self.num_train_timesteps - 1, 0, steps).round().long()
        self.timesteps = ts
        self.prev_timesteps = torch.cat([ts[1:], torch.tensor([-1])])
        self._acp_dev = {}

    def _acp(self, device):
        k = str(device)
        if k not in self._acp_dev:
            self._acp_dev[k] = self.acp.to(device).contiguous()
        return self._acp_dev[k]

    def step(self, xt, noise_pred, i, z=None):
        """One update from self.timesteps[i] to self.prev_timesteps[i]: (x_prev, x0)."""
        B = xt.shape[0]
        t = torch.full((B,), int(self.timesteps[i]), dtype=torch.int64, device=xt.device)
        tp = torch.full((B,), int(self.prev_timesteps[i]), dtype=torch.int64, device=xt.device)
        if self.eta > 0 and z is None:
            z = torch.randn_like(xt)
        return ops.ddim_step(xt.contiguous(), noise_pred.contiguous().to(xt.dtype), t, tp,
                             self._acp(xt.device), eta=self.eta, z=z, clip=self.clip_x0)
