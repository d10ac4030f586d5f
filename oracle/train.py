"""Oracle restatement of one training step (TEST INFRASTRUCTURE ONLY -- never imported by
the product path): train.py:122-134 -- q_sample (linear_noise_scheduler.py:24-46),
UNetAudio conditioning (unet_audio.py:52-61, oracle.unet.audio_conditioned_input),
UNetModel.forward, MSELoss, backward, torch.optim.Adam(lr=1e-2) step (train.py:102-103).
CPU, fp32."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import schedulers as osch
from .unet import audio_conditioned_input, unet_forward


def train_step(P: dict, plan, x0, cond, feat, eps, t, projected_audio_dim, lr=1e-2,
               schedule=(100, 0.00085, 0.012)):
    """One Adam step on the parameter dict P (modified in place).

    Returns (loss, grads, deltas) with grads / deltas keyed like P."""
    tab = osch.linear_tables(*schedule)
    params = {k: v.detach().clone().requires_grad_(True) for k, v in P.items()}
    before = {k: v.detach().clone() for k, v in params.items()}
    opt = torch.optim.Adam(list(params.values()), lr=lr)
    xt = osch.q_sample(tab, x0, eps, t)
    x = audio_conditioned_input(params, xt, cond, feat, projected_audio_dim)
    loss = F.mse_loss(unet_forward(params, plan, x, t), eps)
    loss.backward()
    grads = {k: v.grad.detach().clone() for k, v in params.items()}
    opt.step()
    deltas = {k: params[k].detach() - before[k] for k in params}
    for k in P:
        P[k] = params[k].detach()
    return loss.detach(), grads, deltas


def train_steps(P: dict, plan, batches, projected_audio_dim, lr=1e-2,
                schedule=(100, 0.00085, 0.012), keep_grads=()):
    """Consecutive steps of train.py:107-134 with ONE Adam (its moments carry over):
    batches = [(x0, cond, feat, eps, t), ...].  P is updated in place.

    Returns (losses, {step index: grads}) for the step indices in keep_grads."""
    tab = osch.linear_tables(*schedule)
    params = {k: v.detach().clone().requires_grad_(True) for k, v in P.items()}
    opt = torch.optim.Adam(list(params.values()), lr=lr)
    losses, kept = [], {}
    for i, (x0, cond, feat, eps, t) in enumerate(batches):
        opt.zero_grad()
        xt = osch.q_sample(tab, x0, eps, t)
        x = audio_conditioned_input(params, xt, cond, feat, projected_audio_dim)
        loss = F.mse_loss(unet_forward(params, plan, x, t), eps)
        loss.backward()
        losses.append(loss.detach())
        if i in keep_grads:
            kept[i] = {k: v.grad.detach().clone() for k, v in params.items()}
        opt.step()
    for k in P:
        P[k] = params[k].detach()
    return torch.stack(losses), kept
