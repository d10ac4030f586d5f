"""Generate the golden fixtures under tests/golden/ by IMPORTING the reference.

Run in the build container only (the reference is not on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

It puts /root/reference/video-generation/diffusion on sys.path, builds the
reference modules (unet.py, utils.py, linear_noise_scheduler.py,
noise_scheduler.py), loads deterministic non-zero weights
(oracle.unet.init_params -- the reference's zero_module init outputs exactly
0), runs forward/backward on seeded inputs and saves inputs (when small) and
outputs as .npz.  The reference UNetAudio cannot be constructed offline
(Wav2Vec2Model.from_pretrained by name, unet_audio.py:14), so its 15 lines of
conditioning are applied around the reference UNetModel here
(unet_audio.py:52-61), with the wav2vec2 states given pre-pooled.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

REF = "/root/reference/video-generation/diffusion"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, REF)

import linear_noise_scheduler as ref_lns  # noqa: E402
import noise_scheduler as ref_ns  # noqa: E402
import unet as ref_unet  # noqa: E402
import utils as ref_utils  # noqa: E402

from oracle.fixtures import (FULL2D, FULL2D_SHAPE, TINY3D, TINY3D_SHAPE, TRAIN5_T,  # noqa: E402
                             seeded, train5_inputs)
from oracle.unet import audio_param_shapes, build_plan, init_params, param_shapes  # noqa: E402

torch.set_num_threads(8)


def npy(t):
    return t.detach().cpu().numpy().astype(np.float32) if t.is_floating_point() else \
        t.detach().cpu().numpy()


def save(name, **arrs):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **{k: npy(v) if torch.is_tensor(v) else np.asarray(v)
                                 for k, v in arrs.items()})
    print("wrote", path, os.path.getsize(path), "bytes")


def load_init(module, seed):
    """Load oracle.init_params into a reference module, checking names/shapes agree."""
    sd = module.state_dict()
    shapes = {k: tuple(v.shape) for k, v in sd.items()}
    P = init_params(shapes, seed)
    module.load_state_dict(P)
    return P


# ------------------------------------------------------------------ schedulers
def gen_schedulers():
    out = {}
    v1 = ref_lns.LinearNoiseScheduler(100, 0.00085, 0.012)
    v2 = ref_lns.LinearNoiseSchedulerV2(500, 0.00005, 0.015)
    cs = ref_ns.CosineNoiseScheduler(2000)
    for tag, s in (("v1", v1), ("v2", v2)):
        for k in ("betas", "alphas", "alpha_cum_prod", "sqrt_alpha_cum_prod",
                  "sqrt_one_minus_alpha_cum_prod"):
            out[f"{tag}_{k}"] = getattr(s, k)
    for k in ("alphas_cumprod", "sqrt_alphas_cumprod", "sqrt_one_minus_alphas_cumprod"):
        out[f"cos_{k}"] = getattr(cs, k)
    # add_noise (q_sample), batch of 2 with different t
    x0 = seeded((2, 3, 4, 8, 8), 10, "uniform")
    eps = seeded((2, 3, 4, 8, 8), 11)
    t = torch.tensor([3, 77])
    out.update(qs_x0=x0, qs_eps=eps, qs_t=t, qs_xt=v1.add_noise(x0, eps, t))
    # sample_prev_timestep: B = 1 (the reference broadcasts t against the last dim)
    xt = seeded((1, 3, 4, 8, 8), 12)
    ep = seeded((1, 3, 4, 8, 8), 13)
    out.update(ps_xt=xt, ps_eps=ep)
    for tag, s, ts in (("v1", v1, (0, 1, 50, 99)), ("v2", v2, (0, 249, 499)),
                       ("cos", cs, (0, 1, 1000, 1999))):
        for ti in ts:
            tt = torch.tensor([ti])
            torch.manual_seed(1000 + ti)
            prev, x0p = s.sample_prev_timestep(xt, ep, tt)
            torch.manual_seed(1000 + ti)
            z = torch.randn(xt.shape) if tag == "v1" else torch.randn_like(xt)
            out[f"{tag}_t{ti}_z"] = z
            out[f"{tag}_t{ti}_prev"] = prev
            out[f"{tag}_t{ti}_x0"] = x0p
    # timestep embedding
    tt = torch.tensor([0, 1, 37, 99, 499])
    out["temb_t"] = tt
    for dim in (64, 65, 128):
        out[f"temb_{dim}"] = ref_utils.timestep_embedding(tt, dim)
    save("schedulers.npz", **out)


# ------------------------------------------------------------------ blocks
def grads_of(module, inputs, out, g):
    module.zero_grad(set_to_none=True)
    for x in inputs:
        x.grad = None
    out.backward(g)


def gen_blocks():
    out = {}
    # GroupNorm32 + SiLU (utils.py:54-56,130-137)
    x = seeded((2, 64, 2, 6, 6), 20).requires_grad_(True)
    gn = ref_utils.normalization(64)
    load_init(gn, 21)
    y = F.silu(gn(x))
    g = seeded(y.shape, 22)
    y.backward(g)
    out.update(gn_w=gn.weight, gn_b=gn.bias, gn_y=y, gn_dx=x.grad,
               gn_dw=gn.weight.grad, gn_db=gn.bias.grad)
    # GroupNorm32 alone on an attention-shaped [B, C, N] tensor, C=128 (4 ch/group)
    x2 = (seeded((2, 128, 40), 23) * 3 + 1.5).requires_grad_(True)
    gn2 = ref_utils.normalization(128)
    load_init(gn2, 24)
    y2 = gn2(x2)
    g2 = seeded(y2.shape, 25)
    y2.backward(g2)
    out.update(gn2_w=gn2.weight, gn2_b=gn2.bias, gn2_y=y2, gn2_dx=x2.grad,
               gn2_dw=gn2.weight.grad, gn2_db=gn2.bias.grad)

    # ResBlock 3-D 64 -> 128 with 1x1x1 skip (unet.py:155-268), eval (dropout 0)
    rb = ref_unet.ResBlock(64, 256, 0.0, out_channels=128, dims=3)
    P = load_init(rb, 30)
    x = seeded((2, 64, 2, 6, 6), 31).requires_grad_(True)
    emb = seeded((2, 256), 32).requires_grad_(True)
    y = rb(x, emb)
    g = seeded(y.shape, 33)
    y.backward(g)
    out.update(rb_y=y, rb_dx=x.grad, rb_demb=emb.grad)
    for k in ("in_layers.2.weight", "skip_connection.weight", "out_layers.0.weight",
              "emb_layers.1.weight", "out_layers.3.bias"):
        out["rb_d_" + k] = dict(rb.named_parameters())[k].grad

    # ResBlock 2-D, same channels (identity skip)
    rb2 = ref_unet.ResBlock(64, 256, 0.0, dims=2)
    load_init(rb2, 34)
    x = seeded((2, 64, 10, 10), 35).requires_grad_(True)
    emb = seeded((2, 256), 36)
    y = rb2(x, emb)
    g = seeded(y.shape, 37)
    y.backward(g)
    out.update(rb2_y=y, rb2_dx=x.grad,
               rb2_d_in_w=rb2.in_layers[2].weight.grad)

    # AttentionBlock, joint over T*H*W = 256 tokens (unet.py:271-317)
    ab = ref_unet.AttentionBlock(64, num_heads=1)
    load_init(ab, 40)
    x = seeded((2, 64, 2, 6, 6), 41).requires_grad_(True)
    y = ab(x)
    g = seeded(y.shape, 42)
    y.backward(g)
    out.update(ab_y=y, ab_dx=x.grad, ab_d_qkv_w=ab.qkv.weight.grad,
               ab_d_proj_w=ab.proj_out.weight.grad, ab_d_norm_w=ab.norm.weight.grad)
    # multi-head, legacy and new order, 2-D
    for tag, new_order in (("abh", False), ("abn", True)):
        m = ref_unet.AttentionBlock(64, num_heads=2, use_new_attention_order=new_order)
        load_init(m, 43)
        x = seeded((1, 64, 10, 10), 44).requires_grad_(True)
        y = m(x)
        g = seeded(y.shape, 45)
        y.backward(g)
        out.update({f"{tag}_y": y, f"{tag}_dx": x.grad,
                    f"{tag}_d_qkv_w": m.qkv.weight.grad})
    # spatial / temporal attention: the reference QKVAttentionLegacy applied to
    # per-frame / per-pixel regroupings of a qkv buffer [B, 3C, T*HW]
    B, C, T, HW = 2, 64, 3, 36
    qkv = seeded((B, 3 * C, T * HW), 46)
    att = ref_unet.QKVAttentionLegacy(1)
    u = qkv.reshape(B, 3 * C, T, HW)
    sp = att(u.permute(0, 2, 1, 3).reshape(B * T, 3 * C, HW))
    sp = sp.reshape(B, T, C, HW).permute(0, 2, 1, 3).reshape(B, C, T * HW)
    tp = att(u.permute(0, 3, 1, 2).reshape(B * HW, 3 * C, T))
    tp = tp.reshape(B, HW, C, T).permute(0, 2, 3, 1).reshape(B, C, T * HW)
    jt = att(qkv)
    out.update(st_spatial=sp, st_temporal=tp, st_joint=jt, st_T=T)

    # Upsample / Downsample 3-D with conv (unet.py:93-152)
    up = ref_unet.Upsample(64, True, dims=3)
    load_init(up, 50)
    x = seeded((1, 64, 2, 5, 5), 51).requires_grad_(True)
    y = up(x)
    g = seeded(y.shape, 52)
    y.backward(g)
    out.update(up_y=y, up_dx=x.grad, up_dw=up.conv.weight.grad)
    dn = ref_unet.Downsample(64, True, dims=3)
    load_init(dn, 53)
    x = seeded((1, 64, 2, 9, 9), 54).requires_grad_(True)
    y = dn(x)
    g = seeded(y.shape, 55)
    y.backward(g)
    out.update(dn_y=y, dn_dx=x.grad, dn_dw=dn.op.weight.grad)
    save("blocks.npz", **out)


# ------------------------------------------------------------------ full models
def gen_models():
    # tiny 3-D UNetModel (BASELINE config 1 shape), joint attention
    m = ref_unet.UNetModel(image_size=64, **TINY3D)
    m.eval()
    plan = build_plan(**TINY3D)
    shapes = param_shapes(plan)
    sd = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    assert list(sd) == list(shapes) and all(sd[k] == shapes[k] for k in sd), "plan mismatch"
    load_init(m, 1234)
    x = seeded(TINY3D_SHAPE, 60, "uniform")
    t = torch.tensor([37])
    eps = seeded((1, 3) + TINY3D_SHAPE[2:], 61)
    y = m(x, t)
    loss = F.mse_loss(y, eps)
    loss.backward()
    named = dict(m.named_parameters())
    sel = ("input_blocks.0.0.weight", "out.2.weight", "input_blocks.3.1.qkv.weight",
           "middle_block.0.in_layers.0.weight", "output_blocks.0.0.skip_connection.weight",
           "time_embed.0.weight")
    save("unet_tiny3d.npz", y=y, loss=loss, t=t,
         **{"grad_" + k: named[k].grad for k in sel})

    # full-width 2-D UNetModel (the literal train.py topology) at 32x32, batch 2
    m2 = ref_unet.UNetModel(image_size=32, **FULL2D)
    m2.eval()
    plan2 = build_plan(**FULL2D)
    sd2 = {k: tuple(v.shape) for k, v in m2.state_dict().items()}
    shapes2 = param_shapes(plan2)
    assert list(sd2) == list(shapes2) and all(sd2[k] == shapes2[k] for k in sd2)
    P2 = load_init(m2, 1234)
    x = seeded(FULL2D_SHAPE, 62, "uniform")
    t = torch.tensor([5, 480])
    y = m2(x, t)
    g = seeded(y.shape, 63)
    y.backward(g)
    named2 = dict(m2.named_parameters())
    save("unet_full2d.npz", y=y, t=t, grad_in=named2["input_blocks.0.0.weight"].grad,
         grad_attn=named2["input_blocks.1.1.qkv.weight"].grad,
         grad_out=named2["out.2.weight"].grad)

    # UNetAudio conditioning (unet_audio.py:52-61) restated around the reference
    # UNetModel, 2-D reference semantics, wav2vec2 states pre-pooled.
    cfg = dict(FULL2D)
    A = init_params(audio_param_shapes(768, 128), 77)
    image = seeded((2, 3, 32, 32), 64, "uniform")
    cond = seeded((2, 3, 16, 16), 65, "uniform")
    feat = seeded((2, 768), 66)
    lin = nn.Linear(768, 128)
    lin.weight.data.copy_(A["audio_transformer.transform.0.weight"])
    lin.bias.data.copy_(A["audio_transformer.transform.0.bias"])
    cc = nn.Conv2d(3, 64, 1, bias=False)
    cc.weight.data.copy_(A["cond_conv_in.weight"])
    with torch.no_grad():
        af = F.relu(lin(feat)).view(-1, 128, 1, 1).expand(-1, -1, 32, 32)
        imc = cc(F.interpolate(cond, size=image.shape[-2:]))
        feats = torch.cat([image, imc, af], dim=1)
        y = m2(feats, torch.tensor([5, 480]))
    del cfg
    save("unet_audio2d.npz", y=y, t=torch.tensor([5, 480]))


# ------------------------------------------------------------------ one train step
def gen_train_step():
    """One step of train.py:122-134 on BASELINE config 1's shape (tiny UNet3D, 64x64x8):
    reference add_noise (q_sample) -> conditioning (unet_audio.py:52-61, restated; 5-D
    extension D2: one reference image per clip, one pooled audio window per frame) ->
    reference UNetModel -> MSELoss -> backward -> torch.optim.Adam(lr=1e-2).step().
    Saves the loss and the parameter deltas of one Adam step."""
    m = ref_unet.UNetModel(image_size=64, **TINY3D)
    m.train()  # dropout 0 (the UNetModel default): train and eval agree
    load_init(m, 1234)
    A = init_params(audio_param_shapes(64, 16, im_cond_output_ch=16), 77)
    lin = nn.Linear(64, 16)
    lin.weight.data.copy_(A["audio_transformer.transform.0.weight"])
    lin.bias.data.copy_(A["audio_transformer.transform.0.bias"])
    cc = nn.Conv2d(3, 16, 1, bias=False)
    cc.weight.data.copy_(A["cond_conv_in.weight"])
    T, S = TINY3D_SHAPE[2], TINY3D_SHAPE[3]
    x0 = seeded((1, 3, T, S, S), 70, "uniform")
    cond = seeded((1, 3, 32, 32), 71, "uniform")
    feat = seeded((T, 64), 72)
    eps = seeded((1, 3, T, S, S), 73)
    t = torch.tensor([37])
    sched = ref_lns.LinearNoiseScheduler(100, 0.00085, 0.012)  # train.py:48-52
    params = list(m.parameters()) + list(lin.parameters()) + list(cc.parameters())
    names = [n for n, _ in m.named_parameters()] + \
        ["audio_transformer.transform.0.weight", "audio_transformer.transform.0.bias",
         "cond_conv_in.weight"]
    before = [p.detach().clone() for p in params]
    opt = torch.optim.Adam(params, lr)  # train.py:102 (lr=1e-2)
    opt.zero_grad()
    xt = sched.add_noise(x0, eps, t)
    a = F.relu(lin(feat)).reshape(1, T, 16).permute(0, 2, 1).reshape(1, 16, T, 1, 1)
    a = a.expand(-1, -1, -1, S, S)
    imc = cc(F.interpolate(cond, size=(S, S))).unsqueeze(2).expand(-1, -1, T, -1, -1)
    y = m(torch.cat([xt, imc, a], dim=1), t)
    loss = nn.MSELoss()(y, eps)
    loss.backward()
    grads = {n: p.grad.detach().clone() for n, p in zip(names, params)}
    opt.step()
    sel = ("input_blocks.0.0.weight", "out.2.weight", "input_blocks.3.1.qkv.weight",
           "input_blocks.3.1.proj_out.weight", "middle_block.0.in_layers.0.weight",
           "output_blocks.0.0.skip_connection.weight", "time_embed.0.weight",
           "audio_transformer.transform.0.weight", "cond_conv_in.weight")
    # inputs are regenerated from their seeds by the tests (oracle.fixtures.seeded)
    out = {"t": t, "loss": loss}
    for n, p, b in zip(names, params, before):
        if n in sel:
            out["delta_" + n] = p.detach() - b
            out["grad_" + n] = grads[n]
    save("train_step_tiny3d.npz", **out)


# ------------------------------------------------------------------ five train steps
def gen_train_steps5(lr=1e-2, name="train_steps5_tiny3d.npz"):
    """Five consecutive steps of the reference training loop (train.py:107-134) on BASELINE
    config 1's shape: ONE torch.optim.Adam(lr=1e-2) over the imported reference UNetModel plus
    the restated conditioning (as gen_train_step), a new seeded batch, noise and timestep per
    step.  Saves every step's loss, the step-1 and step-5 gradients and the five-step
    parameter change of selected parameters: the pin of the product Trainer beyond one step
    (the product packs its conv operands per call in step 1 and in one
    batched launch from step 2 on).  lr: train.py:102's 1e-2 (the default fixture), or 1e-4,
    the rate bench.py's headline trains at (train_steps5_tiny3d_lr1e-4.npz, VERDICT r05
    item 4)."""
    m = ref_unet.UNetModel(image_size=64, **TINY3D)
    m.train()
    load_init(m, 1234)
    A = init_params(audio_param_shapes(64, 16, im_cond_output_ch=16), 77)
    lin = nn.Linear(64, 16)
    lin.weight.data.copy_(A["audio_transformer.transform.0.weight"])
    lin.bias.data.copy_(A["audio_transformer.transform.0.bias"])
    cc = nn.Conv2d(3, 16, 1, bias=False)
    cc.weight.data.copy_(A["cond_conv_in.weight"])
    T, S = TINY3D_SHAPE[2], TINY3D_SHAPE[3]
    sched = ref_lns.LinearNoiseScheduler(100, 0.00085, 0.012)
    params = list(m.parameters()) + list(lin.parameters()) + list(cc.parameters())
    names = [n for n, _ in m.named_parameters()] + \
        ["audio_transformer.transform.0.weight", "audio_transformer.transform.0.bias",
         "cond_conv_in.weight"]
    before = [p.detach().clone() for p in params]
    opt = torch.optim.Adam(params, lr)  # train.py:102 (lr=1e-2)
    sel = ("input_blocks.0.0.weight", "out.2.weight", "input_blocks.3.1.qkv.weight",
           "input_blocks.3.1.proj_out.weight", "middle_block.0.in_layers.0.weight",
           "output_blocks.0.0.skip_connection.weight", "time_embed.0.weight",
           "audio_transformer.transform.0.weight", "cond_conv_in.weight")
    out = {"t": torch.tensor(TRAIN5_T)}
    losses = []
    for k, tk in enumerate(TRAIN5_T):
        x0, cond, feat, eps = train5_inputs(k, T, S)
        t = torch.tensor([tk])
        opt.zero_grad()
        xt = sched.add_noise(x0, eps, t)
        a = F.relu(lin(feat)).reshape(1, T, 16).permute(0, 2, 1).reshape(1, 16, T, 1, 1)
        a = a.expand(-1, -1, -1, S, S)
        imc = cc(F.interpolate(cond, size=(S, S))).unsqueeze(2).expand(-1, -1, T, -1, -1)
        y = m(torch.cat([xt, imc, a], dim=1), t)
        loss = nn.MSELoss()(y, eps)
        loss.backward()
        losses.append(float(loss))
        if k in (0, 4):
            for n, p in zip(names, params):
                if n in sel:
                    out[f"grad{k + 1}_{n}"] = p.grad.detach().clone()
        opt.step()
    out["losses"] = torch.tensor(losses)
    for n, p, b in zip(names, params, before):
        if n in sel:
            out["delta5_" + n] = p.detach() - b
    out["lr"] = torch.tensor(lr)
    save(name, **out)


# ------------------------------------------------------------------ sampling trajectories
TRAJ_STEPS = 10
TRAJ_KEEP = (1, 5, 10)  # steps whose x_t / x0 are stored


def _ref_trajectory(model_fn, shape, n_timesteps, steps, seed):
    """The reference sampling loop (test.py:56-65, restated: test.py itself is a script that
    needs torchvision and a checkpoint) over the imported LinearNoiseSchedulerV2(500, 5e-5,
    0.015) (test.py:111).  The initial x_T (test.py:53) and every step's z (randn_like at
    linear_noise_scheduler.py:97) are drawn as oracle.fixtures.seeded(shape, seed + k) and
    injected by replacing torch.randn_like while the loop runs, so the test regenerates them
    from the seeds."""
    sched = ref_lns.LinearNoiseSchedulerV2(500, 0.00005, 0.015)
    xt = seeded(shape, seed)
    zs = iter(seeded(shape, seed + 1 + k) for k in range(steps))
    orig = torch.randn_like
    torch.randn_like = lambda x, *a, **k: next(zs)
    out = {}
    try:
        with torch.no_grad():
            for k, i in enumerate(reversed(range(n_timesteps))):
                if k == steps:
                    break
                t = torch.tensor([i]).long()
                eps = model_fn(xt, t).detach()
                xt, x0 = sched.sample_prev_timestep(xt, eps, t)
                if k + 1 in TRAJ_KEEP or k + 1 == steps:
                    out[f"xt_{k + 1}"] = xt.clone()
                    out[f"x0_{k + 1}"] = x0.clone()
    finally:
        torch.randn_like = orig
    return out


def gen_trajectory():
    """Denoised frames over a sampling trajectory (north_star parity bar):
    the first TRAJ_STEPS steps of a 500-step reverse process, and a whole n_timesteps = 10
    call, on
      * the tiny UNet3D (BASELINE config 1 shape, 64x64x8): conditioning restated around
        the reference UNetModel as in gen_train_step (one reference image per clip, one
        pooled audio window per frame);
      * the full-width 2-D UNetModel at 64x64 (train.py's topology, the reference's literal
        per-frame semantics): UNetAudio's conditioning (unet_audio.py:52-61) restated.
    Audio enters as pooled wav2vec2 states (seeded), as in the other UNetAudio fixtures."""
    out = {}
    # tiny 3-D
    m = ref_unet.UNetModel(image_size=64, **TINY3D)
    m.eval()
    load_init(m, 1234)
    A = init_params(audio_param_shapes(64, 16, im_cond_output_ch=16), 77)
    lin = nn.Linear(64, 16)
    lin.weight.data.copy_(A["audio_transformer.transform.0.weight"])
    lin.bias.data.copy_(A["audio_transformer.transform.0.bias"])
    cc = nn.Conv2d(3, 16, 1, bias=False)
    cc.weight.data.copy_(A["cond_conv_in.weight"])
    T, S = 8, 64
    cond = seeded((1, 3, 32, 32), 80, "uniform")
    feat = seeded((T, 64), 81)

    def tiny(xt, t):
        a = F.relu(lin(feat)).reshape(1, T, 16).permute(0, 2, 1).reshape(1, 16, T, 1, 1)
        a = a.expand(-1, -1, -1, S, S)
        imc = cc(F.interpolate(cond, size=(S, S))).unsqueeze(2).expand(-1, -1, T, -1, -1)
        return m(torch.cat([xt, imc, a], dim=1), t)

    for k, v in _ref_trajectory(tiny, (1, 3, T, S, S), 500, TRAJ_STEPS, 900).items():
        out["tiny3d_500_" + k] = v
    # full-width 2-D at 64x64
    m2 = ref_unet.UNetModel(image_size=64, **FULL2D)
    m2.eval()
    load_init(m2, 1234)
    A2 = init_params(audio_param_shapes(768, 128), 77)
    lin2 = nn.Linear(768, 128)
    lin2.weight.data.copy_(A2["audio_transformer.transform.0.weight"])
    lin2.bias.data.copy_(A2["audio_transformer.transform.0.bias"])
    cc2 = nn.Conv2d(3, 64, 1, bias=False)
    cc2.weight.data.copy_(A2["cond_conv_in.weight"])
    cond2 = seeded((1, 3, 48, 48), 82, "uniform")
    feat2 = seeded((1, 768), 83)

    def full2d(xt, t):
        af = F.relu(lin2(feat2)).view(-1, 128, 1, 1).expand(-1, -1, 64, 64)
        imc = cc2(F.interpolate(cond2, size=xt.shape[-2:]))
        return m2(torch.cat([xt, imc, af], dim=1), t)

    for k, v in _ref_trajectory(full2d, (1, 3, 64, 64), 500, TRAJ_STEPS, 920).items():
        out["full2d_500_" + k] = v
    for k, v in _ref_trajectory(full2d, (1, 3, 64, 64), 10, 10, 940).items():
        out["full2d_10_" + k] = v
    save("trajectory.npz", **out)


if __name__ == "__main__":
    which = sys.argv[1:] or ["schedulers", "blocks", "models", "train_step", "train_steps5",
                             "trajectory"]
    if "schedulers" in which:
        gen_schedulers()
    if "blocks" in which:
        gen_blocks()
    if "models" in which:
        gen_models()
    if "train_step" in which:
        gen_train_step()
    if "train_steps5" in which:
        gen_train_steps5()
    if "train_steps5_lr1e-4" in which:
        gen_train_steps5(1e-4, "train_steps5_tiny3d_lr1e-4.npz")
    if "trajectory" in which:
        gen_trajectory()
