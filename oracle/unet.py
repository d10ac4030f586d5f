"""Oracle restatement of UNetModel / UNetAudio (CPU, fp32, NCDHW), functional.

Topology follows UNetModel.__init__ (unet.py:439-628); forward follows
UNetModel.forward (unet.py:646-675); conditioning follows UNetAudio.forward
(unet_audio.py:51-66) with the wav2vec2 last hidden state passed in already
mean-pooled (the encoder itself is third-party `transformers`: parity
unpinned at that boundary).
"""
from __future__ import annotations

import math
import zlib
from collections import OrderedDict

import torch
import torch.nn.functional as F

from . import nn as onn


def build_plan(in_channels, model_channels, out_channels, num_res_blocks, attention_resolutions,
               channel_mult=(1, 2, 4, 8), dims=2, num_heads=1, num_head_channels=-1,
               num_heads_upsample=-1, conv_resample=True, use_new_attention_order=False,
               attention_mode="joint", audio_attention=0):
    """Layer specs per block, as UNetModel.__init__ builds them (unet.py:476-628)."""
    if num_heads_upsample == -1:
        num_heads_upsample = num_heads

    def heads_for(ch, nh):
        return nh if num_head_channels == -1 else ch // num_head_channels

    ch = first = int(channel_mult[0] * model_channels)
    inputs = [[("conv", in_channels, ch)]]
    skips = [ch]
    ds = 1
    for level, mult in enumerate(channel_mult):
        for _ in range(num_res_blocks):
            out = int(mult * model_channels)
            blk = [("res", ch, out)]
            ch = out
            if ds in attention_resolutions:
                blk.append(("attn", ch, heads_for(ch, num_heads)))
            inputs.append(blk)
            skips.append(ch)
        if level != len(channel_mult) - 1:
            inputs.append([("down", ch)])
            skips.append(ch)
            ds *= 2
    middle = [("res", ch, ch), ("attn", ch, heads_for(ch, num_heads)), ("res", ch, ch)]
    outputs = []
    for level, mult in list(enumerate(channel_mult))[::-1]:
        for i in range(num_res_blocks + 1):
            skip = skips.pop()
            out = int(model_channels * mult)
            blk = [("res", ch + skip, out)]
            ch = out
            if ds in attention_resolutions:
                blk.append(("attn", ch, heads_for(ch, num_heads_upsample)))
            if level and i == num_res_blocks:
                blk.append(("up", ch))
                ds //= 2
            outputs.append(blk)
    return {"input_blocks": inputs, "middle_block": middle, "output_blocks": outputs,
            "model_channels": model_channels, "first_ch": first, "out_channels": out_channels,
            "dims": dims, "legacy": not use_new_attention_order, "conv_resample": conv_resample,
            "attention_mode": attention_mode, "audio_attention": audio_attention}


def _k(dims, k):
    return (k,) * dims


def param_shapes(plan) -> "OrderedDict[str, tuple]":
    """Reference state-dict names -> shapes for a plan."""
    d, mc = plan["dims"], plan["model_channels"]
    ted = 4 * mc
    S = OrderedDict()
    S["time_embed.0.weight"] = (ted, mc)
    S["time_embed.0.bias"] = (ted,)
    S["time_embed.2.weight"] = (ted, ted)
    S["time_embed.2.bias"] = (ted,)

    def layer(pre, spec):
        kind = spec[0]
        if kind == "conv":
            S[pre + "weight"] = (spec[2], spec[1]) + _k(d, 3)
            S[pre + "bias"] = (spec[2],)
        elif kind == "res":
            ci, co = spec[1], spec[2]
            S[pre + "in_layers.0.weight"] = (ci,)
            S[pre + "in_layers.0.bias"] = (ci,)
            S[pre + "in_layers.2.weight"] = (co, ci) + _k(d, 3)
            S[pre + "in_layers.2.bias"] = (co,)
            S[pre + "emb_layers.1.weight"] = (co, ted)
            S[pre + "emb_layers.1.bias"] = (co,)
            S[pre + "out_layers.0.weight"] = (co,)
            S[pre + "out_layers.0.bias"] = (co,)
            S[pre + "out_layers.3.weight"] = (co, co) + _k(d, 3)
            S[pre + "out_layers.3.bias"] = (co,)
            if ci != co:
                S[pre + "skip_connection.weight"] = (co, ci) + _k(d, 1)
                S[pre + "skip_connection.bias"] = (co,)
        elif kind == "attn":
            c = spec[1]
            S[pre + "norm.weight"] = (c,)
            S[pre + "norm.bias"] = (c,)
            S[pre + "qkv.weight"] = (3 * c, c, 1)
            S[pre + "qkv.bias"] = (3 * c,)
            S[pre + "proj_out.weight"] = (c, c, 1)
            S[pre + "proj_out.bias"] = (c,)
            if plan.get("attention_mode") == "spatial_temporal":  # build extension
                S[pre + "temporal_norm.weight"] = (c,)
                S[pre + "temporal_norm.bias"] = (c,)
                S[pre + "temporal_qkv.weight"] = (3 * c, c, 1)
                S[pre + "temporal_qkv.bias"] = (3 * c,)
                S[pre + "temporal_proj_out.weight"] = (c, c, 1)
                S[pre + "temporal_proj_out.bias"] = (c,)
            fa = plan.get("audio_attention", 0)  # audio token width; 0 = no cross-attention
            if fa:
                S[pre + "audio_norm.weight"] = (c,)
                S[pre + "audio_norm.bias"] = (c,)
                S[pre + "audio_q.weight"] = (c, c, 1)
                S[pre + "audio_q.bias"] = (c,)
                S[pre + "audio_kv.weight"] = (2 * c, fa)
                S[pre + "audio_kv.bias"] = (2 * c,)
                S[pre + "audio_proj_out.weight"] = (c, c, 1)
                S[pre + "audio_proj_out.bias"] = (c,)
        elif kind == "down":
            S[pre + "op.weight"] = (spec[1], spec[1]) + _k(d, 3)
            S[pre + "op.bias"] = (spec[1],)
        elif kind == "up":
            S[pre + "conv.weight"] = (spec[1], spec[1]) + _k(d, 3)
            S[pre + "conv.bias"] = (spec[1],)

    for i, blk in enumerate(plan["input_blocks"]):
        for j, spec in enumerate(blk):
            layer(f"input_blocks.{i}.{j}.", spec)
    for j, spec in enumerate(plan["middle_block"]):
        layer(f"middle_block.{j}.", spec)
    for i, blk in enumerate(plan["output_blocks"]):
        for j, spec in enumerate(blk):
            layer(f"output_blocks.{i}.{j}.", spec)
    last = plan["output_blocks"][-1][0][2]
    S["out.0.weight"] = (last,)
    S["out.0.bias"] = (last,)
    S["out.2.weight"] = (plan["out_channels"], plan["first_ch"]) + _k(d, 3)
    S["out.2.bias"] = (plan["out_channels"],)
    return S


def audio_param_shapes(audio_feature_dim, projected_audio_dim, im_cond_input_ch=3,
                       im_cond_output_ch=64):
    """UNetAudio's own parameters (unet_audio.py:43-49), wav2vec2 excluded."""
    S = OrderedDict()
    S["audio_transformer.transform.0.weight"] = (projected_audio_dim, audio_feature_dim)
    S["audio_transformer.transform.0.bias"] = (projected_audio_dim,)
    S["cond_conv_in.weight"] = (im_cond_output_ch, im_cond_input_ch, 1, 1)
    return S


def init_params(shapes, seed: int = 1234) -> dict:
    """Deterministic non-zero init (the reference's zero_module init outputs exactly 0):
    >=2-D: randn / sqrt(fan_in); 1-D weight: 1 + 0.02 randn; 1-D bias: 0.02 randn.
    Each tensor has its own generator seeded from (seed, crc32(name))."""
    P = {}
    for name, shape in shapes.items():
        g = torch.Generator().manual_seed(seed * 1000003 + zlib.crc32(name.encode()))
        if len(shape) >= 2:
            fan_in = math.prod(shape[1:])
            P[name] = torch.randn(shape, generator=g) / math.sqrt(fan_in)
        elif name.endswith("weight"):
            P[name] = 1.0 + 0.02 * torch.randn(shape, generator=g)
        else:
            P[name] = 0.02 * torch.randn(shape, generator=g)
    return P


def _run_block(P, pre, blk, h, emb, plan, attn_mode, context=None):
    d = plan["dims"]
    for j, spec in enumerate(blk):
        lp = f"{pre}{j}."
        kind = spec[0]
        if kind == "conv":
            h = onn.conv(h, P[lp + "weight"], P[lp + "bias"], padding=1)
        elif kind == "res":
            h = onn.resblock(P, lp, h, emb)
        elif kind == "attn":
            h = onn.attention_block(P, lp, h, heads=spec[2], legacy=plan["legacy"],
                                    mode=attn_mode, context=context)
        elif kind == "down":
            h = onn.downsample_block(P, lp, h, d)
        elif kind == "up":
            h = onn.upsample_block(P, lp, h, d)
    return h


def unet_forward(P, plan, x, timesteps, attn_mode=None, context=None):
    """UNetModel.forward (unet.py:646-675), no class conditioning; `context` = audio tokens
    for the audio cross-attention branches (build extension)."""
    mc = plan["model_channels"]
    attn_mode = attn_mode or plan.get("attention_mode", "joint")
    e = onn.timestep_embedding(timesteps, mc)
    e = onn.linear(e, P["time_embed.0.weight"], P["time_embed.0.bias"])
    emb = onn.linear(F.silu(e), P["time_embed.2.weight"], P["time_embed.2.bias"])
    hs = []
    h = x.float()
    for i, blk in enumerate(plan["input_blocks"]):
        h = _run_block(P, f"input_blocks.{i}.", blk, h, emb, plan, attn_mode, context)
        hs.append(h)
    h = _run_block(P, "middle_block.", plan["middle_block"], h, emb, plan, attn_mode, context)
    for i, blk in enumerate(plan["output_blocks"]):
        h = torch.cat([h, hs.pop()], dim=1)
        h = _run_block(P, f"output_blocks.{i}.", blk, h, emb, plan, attn_mode, context)
    h = onn.group_norm(h, P["out.0.weight"], P["out.0.bias"], silu=True)
    return onn.conv(h, P["out.2.weight"], P["out.2.bias"], padding=1)


def audio_conditioned_input(P, image, cond_image, audio_feat, projected_audio_dim):
    """UNetAudio.forward conditioning (unet_audio.py:52-61).

    2-D (reference): image [B,3,H,W], audio_feat [B, F] (wav2vec2 states mean-pooled).
    3-D (build extension D2): image [B,3,T,H,W], one cond image [B,3,h,w] per clip,
    audio_feat [B*T, F] (one audio window per output frame) broadcast over H, W.
    """
    a = F.relu(onn.linear(audio_feat, P["audio_transformer.transform.0.weight"],
                          P["audio_transformer.transform.0.bias"]))
    H, W = image.shape[-2:]
    imc = F.interpolate(cond_image, size=(H, W))
    imc = onn.conv(imc, P["cond_conv_in.weight"])
    if image.dim() == 4:
        a = a.reshape(-1, projected_audio_dim, 1, 1).expand(-1, -1, H, W)
    else:
        B, T = image.shape[0], image.shape[2]
        a = a.reshape(B, T, projected_audio_dim).permute(0, 2, 1)
        a = a.reshape(B, projected_audio_dim, T, 1, 1).expand(-1, -1, -1, H, W)
        imc = imc.unsqueeze(2).expand(-1, -1, T, -1, -1)
    return torch.cat([image, imc, a], dim=1)
