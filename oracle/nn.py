"""Oracle restatement of the UNet building blocks (CPU, fp32, NCDHW).

Functional forms over a parameter dict `P` and a key prefix; the keys are the
reference state-dict names (e.g. "input_blocks.1.0.in_layers.0.weight").
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def timestep_embedding(t: torch.Tensor, dim: int, max_period: float = 10000) -> torch.Tensor:
    """utils.py:140-158."""
    half = dim // 2
    freqs = torch.exp(-math.log(max_period) * torch.arange(half, dtype=torch.float32) / half)
    ang = t.reshape(-1, 1).float() * freqs.reshape(1, -1).to(t.device)
    emb = torch.cat([torch.cos(ang), torch.sin(ang)], dim=1)
    return F.pad(emb, (0, 1)) if dim % 2 else emb


def group_norm(x, w, b, groups=32, eps=1e-5, silu=False):
    """GroupNorm32 (utils.py:54-56: fp32 statistics) [+ nn.SiLU]."""
    y = F.group_norm(x.float(), groups, w.float(), b.float(), eps).to(x.dtype)
    return F.silu(y) if silu else y


def conv(x, w, b=None, stride=1, padding=0):
    """conv_nd (utils.py:59-69) for rank 1/2/3 by the weight's rank."""
    fn = {3: F.conv1d, 4: F.conv2d, 5: F.conv3d}[w.dim()]
    return fn(x, w, b, stride=stride, padding=padding)


def linear(x, w, b):
    return F.linear(x, w, b)


def qkv_attention(qkv: torch.Tensor, heads: int, legacy: bool = True, mode: str = "joint",
                  spatial=None) -> torch.Tensor:
    """QKVAttentionLegacy.forward (unet.py:349-366) / QKVAttention (unet.py:388-401).

    mode "joint" is the reference (all T*H*W tokens attend to each other);
    "spatial" / "temporal" apply the same math to per-frame / per-pixel token
    groups (build extension, pinned by reshape onto the reference primitive).
    """
    B, C3, N = qkv.shape
    ch = C3 // (3 * heads)
    if legacy:
        q, k, v = qkv.reshape(B * heads, 3 * ch, N).split(ch, dim=1)
    else:
        q, k, v = (u.reshape(B * heads, ch, N) for u in qkv.chunk(3, dim=1))

    def group(u):
        if mode == "joint":
            return u
        T = spatial[0]
        u = u.reshape(B * heads, ch, T, N // T)
        if mode == "spatial":
            return u.permute(0, 2, 1, 3).reshape(B * heads * T, ch, N // T)
        return u.permute(0, 3, 1, 2).reshape(B * heads * (N // T), ch, T)

    def ungroup(u):
        if mode == "joint":
            return u
        T = spatial[0]
        if mode == "spatial":
            return u.reshape(B * heads, T, ch, N // T).permute(0, 2, 1, 3).reshape(B * heads, ch, N)
        return u.reshape(B * heads, N // T, ch, T).permute(0, 2, 3, 1).reshape(B * heads, ch, N)

    q, k, v = group(q), group(k), group(v)
    s = 1.0 / math.sqrt(math.sqrt(ch))  # unet.py:360: scale applied to q and to k
    wgt = torch.einsum("bct,bcs->bts", q * s, k * s)
    wgt = torch.softmax(wgt.float(), dim=-1).to(wgt.dtype)  # unet.py:364
    a = torch.einsum("bts,bcs->bct", wgt, v)
    return ungroup(a).reshape(B, heads * ch, N)


def cross_attention(q: torch.Tensor, kv: torch.Tensor, heads: int = 1, frames: int = 1,
                    per_frame: bool = True) -> torch.Tensor:
    """Audio cross-attention (build extension of the north star; the reference conditions on
    audio by concatenation only, unet_audio.py:52-61, so this is pinned by no reference
    output): video tokens q [B, C, T*HW] attend to audio tokens kv [B*T, L, 2C] (k | v
    channel halves; head h at channel offset h*ch), softmax(q k^T / sqrt(ch)) v -- the
    QKVAttention math (unet.py:388-401) with separate key/value tokens."""
    B, C, N = q.shape
    T, L, ch = frames, kv.shape[1], C // heads
    HW = N // T
    k, v = kv[..., :C], kv[..., C:]
    if per_frame:
        qs = q.reshape(B, heads, ch, T, HW).permute(0, 3, 1, 4, 2).reshape(B * T * heads, HW, ch)

        def kvs(u):
            return u.reshape(B * T, L, heads, ch).permute(0, 2, 1, 3).reshape(B * T * heads, L, ch)
    else:
        qs = q.reshape(B, heads, ch, N).permute(0, 1, 3, 2).reshape(B * heads, N, ch)

        def kvs(u):
            return u.reshape(B, T * L, heads, ch).permute(0, 2, 1, 3).reshape(B * heads, T * L, ch)
    w = torch.softmax((qs @ kvs(k).transpose(1, 2)).float() / math.sqrt(ch), dim=-1)
    o = w.to(qs.dtype) @ kvs(v)
    if per_frame:
        return o.reshape(B, T, heads, HW, ch).permute(0, 2, 4, 1, 3).reshape(B, C, N)
    return o.reshape(B, heads, N, ch).permute(0, 1, 3, 2).reshape(B, C, N)


def audio_cross_block(P, pre, h, context, heads=1, frames=1, per_frame=True):
    """The AttentionBlock's audio cross-attention residual branch (build extension):
    h + audio_proj_out(cross_attention(audio_q(GN(h)), audio_kv(context)))."""
    a = group_norm(h, P[pre + "audio_norm.weight"], P[pre + "audio_norm.bias"])
    q = conv(a, P[pre + "audio_q.weight"], P[pre + "audio_q.bias"])
    kv = linear(context, P[pre + "audio_kv.weight"], P[pre + "audio_kv.bias"])
    o = cross_attention(q, kv, heads, frames, per_frame)
    return h + conv(o, P[pre + "audio_proj_out.weight"], P[pre + "audio_proj_out.bias"])


def upsample(x, dims):
    """Upsample.forward (unet.py:112-122), nearest; dims=3 keeps T."""
    if dims == 3:
        return F.interpolate(x, (x.shape[2], x.shape[3] * 2, x.shape[4] * 2), mode="nearest")
    return F.interpolate(x, scale_factor=2, mode="nearest")


def resblock(P, pre, x, emb, dropout_mask=None):
    """ResBlock._forward (unet.py:248-268), no up/down, no scale-shift norm, eval dropout."""
    h = group_norm(x, P[pre + "in_layers.0.weight"], P[pre + "in_layers.0.bias"], silu=True)
    kw = P[pre + "in_layers.2.weight"]
    h = conv(h, kw, P[pre + "in_layers.2.bias"], padding=kw.shape[-1] // 2)
    e = linear(F.silu(emb), P[pre + "emb_layers.1.weight"], P[pre + "emb_layers.1.bias"])
    h = h + e.reshape(list(e.shape) + [1] * (h.dim() - 2)).to(h.dtype)
    h = group_norm(h, P[pre + "out_layers.0.weight"], P[pre + "out_layers.0.bias"], silu=True)
    if dropout_mask is not None:
        h = h * dropout_mask
    ow = P[pre + "out_layers.3.weight"]
    h = conv(h, ow, P[pre + "out_layers.3.bias"], padding=ow.shape[-1] // 2)
    if pre + "skip_connection.weight" in P:
        sw = P[pre + "skip_connection.weight"]
        x = conv(x, sw, P[pre + "skip_connection.bias"], padding=sw.shape[-1] // 2)
    return x + h


def attention_block(P, pre, x, heads=1, legacy=True, mode="joint", context=None,
                    per_frame=True):
    """AttentionBlock._forward (unet.py:311-317).

    mode "spatial_temporal" (build extension): the reference block over per-frame token
    groups, then a second one over per-pixel groups with the temporal_* parameters.
    context (build extension): audio tokens [B*T, L, F] for the audio_* cross-attention
    branch, applied after the self-attention when the block has audio_* parameters."""
    B, C = x.shape[:2]
    spatial = list(x.shape[2:])
    sp = spatial if len(spatial) == 3 else [1] + spatial
    xf = x.reshape(B, C, -1)

    def attend(xf, pfx, md):
        h = group_norm(xf, P[pre + pfx + "norm.weight"], P[pre + pfx + "norm.bias"])
        qkv = conv(h, P[pre + pfx + "qkv.weight"], P[pre + pfx + "qkv.bias"])
        a = qkv_attention(qkv, heads, legacy=legacy, mode=md, spatial=sp)
        return xf + conv(a, P[pre + pfx + "proj_out.weight"], P[pre + pfx + "proj_out.bias"])

    if mode == "spatial_temporal":
        h = attend(attend(xf, "", "spatial"), "temporal_", "temporal")
    else:
        h = attend(xf, "", mode)
    if context is not None and pre + "audio_q.weight" in P:
        h = audio_cross_block(P, pre, h, context, heads, sp[0], per_frame)
    return h.reshape(x.shape)


def upsample_block(P, pre, x, dims, use_conv=True):
    h = upsample(x, dims)
    if use_conv:
        h = conv(h, P[pre + "conv.weight"], P[pre + "conv.bias"], padding=1)
    return h


def downsample_block(P, pre, x, dims):
    """Downsample (unet.py:125-152) with conv_resample=True: 3x3 conv, stride 2 ((1,2,2) in 3-D)."""
    stride = (1, 2, 2) if dims == 3 else 2
    return conv(x, P[pre + "op.weight"], P[pre + "op.bias"], stride=stride, padding=1)
