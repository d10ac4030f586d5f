"""UNet building blocks with the reference's class names, constructor arguments and
state-dict keys (video-generation/diffusion/unet.py, utils.py), running on libvdiff.

Every module keeps the reference's sub-module structure (e.g. ResBlock.in_layers =
Sequential(GroupNorm32, SiLU, conv)) so checkpoints load unchanged, but the forward
passes call the fused HIP ops directly: GN+SiLU(+dropout) is one kernel, the
ResBlock emb-add and skip-add are fused into the conv epilogues, attention is
flash attention, and nothing is ever moved to the CPU.

Activations are channels-last tensors (see vdiff.ops).  Parameters are fp32
masters; `UNetModel.dtype` selects the activation / MFMA dtype (fp32 = parity
mode, bf16 = throughput mode).
"""
from __future__ import annotations

import math
from abc import abstractmethod

import torch as th
import torch.nn as nn
import torch.utils.checkpoint

from . import ops

ATTENTION_MODES = ("joint", "spatial", "temporal", "spatial_temporal")


# ------------------------------------------------------------------ utils.py
class SiLU(nn.SiLU):
    """nn.SiLU on the vd_silu kernel (used by time_embed / emb_layers)."""

    def forward(self, x):
        return ops.silu(x)


class GroupNorm32(nn.GroupNorm):
    """utils.py:54-56: GroupNorm with fp32 statistics, output in the input dtype."""

    def forward(self, x):
        return ops.group_norm_silu(x, self.weight, self.bias, self.num_groups, self.eps,
                                   silu=False)


class _ConvMixin:
    def _check(self):
        if self.groups != 1 or any(d != 1 for d in self.dilation) or self.padding_mode != "zeros":
            raise NotImplementedError("libvdiff conv: groups=1, dilation=1, zero padding only")
        if isinstance(self.padding, str):
            raise NotImplementedError("string padding is not supported")

    def forward(self, x):
        self._check()
        return ops.conv(x, self.weight, self.bias, self.stride, self.padding)


class Conv1d(_ConvMixin, nn.Conv1d):
    pass


class Conv2d(_ConvMixin, nn.Conv2d):
    pass


class Conv3d(_ConvMixin, nn.Conv3d):
    pass


class Linear(nn.Linear):
    def forward(self, x):
        return ops.linear(x, self.weight, self.bias)


def conv_nd(dims, *args, **kwargs):
    """utils.py:59-69."""
    if dims == 1:
        return Conv1d(*args, **kwargs)
    if dims == 2:
        return Conv2d(*args, **kwargs)
    if dims == 3:
        return Conv3d(*args, **kwargs)
    raise ValueError(f"unsupported dimensions: {dims}")


def linear(*args, **kwargs):
    """utils.py:72-76."""
    return Linear(*args, **kwargs)


def avg_pool_nd(dims, *args, **kwargs):
    """utils.py:79-89 (kept for API compatibility; not on the accelerated path)."""
    return {1: nn.AvgPool1d, 2: nn.AvgPool2d, 3: nn.AvgPool3d}[dims](*args, **kwargs)


def update_ema(target_params, source_params, rate=0.99):
    for targ, src in zip(target_params, source_params):
        targ.detach().mul_(rate).add_(src, alpha=1 - rate)


def zero_module(module):
    """utils.py:105-111."""
    for p in module.parameters():
        p.detach().zero_()
    return module


def scale_module(module, scale):
    for p in module.parameters():
        p.detach().mul_(scale)
    return module


def mean_flat(tensor):
    return tensor.mean(dim=list(range(1, len(tensor.shape))))


def normalization(channels):
    """utils.py:130-137: GroupNorm32 with 32 groups."""
    return GroupNorm32(32, channels)


def timestep_embedding(timesteps, dim, max_period=10000):
    """utils.py:140-158 on the vd_timestep_embedding kernel."""
    return ops.timestep_embedding(timesteps, dim, max_period)


def checkpoint(func, inputs, params, flag):
    """utils.py:161-176: recompute `func` in backward when flag is set."""
    if flag:
        return th.utils.checkpoint.checkpoint(func, *inputs, use_reentrant=False)
    return func(*inputs)


class CheckpointFunction(th.autograd.Function):
    """utils.py:179-207, kept for API compatibility (checkpoint() uses torch's
    non-reentrant implementation)."""

    @staticmethod
    def forward(ctx, run_function, length, *args):
        ctx.run_function = run_function
        ctx.input_tensors = list(args[:length])
        ctx.input_params = list(args[length:])
        with th.no_grad():
            return ctx.run_function(*ctx.input_tensors)

    @staticmethod
    def backward(ctx, *output_grads):
        ins = [x.detach().requires_grad_(True) for x in ctx.input_tensors]
        with th.enable_grad():
            outs = ctx.run_function(*[x.view_as(x) for x in ins])
        grads = th.autograd.grad(outs, ins + ctx.input_params, output_grads, allow_unused=True)
        return (None, None) + grads


# ------------------------------------------------------------------ unet.py blocks
class TimestepBlock(nn.Module):
    @abstractmethod
    def forward(self, x, emb):
        """Apply the module to `x` given `emb` timestep embeddings."""


class TimestepEmbedSequential(nn.Sequential, TimestepBlock):
    """unet.py:78-90; `context` (audio tokens, build extension) reaches the attention blocks."""

    def forward(self, x, emb, context=None):
        for layer in self:
            if isinstance(layer, TimestepBlock):
                x = layer(x, emb)
            elif context is not None and isinstance(layer, AttentionBlock):
                x = layer(x, context=context)
            else:
                x = layer(x)
        return x


class Upsample(nn.Module):
    """unet.py:93-122: nearest x2 on (H, W) (T kept for dims=3), optional 3x3 conv."""

    def __init__(self, channels, use_conv, dims=2, out_channels=None):
        super().__init__()
        self.channels = channels
        self.out_channels = out_channels or channels
        self.use_conv = use_conv
        self.dims = dims
        if use_conv:
            self.conv = conv_nd(dims, self.channels, self.out_channels, 3, padding=1)

    def forward(self, x):
        assert x.shape[1] == self.channels
        if self.dims == 1:
            raise NotImplementedError("1-D Upsample is not on the accelerated path")
        x = ops.upsample_nearest_hw(x)
        return self.conv(x) if self.use_conv else x


class Downsample(nn.Module):
    """unet.py:125-152: stride-2 3x3 conv ((1,2,2) for dims=3)."""

    def __init__(self, channels, use_conv, dims=2, out_channels=None):
        super().__init__()
        self.channels = channels
        self.out_channels = out_channels or channels
        self.use_conv = use_conv
        self.dims = dims
        stride = 2 if dims != 3 else (1, 2, 2)
        if use_conv:
            self.op = conv_nd(dims, self.channels, self.out_channels, 3, stride=stride, padding=1)
        else:
            assert self.channels == self.out_channels
            self.op = avg_pool_nd(dims, kernel_size=stride, stride=stride)

    def forward(self, x):
        assert x.shape[1] == self.channels
        if not self.use_conv:
            raise NotImplementedError("avg-pool Downsample (conv_resample=False) is not "
                                      "on the accelerated path")
        return self.op(x)


class ResBlock(TimestepBlock):
    """unet.py:155-268.

    forward = conv2(dropout(silu(GN2(conv1(silu(GN1(x))) + emb_layers(emb))))) + skip(x)
    with GN+SiLU(+dropout) fused, the emb add fused into conv1's epilogue and the skip
    add fused into conv2's epilogue.
    """

    def __init__(self, channels, emb_channels, dropout, out_channels=None, use_conv=False,
                 use_scale_shift_norm=False, dims=2, use_checkpoint=False, up=False, down=False):
        super().__init__()
        self.channels = channels
        self.emb_channels = emb_channels
        self.dropout = dropout
        self.out_channels = out_channels or channels
        self.use_conv = use_conv
        self.use_checkpoint = use_checkpoint
        self.use_scale_shift_norm = use_scale_shift_norm
        if use_scale_shift_norm or up or down:
            raise NotImplementedError("use_scale_shift_norm / resblock_updown are not used by "
                                      "the reference train.py/test.py path and not accelerated")
        self.in_layers = nn.Sequential(
            normalization(channels), SiLU(),
            conv_nd(dims, channels, self.out_channels, 3, padding=1))
        self.updown = False
        self.h_upd = self.x_upd = nn.Identity()
        self.emb_layers = nn.Sequential(SiLU(), linear(emb_channels, self.out_channels))
        self.out_layers = nn.Sequential(
            normalization(self.out_channels), SiLU(), nn.Dropout(p=dropout),
            zero_module(conv_nd(dims, self.out_channels, self.out_channels, 3, padding=1)))
        if self.out_channels == channels:
            self.skip_connection = nn.Identity()
        elif use_conv:
            self.skip_connection = conv_nd(dims, channels, self.out_channels, 3, padding=1)
        else:
            self.skip_connection = conv_nd(dims, channels, self.out_channels, 1)

    def forward(self, x, emb):
        return checkpoint(self._forward, (x, emb), self.parameters(), self.use_checkpoint)

    def _forward(self, x, emb):
        gn1, conv1 = self.in_layers[0], self.in_layers[2]
        gn2, drop, conv2 = self.out_layers[0], self.out_layers[2], self.out_layers[3]
        # x also feeds the skip branch: its two gradients meet inside GN1's backward
        h, xs = ops.group_norm_silu_pass(x, gn1.weight, gn1.bias, gn1.num_groups, gn1.eps)
        emb_out = emb[self] if isinstance(emb, EmbTable) else self.emb_layers(emb)
        h = ops.conv(h, conv1.weight, conv1.bias, conv1.stride, conv1.padding, chan_add=emb_out)
        p = drop.p if self.training else 0.0
        h = ops.group_norm_silu(h, gn2.weight, gn2.bias, gn2.num_groups, gn2.eps, dropout=p)
        skip = self.skip_connection(xs)
        return ops.conv(h, conv2.weight, conv2.bias, conv2.stride, conv2.padding, residual=skip)


class EmbTable:
    """Every ResBlock's emb_layers(emb) = Linear(SiLU(emb)) (unet.py:211-217) of one forward,
    computed as ONE GEMM: the blocks share `emb`, so SiLU runs once and the per-block
    [Cout, 256] weights are stacked into one [sum Cout, 256] operand (one launch instead of
    one per block, forward and backward alike; gradients reach each block's own weight and
    bias through the stacking).  Passed down TimestepEmbedSequential in place of `emb`.
    A [B, 256] x [256, 2752] product at B = 1 is a GEMV: it runs on torch's BLAS (SURVEY
    2.2 keeps the time-embedding MLPs in PyTorch) -- the implicit-GEMM kernel walks the
    2752-long K of its backward in one sequential tile loop (0.23 ms measured)."""

    def __init__(self, emb, blocks):
        lins = [rb.emb_layers[1] for rb in blocks]
        w = th.cat([lin.weight for lin in lins])
        b = th.cat([lin.bias for lin in lins])
        out = th.nn.functional.linear(th.nn.functional.silu(emb), w, b)
        self.rows = dict(zip(map(id, blocks), out.split([lin.out_features for lin in lins],
                                                         dim=-1)))
        self.emb = emb

    def __getitem__(self, block):
        return self.rows[id(block)]


def emb_table(model, emb):
    """EmbTable over the model's ResBlocks, or `emb` itself when the blocks do not all share
    the reference emb_layers structure.  The block list is cached together with the identity
    of the module that built it: nn.DataParallel replicas (test.py:101) copy __dict__
    shallowly, so a replica sees the original's cache under a different owner and rebuilds
    it from its own (per-device) blocks."""
    cached = model.__dict__.get("_resblocks")
    if cached is None or cached[0] != id(model):
        blocks = [m for m in model.modules() if isinstance(m, ResBlock)]
        ok = all(isinstance(rb.emb_layers[0], SiLU) and isinstance(rb.emb_layers[1], nn.Linear)
                 for rb in blocks)
        cached = (id(model), blocks if ok else [])
        model.__dict__["_resblocks"] = cached
    blocks = cached[1]
    return EmbTable(emb, blocks) if blocks else emb


class QKVAttentionLegacy(nn.Module):
    """unet.py:340-366: heads split before q/k/v ([N, H*3*C, T] input)."""

    def __init__(self, n_heads):
        super().__init__()
        self.n_heads = n_heads

    def forward(self, qkv, mode="joint", spatial=None):
        return ops.attention(qkv, self.n_heads, mode=mode, spatial=spatial, legacy=True)


class QKVAttention(nn.Module):
    """unet.py:373-401: q/k/v split before heads ([N, 3*H*C, T] input)."""

    def __init__(self, n_heads):
        super().__init__()
        self.n_heads = n_heads

    def forward(self, qkv, mode="joint", spatial=None):
        return ops.attention(qkv, self.n_heads, mode=mode, spatial=spatial, legacy=False)


class AttentionBlock(nn.Module):
    """unet.py:271-317: x + proj_out(attention(qkv(GN(x)))).

    attention_mode: "joint" (reference: all T*H*W tokens), "spatial" (per frame),
    "temporal" (per pixel) or "spatial_temporal" (spatial with the reference
    parameters, then temporal with extra temporal_* parameters, zero-initialised
    projection).  The reference always recomputes this block in backward
    (utils.py:161, unet.py:309); flash attention keeps only O(N) state, so no
    recompute is needed.
    """

    def __init__(self, channels, num_heads=1, num_head_channels=-1, use_checkpoint=False,
                 use_new_attention_order=False, attention_mode="joint", audio_attention=False,
                 audio_context_dim=768, audio_per_frame=True):
        super().__init__()
        self.channels = channels
        if num_head_channels == -1:
            self.num_heads = num_heads
        else:
            assert channels % num_head_channels == 0, \
                f"q,k,v channels {channels} is not divisible by num_head_channels {num_head_channels}"
            self.num_heads = channels // num_head_channels
        if attention_mode not in ATTENTION_MODES:
            raise ValueError(f"attention_mode must be one of {ATTENTION_MODES}")
        self.attention_mode = attention_mode
        self.use_checkpoint = use_checkpoint
        self.legacy = not use_new_attention_order
        self.norm = normalization(channels)
        self.qkv = conv_nd(1, channels, channels * 3, 1)
        self.attention = (QKVAttentionLegacy if self.legacy else QKVAttention)(self.num_heads)
        self.proj_out = zero_module(conv_nd(1, channels, channels, 1))
        if attention_mode == "spatial_temporal":
            self.temporal_norm = normalization(channels)
            self.temporal_qkv = conv_nd(1, channels, channels * 3, 1)
            self.temporal_proj_out = zero_module(conv_nd(1, channels, channels, 1))
        # audio cross-attention (north_star build extension; the reference conditions on audio
        # by concatenation only, unet_audio.py:52-61): queries from the video tokens, keys /
        # values from the audio tokens of the clip's frames, zero-initialised projection
        self.audio_attention = audio_attention
        self.audio_per_frame = audio_per_frame
        if audio_attention:
            self.audio_norm = normalization(channels)
            self.audio_q = conv_nd(1, channels, channels, 1)
            self.audio_kv = linear(audio_context_dim, 2 * channels)
            self.audio_proj_out = zero_module(conv_nd(1, channels, channels, 1))

    def forward(self, x, context=None):
        if context is None:
            return checkpoint(self._forward, (x,), self.parameters(), self.use_checkpoint)
        return checkpoint(self._forward, (x, context), self.parameters(), self.use_checkpoint)

    def _attend(self, xf, norm, qkv_conv, proj, mode, spatial):
        h, xs = ops.group_norm_silu_pass(xf, norm.weight, norm.bias, norm.num_groups, norm.eps,
                                         silu=False)
        qkv = ops.conv(h, qkv_conv.weight, qkv_conv.bias)
        a = ops.attention(qkv, self.num_heads, mode=mode, spatial=spatial, legacy=self.legacy)
        return ops.conv(a, proj.weight, proj.bias, residual=xs)

    def _cross(self, h, context, frames):
        """h + audio_proj_out(cross_attention(audio_q(GN(h)), audio_kv(audio tokens)))."""
        a = ops.group_norm_silu(h, self.audio_norm.weight, self.audio_norm.bias,
                                self.audio_norm.num_groups, self.audio_norm.eps, silu=False)
        q = ops.conv(a, self.audio_q.weight, self.audio_q.bias)
        kv = ops.linear(context.to(h.dtype), self.audio_kv.weight, self.audio_kv.bias)
        o = ops.cross_attention(q, kv, self.num_heads, frames, self.audio_per_frame)
        return ops.conv(o, self.audio_proj_out.weight, self.audio_proj_out.bias, residual=h)

    def _forward(self, x, context=None):
        b, c, *spatial = x.shape
        x = ops.to_cl(x)
        xf = x.reshape(b, c, -1)
        sp = tuple(spatial) if len(spatial) == 3 else (1,) + tuple(spatial)
        mode = self.attention_mode
        if mode == "spatial_temporal":
            h = self._attend(xf, self.norm, self.qkv, self.proj_out, "spatial", sp)
            h = self._attend(h, self.temporal_norm, self.temporal_qkv, self.temporal_proj_out,
                             "temporal", sp)
        else:
            h = self._attend(xf, self.norm, self.qkv, self.proj_out, mode, sp)
        if self.audio_attention and context is not None:
            h = self._cross(h, context, sp[0])
        return h.reshape(b, c, *spatial)


def cat_channels(a, b):
    """th.cat([a, b], dim=1) into a channels-last buffer (the skip concat, unet.py:672)."""
    out = ops.empty_cl([a.shape[0], a.shape[1] + b.shape[1]] + list(a.shape[2:]), a.dtype,
                       a.device)
    out[:, :a.shape[1]] = a
    out[:, a.shape[1]:] = b
    return out


class _CatFn(th.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        ctx.ca = a.shape[1]
        return cat_channels(a, b)

    @staticmethod
    def backward(ctx, g):
        return g[:, :ctx.ca], g[:, ctx.ca:]


# ------------------------------------------------------------------ UNetModel
class UNetModel(nn.Module):
    """unet.py:408-675 with the same constructor and forward(x, timesteps, y=None).

    Extensions (keyword-only, defaults reproduce the reference):
      attention_mode: "joint" | "spatial" | "temporal" | "spatial_temporal"
      use_bf16: run activations / MFMA in bf16 (fp32 master weights).  use_fp16=True
                maps to bf16 as well (gfx950 path has no fp16 kernels).
    """

    def __init__(self, image_size, in_channels, model_channels, out_channels, num_res_blocks,
                 attention_resolutions, dropout=0, channel_mult=(1, 2, 4, 8), conv_resample=True,
                 dims=2, num_classes=None, use_checkpoint=False, use_fp16=False, num_heads=1,
                 num_head_channels=-1, num_heads_upsample=-1, use_scale_shift_norm=False,
                 resblock_updown=False, use_new_attention_order=False, *,
                 attention_mode="joint", use_bf16=False, audio_attention=False,
                 audio_context_dim=768):
        super().__init__()
        if num_heads_upsample == -1:
            num_heads_upsample = num_heads
        self.image_size = image_size
        self.in_channels = in_channels
        self.model_channels = model_channels
        self.out_channels = out_channels
        self.num_res_blocks = num_res_blocks
        self.attention_resolutions = attention_resolutions
        self.dropout = dropout
        self.channel_mult = channel_mult
        self.conv_resample = conv_resample
        self.num_classes = num_classes
        self.use_checkpoint = use_checkpoint
        self.dtype = th.bfloat16 if (use_fp16 or use_bf16) else th.float32
        self.num_heads = num_heads
        self.num_head_channels = num_head_channels
        self.num_heads_upsample = num_heads_upsample
        self.attention_mode = attention_mode
        self.audio_attention = audio_attention
        self.dims = dims

        time_embed_dim = model_channels * 4
        self.time_embed = nn.Sequential(linear(model_channels, time_embed_dim), SiLU(),
                                        linear(time_embed_dim, time_embed_dim))
        if self.num_classes is not None:
            self.label_emb = nn.Embedding(num_classes, time_embed_dim)

        def res(ci, co):
            return ResBlock(ci, time_embed_dim, dropout, out_channels=co, dims=dims,
                            use_checkpoint=use_checkpoint,
                            use_scale_shift_norm=use_scale_shift_norm)

        def attn(ch, nh):
            return AttentionBlock(ch, use_checkpoint=use_checkpoint, num_heads=nh,
                                  num_head_channels=num_head_channels,
                                  use_new_attention_order=use_new_attention_order,
                                  attention_mode=attention_mode,
                                  audio_attention=audio_attention,
                                  audio_context_dim=audio_context_dim)

        if resblock_updown:
            raise NotImplementedError("resblock_updown is not on the accelerated path")
        ch = input_ch = int(channel_mult[0] * model_channels)
        self.input_blocks = nn.ModuleList(
            [TimestepEmbedSequential(conv_nd(dims, in_channels, ch, 3, padding=1))])
        self._feature_size = ch
        input_block_chans = [ch]
        ds = 1
        for level, mult in enumerate(channel_mult):
            for _ in range(num_res_blocks):
                layers = [res(ch, int(mult * model_channels))]
                ch = int(mult * model_channels)
                if ds in attention_resolutions:
                    layers.append(attn(ch, num_heads))
                self.input_blocks.append(TimestepEmbedSequential(*layers))
                self._feature_size += ch
                input_block_chans.append(ch)
            if level != len(channel_mult) - 1:
                self.input_blocks.append(TimestepEmbedSequential(
                    Downsample(ch, conv_resample, dims=dims, out_channels=ch)))
                input_block_chans.append(ch)
                ds *= 2
                self._feature_size += ch
        self.middle_block = TimestepEmbedSequential(res(ch, ch), attn(ch, num_heads), res(ch, ch))
        self._feature_size += ch
        self.output_blocks = nn.ModuleList([])
        for level, mult in list(enumerate(channel_mult))[::-1]:
            for i in range(num_res_blocks + 1):
                ich = input_block_chans.pop()
                layers = [res(ch + ich, int(model_channels * mult))]
                ch = int(model_channels * mult)
                if ds in attention_resolutions:
                    layers.append(attn(ch, num_heads_upsample))
                if level and i == num_res_blocks:
                    layers.append(Upsample(ch, conv_resample, dims=dims, out_channels=ch))
                    ds //= 2
                self.output_blocks.append(TimestepEmbedSequential(*layers))
                self._feature_size += ch
        self.out = nn.Sequential(normalization(ch), SiLU(),
                                 zero_module(conv_nd(dims, input_ch, out_channels, 3, padding=1)))

    def convert_to_fp16(self):
        """unet.py:630-636 analogue: low-precision (bf16) activations, fp32 masters."""
        self.dtype = th.bfloat16

    def convert_to_fp32(self):
        self.dtype = th.float32

    def forward(self, x, timesteps, y=None, *, context=None):
        """unet.py:646-675; `context` = audio tokens [B*T, L, F] for the audio
        cross-attention branches (audio_attention=True, build extension)."""
        assert (y is not None) == (self.num_classes is not None), \
            "must specify y if and only if the model is class-conditional"
        hs = []
        emb = self.time_embed(timestep_embedding(timesteps, self.model_channels))
        if self.num_classes is not None:
            assert y.shape == (x.shape[0],)
            emb = emb + self.label_emb(y)
        h = ops.to_cl(x.type(self.dtype))
        emb = emb_table(self, emb)
        for module in self.input_blocks:
            h = module(h, emb, context)
            hs.append(h)
        h = self.middle_block(h, emb, context)
        for module in self.output_blocks:
            h = _CatFn.apply(h, hs.pop())
            h = module(h, emb, context)
        gn, conv = self.out[0], self.out[2]
        h = ops.group_norm_silu(h, gn.weight, gn.bias, gn.num_groups, gn.eps)
        h = ops.conv(h, conv.weight, conv.bias, conv.stride, conv.padding)
        return h.type(x.dtype).contiguous()
