"""UNetAudio: the audio + reference-image conditioned denoiser (reference
video-generation/diffusion/unet_audio.py), 2-D (reference) and 5-D (frame stacks).

Conditioning (unet_audio.py:52-61): wav2vec2 last hidden state -> mean over time ->
Linear+ReLU -> broadcast over (H, W); the reference image -> 1x1 conv (3->64, no
bias) -> nearest resize to (H, W); concat [x | image-cond | audio] (+ zero channel
padding to a multiple of 8) is written by one kernel (vd_cond_concat) straight into
the first conv's channels-last input.

5-D extension: image [B, 3, T, H, W]; one reference image per clip
broadcast over T; one audio window per output frame ([B*T, samples] or pre-pooled
features [B*T, F]) broadcast over (H, W).  With T = 1 / dims = 2 this is the
reference computation.

Audio cross-attention (north_star build extension, audio_attention=True): every attention
block adds a cross-attention branch whose queries are the video tokens and whose keys /
values are the (unpooled) wav2vec2 hidden states of the frame's audio window, 12 tokens
per 4000-sample window (vdiff.nn.AttentionBlock, ops.cross_attention).  Off by default:
the reference conditions by concatenation only.
"""
from __future__ import annotations

import os

import warnings

import torch
import torch as th
import torch.nn as nn

from . import ops
from .nn import Conv2d, Linear, UNetModel


class _WeightNormReduce(nn.Module):
    """w = g * v / ||v|| (norm over every dim but `dim`): the weight-norm parametrization of
    wav2vec2's positional conv (transformers Wav2Vec2PositionalConvEmbedding, dim = 2) as a
    plain reduction.  torch._weight_norm's last-dim kernel took 0.47 ms per call forward and
    0.47 ms backward on MI355X for the [768, 48, 128] weight (profiles/r02_train_kernel_stats_
    prepair.md); same math, same parameters (original0 = g, original1 = v)."""

    def __init__(self, dim):
        super().__init__()
        self.dim = dim

    def forward(self, weight_g, weight_v):
        dims = [d for d in range(weight_v.dim()) if d != self.dim]
        norm = weight_v.float().pow(2).sum(dim=dims, keepdim=True).sqrt()
        return (weight_v * (weight_g / norm)).to(weight_v.dtype)


def _mask_hidden_states(self, hidden_states, mask_time_indices=None, attention_mask=None):
    """transformers Wav2Vec2Model._mask_hidden_states (SpecAugment in training) with the
    same masks (the same numpy draws of _compute_mask_indices) applied by torch.where
    instead of a boolean index_put: the index_put's nonzero and the pageable mask upload made
    the host wait for the GPU at every train step (measured 6.6 ms of idle GPU per step in
    the wav2vec2 forward); the mask now goes up asynchronously from pinned memory."""
    from transformers.models.wav2vec2.modeling_wav2vec2 import _compute_mask_indices
    cfg = self.config
    if not getattr(cfg, "apply_spec_augment", True):
        return hidden_states
    B, L, Hd = hidden_states.size()
    dev = hidden_states.device

    def upload(m):
        t = torch.from_numpy(m) if not torch.is_tensor(m) else m
        if t.device.type == "cpu" and dev.type == "cuda":
            t = t.pin_memory().to(dev, non_blocking=True)
        return t.to(device=dev, dtype=torch.bool)

    if mask_time_indices is not None:
        mt = upload(mask_time_indices)
    elif cfg.mask_time_prob > 0 and self.training:
        mt = upload(_compute_mask_indices((B, L), mask_prob=cfg.mask_time_prob,
                                          mask_length=cfg.mask_time_length,
                                          attention_mask=attention_mask,
                                          min_masks=cfg.mask_time_min_masks))
    else:
        mt = None
    if mt is not None:
        hidden_states = torch.where(mt[..., None], self.masked_spec_embed.to(hidden_states.dtype),
                                    hidden_states)
    if cfg.mask_feature_prob > 0 and self.training:
        mf = upload(_compute_mask_indices((B, Hd), mask_prob=cfg.mask_feature_prob,
                                          mask_length=cfg.mask_feature_length,
                                          min_masks=cfg.mask_feature_min_masks))
        hidden_states = torch.where(mf[:, None, :], hidden_states.new_zeros(()), hidden_states)
    return hidden_states


def _patch_wav2vec2(model):
    """Host-overhead fixes that keep the math: weight norm as a reduction, SpecAugment
    masks without host syncs."""
    import types
    _swap_weight_norm(model)
    model._mask_hidden_states = types.MethodType(_mask_hidden_states, model)


def _swap_weight_norm(model):
    from torch.nn.utils.parametrizations import _WeightNorm
    for mod in model.modules():
        plist = getattr(getattr(mod, "parametrizations", None), "weight", None)
        if plist is None:
            continue
        for i, p in enumerate(plist):
            if isinstance(p, _WeightNorm):
                plist[i] = _WeightNormReduce(p.dim)


class Wav2Vec2Encoder(nn.Module):
    """unet_audio.py:10-18.  `pretrained=None` loads local weights if the HF cache has
    them (no network in this build) and otherwise builds wav2vec2-base from its config
    with random weights (architecture identical: hidden 768, 12 layers)."""

    def __init__(self, model_name="facebook/wav2vec2-base-960h", cache_dir=None, pretrained=None):
        super().__init__()
        from transformers import Wav2Vec2Config, Wav2Vec2Model
        model = None
        if pretrained is not False:
            try:
                model = Wav2Vec2Model.from_pretrained(model_name, cache_dir=cache_dir,
                                                      local_files_only=True)
            except Exception as e:  # no local weights
                if pretrained:
                    raise
                warnings.warn(f"wav2vec2 weights for {model_name!r} not available offline "
                              f"({type(e).__name__}); using a random-init wav2vec2-base")
        if model is None:
            model = Wav2Vec2Model(Wav2Vec2Config())
        _patch_wav2vec2(model)
        self.wav2vec2 = model

    def forward(self, audio_input):
        if isinstance(audio_input, dict):
            return self.wav2vec2(**audio_input, output_hidden_states=True).last_hidden_state
        return self.wav2vec2(audio_input).last_hidden_state


class AudioFeatureTransformer(nn.Module):
    """unet_audio.py:21-30: Linear + ReLU."""

    def __init__(self, input_dim, output_dim):
        super().__init__()
        self.transform = nn.Sequential(Linear(input_dim, output_dim), nn.ReLU())

    def forward(self, x):
        return self.transform(x)


class UNetAudio(UNetModel):
    """unet_audio.py:32-66, same constructor arguments (plus keyword-only
    extensions of UNetModel and `audio_encoder_pretrained` / `freeze_audio_encoder`)."""

    def __init__(self, image_size, in_channels, model_channels, out_channels, num_res_blocks,
                 attention_resolutions, image_cond=True, im_cond_input_ch=3, im_cond_output_ch=64,
                 dropout=0.1, channel_mult=(1, 2, 4), conv_resample=True, dims=2,
                 num_classes=None, use_checkpoint=False, use_fp16=False, num_heads=1,
                 num_head_channels=-1, num_heads_upsample=-1, use_scale_shift_norm=False,
                 resblock_updown=False, use_new_attention_order=False, audio_feature_dim=512,
                 projected_audio_dim=256, *, attention_mode="joint", use_bf16=False,
                 audio_encoder_pretrained=None, freeze_audio_encoder=False, audio_encoder=True,
                 audio_attention=False):
        super().__init__(image_size,
                         in_channels + projected_audio_dim + (im_cond_output_ch if image_cond else 0),
                         model_channels, out_channels, num_res_blocks, attention_resolutions,
                         dropout, channel_mult, conv_resample, dims, num_classes, use_checkpoint,
                         use_fp16, num_heads, num_head_channels, num_heads_upsample,
                         use_scale_shift_norm, resblock_updown, use_new_attention_order,
                         attention_mode=attention_mode, use_bf16=use_bf16,
                         audio_attention=audio_attention, audio_context_dim=audio_feature_dim)
        self.audio_encoder = Wav2Vec2Encoder(pretrained=audio_encoder_pretrained) \
            if audio_encoder else None
        if self.audio_encoder is not None and freeze_audio_encoder:
            self.audio_encoder.requires_grad_(False)
        self.audio_transformer = AudioFeatureTransformer(audio_feature_dim, projected_audio_dim)
        self.projected_audio_dim = projected_audio_dim
        self.image_size = image_size
        self.image_cond = image_cond
        self.x_channels = in_channels
        if self.image_cond:
            self.cond_conv_in = Conv2d(in_channels=im_cond_input_ch,
                                       out_channels=im_cond_output_ch, kernel_size=1, bias=False)

    def encode_audio(self, audio):
        """wav2vec2 states of each audio window: mean-pooled over time, [B*T, F] -- or, with
        audio_attention, the tokens themselves [B*T, L, F] (their mean is the pooled vector).
        `audio` is the processor dict ({'input_values': [B*T, samples]}) or already-encoded
        features / tokens (lets a sampler encode the audio once instead of at every step)."""
        F_ = self.audio_transformer.transform[0].in_features
        if th.is_tensor(audio) and audio.shape[-1] == F_:
            return audio
        if self.audio_encoder is None:
            raise ValueError("model built without an audio encoder: pass encoded features")
        if (self.dtype == th.bfloat16 and next(self.audio_encoder.parameters()).is_cuda
                and os.environ.get("VDIFF_W2V_BF16")):
            # opt-in bf16 wav2vec2: GEMMs / convs under autocast, fp32
            # master weights and pooled output.  Off by default: same-box A/B of the
            # train step measured 427-429 ms with it against 423-424 without (MIOpen's
            # bf16 convolutions for the feature extractor are slower than its fp32 ones)
            with th.autocast("cuda", dtype=th.bfloat16):
                tokens = self.audio_encoder(audio).float()
        else:
            tokens = self.audio_encoder(audio)
        return tokens if self.audio_attention else tokens.mean(dim=1)

    def forward(self, image, cond_image, audio, timesteps, y=None):
        B = image.shape[0]
        T = image.shape[2] if image.dim() == 5 else 1
        enc = self.encode_audio(audio).float()
        tokens = enc if enc.dim() == 3 else None
        if self.audio_attention and tokens is None:
            raise ValueError("audio_attention needs the audio tokens [B*T, L, F], not pooled "
                             "features")
        feats = tokens.mean(dim=1) if tokens is not None else enc
        a = self.audio_transformer(feats).reshape(B, T, self.projected_audio_dim)
        if self.image_cond:
            imc = self.cond_conv_in(cond_image.type(self.dtype) if cond_image.dim() == 4
                                    else cond_image[:, :, 0].type(self.dtype))
        else:
            imc = image.new_zeros(B, 0, 1, 1)
        x = ops.cond_concat(image.type(self.dtype), imc, a, cpad=(self.in_channels + 7) // 8 * 8)
        ctx = tokens if self.audio_attention else None
        return self._unet_forward_padded(x, timesteps, y, image.dtype, ctx)

    def _unet_forward_padded(self, x, timesteps, y, out_dtype, context=None):
        # The concat buffer carries zero padding channels up to a multiple of 8; the
        # first conv's weight is zero-extended to match (same result as the reference
        # 195-channel conv, no extra pad copy).
        first = self.input_blocks[0][0]
        w = first.weight
        if x.shape[1] != w.shape[1]:
            w = th.nn.functional.pad(w, [0] * (2 * (w.dim() - 2)) + [0, x.shape[1] - w.shape[1]])
        assert y is None or self.num_classes is not None
        hs = []
        emb = self.time_embed(ops.timestep_embedding(timesteps, self.model_channels))
        if self.num_classes is not None:
            emb = emb + self.label_emb(y)
        h = ops.conv(x, w, first.bias, first.stride, first.padding)
        hs.append(h)
        from .nn import emb_table
        emb = emb_table(self, emb)
        for module in list(self.input_blocks)[1:]:
            h = module(h, emb, context)
            hs.append(h)
        h = self.middle_block(h, emb, context)
        from .nn import _CatFn
        for module in self.output_blocks:
            h = _CatFn.apply(h, hs.pop())
            h = module(h, emb, context)
        gn, conv = self.out[0], self.out[2]
        h = ops.group_norm_silu(h, gn.weight, gn.bias, gn.num_groups, gn.eps)
        h = ops.conv(h, conv.weight, conv.bias, conv.stride, conv.padding)
        return h.type(out_dtype).contiguous()
