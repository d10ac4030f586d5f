"""Drop-in for video-generation/diffusion/unet.py on libvdiff (MI355X).

UNetModel, ResBlock, AttentionBlock, QKVAttention(Legacy), Upsample, Downsample,
TimestepBlock and TimestepEmbedSequential keep the reference constructors and
state-dict keys; forwards run on the HIP kernels.  Not on the reference's entry paths
and not provided: AttentionPool2d, EncoderUNetModel, the thop FLOP hook.
"""
import torch
import torch.nn.functional as F

import _vdiff_path  # noqa: F401
from vdiff.nn import (AttentionBlock, Downsample, QKVAttention, QKVAttentionLegacy,  # noqa: F401
                      ResBlock, TimestepBlock, TimestepEmbedSequential, UNetModel, Upsample)
from vdiff.unet_audio import Wav2Vec2Encoder  # noqa: F401


class SuperResModel(UNetModel):
    """unet.py:678-692: UNet conditioned on a bilinearly upsampled low-res image."""

    def __init__(self, image_size, in_channels, *args, **kwargs):
        super().__init__(image_size, in_channels * 2, *args, **kwargs)

    def forward(self, x, timesteps, low_res=None, **kwargs):
        upsampled = F.interpolate(low_res, x.shape[2:], mode="bilinear")
        return super().forward(torch.cat([x, upsampled], dim=1), timesteps, **kwargs)
