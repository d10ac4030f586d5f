"""vdiff -- MI355X-native video-diffusion denoiser hot path (gfx950 HIP kernels behind a
C-ABI, PyTorch-ROCm for memory/streams/torch.distributed).

Drop-in for the reference's video-generation/diffusion Python API: see
lipreading-video-generation_amd/video-generation/diffusion/*.py for the flat module
names (unet, unet_audio, utils, linear_noise_scheduler, noise_scheduler).
"""
from . import _lib, ops  # noqa: F401
from .nn import (AttentionBlock, Downsample, GroupNorm32, QKVAttention,  # noqa: F401
                 QKVAttentionLegacy, ResBlock, TimestepBlock, TimestepEmbedSequential, UNetModel,
                 Upsample, conv_nd, linear, normalization, timestep_embedding, zero_module)
from .schedulers import (CosineNoiseScheduler, DDIMSampler, LinearNoiseScheduler,  # noqa: F401
                         LinearNoiseSchedulerV2)

__version__ = "0.1.0"
