"""Drop-in for video-generation/diffusion/noise_scheduler.py (HIP kernels), plus the
build's DDIM sampler."""
import _vdiff_path  # noqa: F401
from vdiff.schedulers import CosineNoiseScheduler, DDIMSampler  # noqa: F401
