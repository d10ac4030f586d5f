"""Drop-in for video-generation/diffusion/linear_noise_scheduler.py (HIP kernels)."""
import _vdiff_path  # noqa: F401
from vdiff.schedulers import LinearNoiseScheduler, LinearNoiseSchedulerV2  # noqa: F401
