"""Drop-in for video-generation/diffusion/utils.py on libvdiff (MI355X).

NN utilities map to vdiff.nn.  The reference's GPU picker (utils.py:13-46) shells out
to nvidia-smi; here the device comes from torchrun's LOCAL_RANK (one process per GPU)
and nothing is ever shelled out.
"""
import os

import torch

import _vdiff_path  # noqa: F401
from vdiff.nn import (CheckpointFunction, GroupNorm32, SiLU, avg_pool_nd,  # noqa: F401
                      checkpoint, conv_nd, linear, mean_flat, normalization, scale_module,
                      timestep_embedding, update_ema, zero_module)


def query_gpu_usage():
    """[(index, utilization %, memory used MiB)] for the visible devices (utilization is
    not exposed through torch; reported as 0)."""
    out = []
    for i in range(torch.cuda.device_count()):
        free, total = torch.cuda.mem_get_info(i)
        out.append((i, 0, (total - free) // 2 ** 20))
    return out


def select_gpus(max_util=10, max_mem=500, max_gpus=8):
    return [str(i) for i, _, _ in query_gpu_usage()][:max_gpus]


def set_visible_devices():
    """Pick this process's GPU: LOCAL_RANK under torchrun, else device 0."""
    if not torch.cuda.is_available():
        raise RuntimeError("No available GPU found!")
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
