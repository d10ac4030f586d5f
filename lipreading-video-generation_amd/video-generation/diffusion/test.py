"""Sampling entry point (drop-in for video-generation/diffusion/test.py) on MI355X.

    python test.py [--ckpt model.pth] [--sampler ddpm-v2|ddim] [--steps 500] [--dims 3]

Defaults reproduce test.py:33-152: UNetAudio(128, 3, 64, 3, 2, (1,2,4), 768, 128),
LinearNoiseSchedulerV2(500, 5e-5, 0.015) ancestral sampling over 500 steps, x0
written every 50 steps.  Differences: no per-step torch.cuda.empty_cache() (test.py:58)
and the audio is encoded once per clip, not at every step; --sampler ddim runs the
build's 50-step DDIM; conditioning is synthetic unless --cond-npz gives a reference
image [3, H, W] and audio [T, 4000] (the reference reads a /proj/... dataset item).
Outputs are .npy (and .png when Pillow is importable).
"""
import argparse
import os

import numpy as np
import torch

import _vdiff_path  # noqa: F401
from vdiff.engine import reinit_nonzero, sample_ddim, sample_ddpm, synthetic_clip

from linear_noise_scheduler import LinearNoiseSchedulerV2
from noise_scheduler import DDIMSampler
from unet_audio import UNetAudio

config = {
    "dataset_params": {"im_size": 128, "im_channels": 3, "frame_rate": 30},
    "ldm_params": {"model_channels": 64, "num_res_blocks": 2, "attention_resolutions": (1, 2, 4),
                   "z_channels": 3},
    "train_params": {"ldm_ckpt_name": None},
}


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--ckpt", default=None)
    ap.add_argument("--sampler", default="ddpm-v2", choices=["ddpm-v2", "ddim"])
    ap.add_argument("--steps", type=int, default=None, help="500 (ddpm-v2) / 50 (ddim)")
    ap.add_argument("--dims", type=int, default=2)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--image-size", type=int, default=config["dataset_params"]["im_size"])
    ap.add_argument("--attention-mode", default="joint")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--out-dir", default="lipreading_generated_images")
    ap.add_argument("--cond-npz", default=None)
    ap.add_argument("--save-every", type=int, default=50)
    ap.add_argument("--seed", type=int, default=0)
    return ap.parse_args(argv)


def load_model_and_scheduler(cfg, args, device):
    """test.py:86-113."""
    model = UNetAudio(image_size=args.image_size,
                      in_channels=cfg["ldm_params"]["z_channels"],
                      model_channels=cfg["ldm_params"]["model_channels"],
                      out_channels=cfg["dataset_params"]["im_channels"],
                      num_res_blocks=cfg["ldm_params"]["num_res_blocks"],
                      attention_resolutions=cfg["ldm_params"]["attention_resolutions"],
                      audio_feature_dim=768, projected_audio_dim=128, dims=args.dims,
                      use_bf16=args.dtype == "bf16", attention_mode=args.attention_mode)
    if args.ckpt:
        model.load_state_dict(torch.load(args.ckpt, map_location="cpu", weights_only=True))
    else:
        reinit_nonzero(model, seed=args.seed)
    scheduler = LinearNoiseSchedulerV2(num_timesteps=500, beta_start=0.00005, beta_end=0.015)
    return model.to(device), scheduler


def save_frame(x0, path):
    ims = ((x0.float().clamp(-1, 1) + 1) / 2).cpu().numpy()
    np.save(path + ".npy", ims)
    try:
        from PIL import Image
        img = ims[0] if ims.ndim == 4 else ims[0][:, 0]
        Image.fromarray((img.transpose(1, 2, 0) * 255).astype(np.uint8)).save(path + ".png")
    except ImportError:
        pass


def main(argv=None):
    args = parse(argv)
    if not torch.cuda.is_available():
        raise RuntimeError("test.py runs on the MI355X kernels only")
    device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(device)
    os.makedirs(args.out_dir, exist_ok=True)
    model, scheduler = load_model_and_scheduler(config, args, device)
    frames = args.frames if args.dims == 3 else 1
    if args.cond_npz:
        z = np.load(args.cond_npz, allow_pickle=False)
        cond = torch.from_numpy(z["image"]).float()[None].to(device)
        audio = {"input_values": torch.from_numpy(z["audio"]).float().to(device)}
    else:
        clip = synthetic_clip(1, frames, args.image_size, 500, device, seed=args.seed,
                              dims=args.dims)
        cond, audio = clip.cond, clip.audio
    shape = (1, 3, frames, args.image_size, args.image_size) if args.dims == 3 else \
        (1, 3, args.image_size, args.image_size)
    g = torch.Generator(device=device).manual_seed(args.seed)

    def cb(i, xt, x0):
        if (i + 1) % args.save_every == 0 or i == 0:
            save_frame(x0, os.path.join(args.out_dir, f"x0_{i}"))

    if args.sampler == "ddim":
        sampler = DDIMSampler(scheduler, steps=args.steps or 50)
        xt, x0 = sample_ddim(model, sampler, cond, audio, shape, generator=g, callback=cb)
    else:
        xt, x0 = sample_ddpm(model, scheduler, cond, audio, shape, n_timesteps=args.steps,
                             generator=g, callback=cb)
    print("All images have been processed and saved.")
    return x0


if __name__ == "__main__":
    main()
