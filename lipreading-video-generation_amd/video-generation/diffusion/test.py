"""Sampling entry point (drop-in for video-generation/diffusion/test.py) on MI355X.

    python test.py [--ckpt model.pth | --random-init] [--sampler ddpm-v2|ddim] [--steps 500]

Reference API kept (importable without running anything, unlike the reference script):
  * `config` -- the dict of test.py:33-49 (same keys; `ldm_params` may also carry the
    build's `dims` / `frames` / `attention_mode` / `dtype`);
  * `load_model_and_scheduler(config)` -- test.py:86-113: UNetAudio(128, 3, 64, 3, 2,
    (1,2,4), audio_feature_dim=768, projected_audio_dim=128), state_dict from
    config['train_params']['ldm_ckpt_name'], LinearNoiseSchedulerV2(500, 5e-5, 0.015);
  * `sample_images(model, scheduler, img_cond, audio_cond, n_timesteps=500)` --
    test.py:51-83: DDPM-V2 ancestral sampling from N(0, 1) over n_timesteps, x0 saved as
    PNG every 50 steps into lipreading_generated_images/ (plus .npy); returns the final x0
    (the reference returns None).

Deliberate differences: no nn.DataParallel wrapper (test.py:101; multi-GPU sampling runs
one process per GPU) and no per-step torch.cuda.empty_cache() (test.py:58); the audio is
encoded once per clip, not at every step.  A reference checkpoint carries the wav2vec2
weights (train.py:137 saves the whole UNetAudio), so with a checkpoint the encoder is built
from its config only; without one the model gets seeded smoke weights and a random
wav2vec2 -- only when asked for (`ldm_ckpt_name` None here, or --random-init).
Conditioning comes from --cond-npz (reference image [3, H, W] and audio [T, 4000]) or is
synthetic (the reference reads a /proj/... dataset item).
"""
import argparse
import os
import warnings

import numpy as np
import torch

import _vdiff_path  # noqa: F401
from vdiff.engine import reinit_nonzero, sample_ddim, synthetic_clip
from vdiff.ops import frozen_weights

from linear_noise_scheduler import LinearNoiseSchedulerV2
from noise_scheduler import DDIMSampler
from unet_audio import UNetAudio

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")

config = {
    "dataset_params": {"im_path": "/path/to/data", "im_size": 128, "im_channels": 3,
                       "frame_rate": 30},
    "ldm_params": {"model_channels": 64, "num_res_blocks": 2, "attention_resolutions": (1, 2, 4),
                   "z_channels": 3},
    # the reference points at a /proj/... checkpoint; None = seeded smoke weights
    "train_params": {"ldm_ckpt_name": None},
}

OUT_DIR = "lipreading_generated_images"


def _strip_module(sd):
    """Accept checkpoints saved from an nn.DataParallel wrapper ("module." keys)."""
    if sd and all(k.startswith("module.") for k in sd):
        return {k[len("module."):]: v for k, v in sd.items()}
    return sd


def load_model_and_scheduler(config, *, seed=0):
    """test.py:86-113."""
    lp = config["ldm_params"]
    ckpt = config["train_params"].get("ldm_ckpt_name")
    model = UNetAudio(
        image_size=config["dataset_params"]["im_size"],
        in_channels=lp["z_channels"],
        model_channels=lp["model_channels"],
        out_channels=config["dataset_params"]["im_channels"],
        num_res_blocks=lp["num_res_blocks"],
        attention_resolutions=lp["attention_resolutions"],
        audio_feature_dim=768,
        projected_audio_dim=128,
        dims=lp.get("dims", 2),
        attention_mode=lp.get("attention_mode", "joint"),
        use_bf16=lp.get("dtype", "bf16") == "bf16",
        audio_attention=lp.get("audio_attention", False),
        # with a checkpoint the wav2vec2 weights come from it; without one the random
        # encoder is the explicitly requested smoke mode
        audio_encoder_pretrained=False)
    if ckpt:
        sd = torch.load(ckpt, map_location="cpu", weights_only=True)
        model.load_state_dict(_strip_module(sd))
    else:
        warnings.warn("test.py: no checkpoint (ldm_ckpt_name is None): seeded smoke weights "
                      "and a random-init wav2vec2")
        reinit_nonzero(model, seed=seed)
    model = model.to(device)
    scheduler = LinearNoiseSchedulerV2(num_timesteps=500, beta_start=0.00005, beta_end=0.015)
    return model, scheduler


def save_frame(x0, path):
    """x0 in [-1, 1] -> (x0 + 1) / 2 as .npy and, for the first frame, .png (test.py:71-81).
    The PNG quantises as transforms.ToPILImage does (mul(255) then truncation to uint8); the
    clamp to [-1, 1] is a documented difference (the reference lets out-of-range values wrap
    in .byte())."""
    ims = ((x0.float().clamp(-1, 1) + 1) / 2).cpu().numpy()
    np.save(path + ".npy", ims)
    try:
        from PIL import Image
        img = ims[0] if ims.ndim == 4 else ims[0][:, 0]
        Image.fromarray((img.transpose(1, 2, 0) * 255).astype(np.uint8)).save(path + ".png")
    except ImportError:
        pass


def _frames_of(model, audio_cond):
    """Frames to generate: 1 for the reference 2-D model; for dims=3 one per audio window."""
    if getattr(model, "dims", 2) != 3:
        return None
    a = audio_cond["input_values"] if isinstance(audio_cond, dict) else audio_cond
    return a.shape[0]


@torch.no_grad()
def sample_images(model, scheduler, img_cond, audio_cond, n_timesteps=500, *, out_dir=OUT_DIR,
                  save_every=50, generator=None, noise=None, max_steps=None, callback=None):
    """test.py:51-83: reverse process i = n_timesteps-1 .. 0 with
    scheduler.sample_prev_timestep (LinearNoiseSchedulerV2 in test.py), x0 saved every
    `save_every` steps and at i == 0; returns the final x0.

    Keyword-only extensions: `noise(shape)` supplies x_T and each step's z instead of
    torch.randn (injected noise: the trajectory parity tests); `max_steps` stops after that
    many steps; `callback(i, xt, x0)` sees every step's output."""
    model.eval()
    dev = img_cond.device
    S = config["dataset_params"]["im_size"]
    T = _frames_of(model, audio_cond)
    shape = (1, 3, S, S) if T is None else (1, 3, T, S, S)
    os.makedirs(out_dir, exist_ok=True)
    draw = noise or (lambda shp: torch.randn(shp, generator=generator, device=dev))
    feats = model.encode_audio(audio_cond)  # once per clip (the reference: every step)
    xt = draw(shape).to(dev)
    x0 = None
    with frozen_weights():  # packed conv weights reused across the steps
        for k, i in enumerate(reversed(range(n_timesteps))):
            if max_steps is not None and k == max_steps:
                break
            t = torch.tensor([i], dtype=torch.long, device=dev)
            eps = model(xt, img_cond, feats, t)
            z = draw(xt.shape).to(dev)
            xt, x0 = scheduler.sample_prev_timestep(xt, eps, t, z=z)
            if callback is not None:
                callback(i, xt, x0)
            if (i + 1) % save_every == 0 or i == 0:
                save_frame(x0, os.path.join(out_dir, f"x0_{i}"))
    print("All images have been processed and saved.")
    return x0


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--ckpt", default=None)
    ap.add_argument("--random-init", action="store_true",
                    help="no checkpoint: seeded smoke weights and a random wav2vec2")
    ap.add_argument("--sampler", default="ddpm-v2", choices=["ddpm-v2", "ddim"])
    ap.add_argument("--steps", type=int, default=None, help="500 (ddpm-v2) / 50 (ddim)")
    ap.add_argument("--dims", type=int, default=2)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--image-size", type=int, default=config["dataset_params"]["im_size"])
    ap.add_argument("--attention-mode", default="joint")
    ap.add_argument("--audio-attention", action="store_true",
                    help="audio cross-attention branches (build extension)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--out-dir", default=OUT_DIR)
    ap.add_argument("--cond-npz", default=None)
    ap.add_argument("--save-every", type=int, default=50)
    ap.add_argument("--seed", type=int, default=0)
    return ap.parse_args(argv)


def main(argv=None):
    args = parse(argv)
    if not torch.cuda.is_available():
        raise RuntimeError("test.py runs on the MI355X kernels only")
    if not args.ckpt and not args.random_init:
        raise SystemExit("test.py: pass --ckpt <state_dict> (the reference loads "
                         "ldm_ckpt_name) or --random-init for seeded smoke weights")
    global device
    device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(device)
    cfg = {k: dict(v) for k, v in config.items()}
    cfg["dataset_params"]["im_size"] = args.image_size
    cfg["ldm_params"].update(dims=args.dims, attention_mode=args.attention_mode,
                             dtype=args.dtype, audio_attention=args.audio_attention)
    cfg["train_params"]["ldm_ckpt_name"] = args.ckpt
    config.update(cfg)
    model, scheduler = load_model_and_scheduler(config, seed=args.seed)
    frames = args.frames if args.dims == 3 else 1
    if args.cond_npz:
        z = np.load(args.cond_npz, allow_pickle=False)
        cond = torch.from_numpy(z["image"]).float()[None].to(device)
        audio = {"input_values": torch.from_numpy(z["audio"]).float().to(device)}
    else:
        clip = synthetic_clip(1, frames, args.image_size, 500, device, seed=args.seed,
                              dims=args.dims)
        cond, audio = clip.cond, clip.audio
    g = torch.Generator(device=device).manual_seed(args.seed)
    if args.sampler == "ddim":
        os.makedirs(args.out_dir, exist_ok=True)
        shape = (1, 3, frames, args.image_size, args.image_size) if args.dims == 3 else \
            (1, 3, args.image_size, args.image_size)
        sampler = DDIMSampler(scheduler, steps=args.steps or 50)

        def cb(i, xt, x0):
            if (i + 1) % args.save_every == 0 or i == sampler.steps - 1:
                save_frame(x0, os.path.join(args.out_dir, f"x0_{i}"))

        _, x0 = sample_ddim(model, sampler, cond, audio, shape, generator=g, callback=cb)
        print("All images have been processed and saved.")
        return x0
    return sample_images(model, scheduler, cond, audio, n_timesteps=args.steps or 500,
                         out_dir=args.out_dir, save_every=args.save_every, generator=g)


if __name__ == "__main__":
    main()
