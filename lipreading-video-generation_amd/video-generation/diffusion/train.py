"""Training entry point (drop-in for video-generation/diffusion/train.py) on MI355X.

    python train.py [--synthetic] [--dims 3 --frames 16 --image-size 128] ...
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 train.py ...

Defaults reproduce train.py:46-139: LinearNoiseScheduler(100, 0.00085, 0.012),
UNetAudio(128, 3, 64, 3, 2, (1,2,4), audio_feature_dim=768, projected_audio_dim=128),
Adam lr 1e-2, MSE on eps, batch 8, 10 epochs, state_dict saved every epoch.
Deliberate differences: t ~ U{0..num_timesteps-1} (the reference's randint(0, 500)
indexes a 100-entry table and crashes); one process per GPU with RCCL
gradient all-reduce instead of a single device; --synthetic clips when the
reference's /proj/... FrameItem pickle and decord/torchaudio stack are absent, or
--data <dir> for clips in the build's decoded-clip format (vdiff.data).
Initialisation is the reference's (zero_module layers included, unet.py:222-224, 306,
627) and wav2vec2 must load its pretrained weights (unet_audio.py:14) unless
--random-audio-encoder (or --resume, whose checkpoint carries them) is given;
--reinit-nonzero replaces the zero-initialised layers with seeded weights (benchmarks and
smoke runs only).
"""
import argparse
import os
import sys
import time

import torch

import _vdiff_path  # noqa: F401
from vdiff.ddp import broadcast_parameters, init_from_env
from vdiff.engine import Trainer, reinit_nonzero, synthetic_clip

from linear_noise_scheduler import LinearNoiseScheduler
from unet_audio import UNetAudio


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--synthetic", action="store_true", default=True)
    ap.add_argument("--data", default=None,
                    help="frame index (JSON lines, vdiff.data) over .vdclip files: real clips "
                         "instead of synthetic ones")
    ap.add_argument("--fix-audio-resample", action="store_true",
                    help="resample audio from the track's rate (the reference resamples from "
                         "orig_freq = channel count, dataset.py:53)")
    ap.add_argument("--dims", type=int, default=2, help="2 = reference per-frame, 3 = UNet3D")
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--image-size", type=int, default=128)
    ap.add_argument("--model-channels", type=int, default=64)
    ap.add_argument("--channel-mult", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--num-res-blocks", type=int, default=2)
    ap.add_argument("--attention-resolutions", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--attention-mode", default="joint",
                    choices=["joint", "spatial", "temporal", "spatial_temporal"])
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--batch-size", type=int, default=8, help="clips (dims=3) or frames per GPU")
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--steps-per-epoch", type=int, default=5000 // 8)
    ap.add_argument("--lr", type=float, default=1e-2)
    ap.add_argument("--num-timesteps", type=int, default=100)
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--freeze-audio-encoder", action="store_true")
    ap.add_argument("--audio-attention", action="store_true",
                    help="audio cross-attention branches in every attention block (build "
                         "extension; the reference conditions by concatenation only)")
    ap.add_argument("--ckpt", default="best_diffusion.pth")
    ap.add_argument("--resume", default=None, help="checkpoint with model/optimizer/step")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--random-audio-encoder", action="store_true",
                    help="random-init wav2vec2-base when its pretrained weights are absent")
    ap.add_argument("--reinit-nonzero", action="store_true",
                    help="seeded weights for the zero-initialised layers (smoke / bench only)")
    return ap.parse_args(argv)


def build_model(args):
    return UNetAudio(image_size=args.image_size, in_channels=3,
                     model_channels=args.model_channels, out_channels=3,
                     num_res_blocks=args.num_res_blocks,
                     attention_resolutions=tuple(args.attention_resolutions),
                     channel_mult=tuple(args.channel_mult), dropout=args.dropout,
                     dims=args.dims, audio_feature_dim=768, projected_audio_dim=128,
                     use_bf16=args.dtype == "bf16", attention_mode=args.attention_mode,
                     freeze_audio_encoder=args.freeze_audio_encoder,
                     audio_attention=args.audio_attention,
                     # True: the pretrained weights must load (raises when absent);
                     # False: architecture only (random init, or weights from --resume)
                     audio_encoder_pretrained=not (args.random_audio_encoder or args.resume))


def train(argv=None):
    args = parse(argv)
    rank, world, local = init_from_env()
    if not torch.cuda.is_available():
        raise RuntimeError("train.py runs on the MI355X kernels only (no CPU path); the CPU "
                           "restatement lives in oracle/ for testing")
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    torch.manual_seed(args.seed + rank)
    scheduler = LinearNoiseScheduler(num_timesteps=args.num_timesteps, beta_start=0.00085,
                                     beta_end=0.012)
    model = build_model(args)
    if args.reinit_nonzero:
        reinit_nonzero(model, seed=args.seed)
    model = model.to(device)
    broadcast_parameters(model)
    trainer = Trainer(model, scheduler, lr=args.lr)
    start_epoch = 0
    if args.resume:
        state = torch.load(args.resume, map_location=device, weights_only=True)
        model.load_state_dict(state["model"])
        trainer.opt.load_state_dict(state["optimizer"])
        start_epoch = int(state["epoch"]) + 1
    if rank == 0:
        print(f"Training on {device} x{world}: {sum(p.numel() for p in model.parameters()) / 1e6:.1f}"
              f" M params, dims={args.dims}, {args.attention_mode} attention, {args.dtype}")
    frames = args.frames if args.dims == 3 else 1
    batcher = None
    if args.data:
        from vdiff.data import ClipBatcher, load_frame_items
        items = load_frame_items(args.data)
        # DistributedSampler-equivalent: each rank draws from its own seed
        batcher = ClipBatcher(items, args.batch_size, frames, args.num_timesteps, device,
                              size=args.image_size, seed=args.seed * world + rank,
                              bug_compatible=not args.fix_audio_resample, dims=args.dims)
    loss = torch.zeros(())
    for epoch in range(start_epoch, args.epochs):
        t0 = time.time()
        loss_sum = torch.zeros((), device=device)  # the epoch's mean loss, summed on the device
        for step in range(args.steps_per_epoch):
            if batcher is not None:
                clip = batcher.next()
            else:
                clip = synthetic_clip(args.batch_size, frames, args.image_size,
                                      args.num_timesteps, device,
                                      seed=(epoch * 1000003 + step) * world + rank, dims=args.dims)
            loss = trainer.step(clip)
            loss_sum += loss
        trainer.check_finite()  # the device-side NaN/Inf record, read once per epoch
        if rank == 0:
            dt = time.time() - t0
            fps = world * args.batch_size * frames * args.steps_per_epoch / dt
            # the reference prints the epoch's last loss (train.py:136); the mean is added
            print(f"Finished epoch {epoch + 1} | Loss: {loss.item()} | mean "
                  f"{loss_sum.item() / args.steps_per_epoch:.5f} | {fps:.2f} frames/s", flush=True)
            torch.save(model.state_dict(), args.ckpt)
            torch.save({"model": model.state_dict(), "optimizer": trainer.opt.state_dict(),
                        "epoch": epoch}, args.ckpt + ".resume")
    if rank == 0:
        print("Done Training ...")
    return float(loss)


if __name__ == "__main__":
    train()
