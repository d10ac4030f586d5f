#!/usr/bin/env python3
"""Benchmark: train-step frames/sec + DDIM steps/sec, 128x128x16 UNet3D (BASELINE.json).

    python bench.py --gpus N --steps K --warmup W
    N > 1 without a launcher: the process starts `python -m torch.distributed.run
    --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py ...`
    itself (before anything touches the GPU) and exits with its status; under an external
    launcher WORLD_SIZE must equal --gpus.  VDIFF_DIST_BACKEND=gloo rehearses N ranks on
    fewer GPUs (ranks share GPUs round-robin).

Workload (BASELINE config 2/3): the audio + reference-image conditioned UNet3D of
train.py:88-97 with dims=3 (model_channels 64, mult (1,2,4), 2 res blocks,
attention at every level, 1 head, 195 input channels), joint attention over all
T*H*W tokens (the reference semantics), bf16 activations / fp32 master weights,
dropout 0.1 in train mode, random-init wav2vec2-base audio encoder (trainable, as
the reference), Adam at --lr (default 1e-4, the rate at which this model learns: train.py:102
uses 1e-2, at which the loss spikes and the network collapses to outputting 0, and at 1e-3 it
also stays at the output-0 loss; the kernels then run faster on the collapsing operands --
DESIGN section 5).  One synthetic clip [1, 3, 16, 128, 128] (+16 audio
windows of 4000 samples) per GPU and step -- a bank of distinct clips with their own noise and
timestep, generated on the device before timing (train.py:122-125 draws new ones each step).  A step = q_sample
+ forward + MSE + backward + RCCL gradient all-reduce + Adam.  Weak scaling.

Secondary: DDIM steps/sec = one 50-step-DDIM denoising step (UNet forward at
B=1 + DDIM update) on the same model, audio encoded once per clip.

roofline: the flash-attention UNIT with the largest share of the timed train step
(the forward launch, or the dQ + dK/dV launch pair of the backward), timed per launch
with HIP events on its launch stream; FLOP per unit is the algorithmic count of SURVEY
8(d) (vdiff.flops.attention_unit_flops: forward 4 N^2 D, backward 8 N^2 D, no credit
for recompute; executed_frac counts the products the kernels run); peak = 2.5 PF/s
bf16 dense (MI355X_MICROARCH.md).  traffic: HBM bytes per unit from the committed
rocprofv3 PMC summary (profiles/pmc_traffic.json) if present, else null.
cpu_baseline: the oracle (fp32 torch-CPU restatement of the reference) train step
timed on the host cores as BASELINE.md section 3 plans -- the config-2 model in
spatial_temporal mode on a bounded 2-frame clip, and config 1 (tiny UNet3D, joint);
no FLOP extrapolation (see "sample").
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0
PEAK_F32_TFLOPS = 157.3
METRIC = "train-step frames/sec + DDIM steps/sec, 128x128x16 UNet3D at 1/2/4/8 GPUs"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--clips-per-gpu", type=int, default=1)
    ap.add_argument("--mode", default="joint",
                    choices=["joint", "spatial", "temporal", "spatial_temporal"])
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--ddim-steps", type=int, default=None, help="timed DDIM steps (default: --steps)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-frames", type=int, default=2,
                    help="frames of the bounded CPU-baseline clip (config-2 model, "
                         "spatial_temporal)")
    ap.add_argument("--only", choices=["train", "ddim", "ddim_st", "vivit", "all"], default="all",
                    help="ddim_st: only the spatial_temporal DDIM leg (profiling)")
    ap.add_argument("--ddim-eager", action="store_true",
                    help="DDIM legs without the HIP-graph replay (A/B)")
    ap.add_argument("--vivit-steps", type=int, default=20,
                    help="timed ViViT fine-tune steps (BASELINE config 5); 0 skips the leg")
    ap.add_argument("--vivit-batch", type=int, default=16, help="clips per GPU (reference: 16)")
    ap.add_argument("--vivit-eager", action="store_true",
                    help="no HIP-graph capture of the ViViT step")
    ap.add_argument("--vivit-graph-ddp", action="store_true",
                    help="N > 1: graph replays around one all-reduce instead of the eager step "
                         "with the bucketed all-reduce (rehearsed over gloo only, so opt-in)")
    ap.add_argument("--xattn-steps", type=int, default=-1,
                    help="timed train steps with audio cross-attention (build extension, "
                         "auxiliary leg) after --warmup untimed ones, from the benchmark init "
                         "at --lr like the headline; -1 (default): --steps, so both legs time "
                         "the same step indices (the clock follows the weights, DESIGN 5); "
                         "0 skips it")
    ap.add_argument("--st-steps", type=int, default=-1,
                    help="timed train steps of the spatial_temporal leg (auxiliary: the build's "
                         "default attention mode, SURVEY D1) after --warmup untimed ones; -1: "
                         "--steps; 0 skips it")
    ap.add_argument("--train-graph", action="store_true",
                    help="auxiliary leg: graph-replayed train step paired with an eager one "
                         "(DESIGN section 9 item 3)")
    ap.add_argument("--timer-convs", action="store_true",
                    help="per-launch conv events inside the timed train steps too (the round-2 "
                         "measurement; A/B of the events' own cost)")
    ap.add_argument("--c4-steps", type=int, default=3,
                    help="timed DDIM steps at BASELINE config 4 (256x256x25); 0 skips the leg")
    ap.add_argument("--lr", type=float, default=1e-4,
                    help="Adam lr of the timed train steps.  train.py:102 uses 1e-2; from this "
                         "init the loss then spikes to 20-90 within 25 steps and reached NaN in "
                         "one of three runs (profiles/r04k_*, r04m_*); at 1e-2 and at 1e-3 the "
                         "model settles on the output-0 solution (mean loss 1.000 over 320 "
                         "steps) while at 1e-4 it learns (1.03 -> 0.73, profiles/"
                         "r05_train_curve.txt), and the chip's clock follows the operands "
                         "(one box: 48.8 frames/s at 1e-3, 46.9 at 1e-4, profiles/r05x_lr_ab.txt)"
                         ", so the headline trains at 1e-4")
    ap.add_argument("--init", choices=["nonzero", "reference"], default="nonzero",
                    help="train-leg init: 'nonzero' re-initialises the reference's zero_module "
                         "layers (engine.reinit_nonzero); 'reference' keeps train.py's init")
    return ap.parse_args()


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def seed_host(seed):
    """torch (CPU and device generators), numpy and random: the wav2vec2 encoder draws its
    SpecAugment masks and LayerDrop decisions from the host RNGs every step, so a run's loss
    sequence is reproducible only with all three seeded."""
    import random
    import numpy as np
    torch.manual_seed(seed)
    np.random.seed(seed % (2 ** 32))
    random.seed(seed)


def build_model(args, device, audio_attention=False, init=None):
    from vdiff.engine import reinit_nonzero
    from vdiff.unet_audio import UNetAudio
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        model = UNetAudio(image_size=args.size, in_channels=3, model_channels=64, out_channels=3,
                          num_res_blocks=2, attention_resolutions=(1, 2, 4),
                          audio_feature_dim=768, projected_audio_dim=128, dims=3,
                          use_bf16=args.dtype == "bf16", attention_mode=args.mode,
                          audio_encoder_pretrained=False, audio_attention=audio_attention,
                          dropout=float(os.environ.get("VDIFF_BENCH_DROPOUT", "0.1")))
    if (init or getattr(args, "init", "nonzero")) == "nonzero":
        reinit_nonzero(model, seed=1234)
    return model.to(device)


def clip_bank(args, n, device, seed):
    """n distinct synthetic train clips (x0, cond, audio, eps, t), generated on the device
    before the timed region (resident in HBM): each step trains on its own clip with its own
    noise and timestep, as the reference loop draws a new batch, torch.randn_like(im) and
    randint t every step (train.py:122-125)."""
    from vdiff.engine import synthetic_clip
    return [synthetic_clip(args.clips_per_gpu, args.frames, args.size, 100, device,
                           seed=seed * 1000 + i) for i in range(n)]


def ddim_stepper(args, model, sampler, cond, feats, xt):
    """One DDIM denoising step per call, i -> the update from sampler.timesteps[i]: the
    product's HIP-graph replay (vdiff.engine.DDIMGraph, as engine.sample_ddim runs it) or,
    with --ddim-eager, the eager UNet forward + sampler.step."""
    from vdiff.engine import DDIMGraph
    if not args.ddim_eager:
        return DDIMGraph(model, sampler, cond, feats, xt).step
    state = {"x": xt}

    def step(i):
        t = torch.full((xt.shape[0],), int(sampler.timesteps[i]), dtype=torch.int64,
                       device=xt.device)
        state["x"], _ = sampler.step(state["x"], model(state["x"], cond, feats, t), i)
    return step


def barrier_sync(world):
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
        torch.cuda.synchronize()


def max_over_ranks(x, world, device):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _pmc_traffic(keys):
    """HBM bytes per launch from the committed PMC summary (profiles/pmc_traffic.json),
    summed over `keys`; None unless every key is present."""
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(pmc) as f:
            tab = json.load(f)
        vals = [tab[k].get("hbm_bytes_per_launch") for k in keys]
    except (OSError, ValueError, KeyError):
        return None
    return None if any(v is None for v in vals) else sum(vals)


def pick_roofline(summary, dtype, pmc=True):
    """Per-kernel executed rates, then per-UNIT algorithmic rates: unit "fwd"
    = one forward launch (2 products); unit "bwd" = the dQ + dK/dV launch pair (4
    products: backward = 2x forward, recompute not credited).  The roofline object is the
    unit with the largest total time in the timed step."""
    from vdiff.flops import attention_kernel_flops, attention_unit_flops
    peak = PEAK_BF16_TFLOPS if dtype == "bf16" else PEAK_F32_TFLOPS
    rows, kern = [], {}
    for (kind, hd, n, nseq), (cnt, tot_ms) in summary.items():
        if n <= 32:  # the short-sequence kernels are HBM-bound: short_attention_roofline
            continue
        f = attention_kernel_flops(kind, n, hd, nseq)
        avg_s = tot_ms / cnt / 1e3
        kern[(kind, hd, n, nseq)] = (cnt, tot_ms)
        rows.append({"kernel": kind, "head_dim": hd, "seq_len": n, "nseq": nseq, "launches": cnt,
                     "total_ms": round(tot_ms, 3), "avg_ms": round(tot_ms / cnt, 4),
                     "executed_tflop_per_launch": round(f / 1e12, 4),
                     "executed_tflops": round(f / avg_s / 1e12, 1),
                     "executed_frac": round(f / avg_s / 1e12 / peak, 4)})
    rows.sort(key=lambda r: -r["total_ms"])
    units = []
    for (kind, hd, n, nseq), (cnt, tot) in kern.items():
        if kind == "attn_fwd":
            parts, unit = [(cnt, tot)], "fwd"
            ex = attention_kernel_flops("attn_fwd", n, hd, nseq)
        elif kind == "attn_bwd_dq" and ("attn_bwd_dkdv", hd, n, nseq) in kern:
            parts, unit = [(cnt, tot), kern[("attn_bwd_dkdv", hd, n, nseq)]], "bwd"
            ex = (attention_kernel_flops("attn_bwd_dq", n, hd, nseq)
                  + attention_kernel_flops("attn_bwd_dkdv", n, hd, nseq))
        else:
            continue
        avg_s = sum(t / c for c, t in parts) / 1e3  # one unit = one launch of each kernel
        f = attention_unit_flops(unit, n, hd, nseq)
        units.append({"unit": unit, "kernels": "attn_fwd" if unit == "fwd"
                      else "attn_bwd_dq + attn_bwd_dkdv", "head_dim": hd, "seq_len": n,
                      "nseq": nseq, "launches": parts[0][0],
                      "total_ms": round(sum(t for _, t in parts), 3),
                      "avg_ms": round(avg_s * 1e3, 4), "alg_tflop": round(f / 1e12, 4),
                      "tflops": round(f / avg_s / 1e12, 1),
                      "frac": round(f / avg_s / 1e12 / peak, 4),
                      "executed_frac": round(ex / avg_s / 1e12 / peak, 4)})
    units.sort(key=lambda r: -r["total_ms"])
    if not units:
        return None, rows, units
    top = units[0]
    names = ["attn_fwd"] if top["unit"] == "fwd" else ["attn_bwd_dq", "attn_bwd_dkdv"]
    # the committed PMC rows are per-launch bytes at the headline's joint shapes
    traffic = _pmc_traffic([f"{k}_d{top['head_dim']}" for k in names]) if pmc else None
    roof = {"bound": "mfma", "achieved": top["tflops"], "peak": peak, "unit": "TFLOP/s",
            "frac": top["frac"], "traffic": traffic, "executed_frac": top["executed_frac"],
            "kernel": f"{top['kernels']} (head_dim {top['head_dim']}, seq {top['seq_len']}, "
                      f"{top['nseq']} seq/launch)",
            "alg_flop_per_unit": top["alg_tflop"] * 1e12, "avg_unit_ms": top["avg_ms"],
            "note": "frac = algorithmic FLOP (SURVEY 8d: bwd = 2x fwd = 4 products, no "
                    "recompute credit) / the unit's summed per-launch kernel time / peak; "
                    "executed_frac counts the products the kernels run (bwd pair: 7)"}
    return roof, rows, units


def _oracle_train_rate(cfg, shape, mode, audio_dim, imc_dim, budget_s, max_steps):
    """Oracle fp32 train steps (q_sample + conditioning + fwd + MSE + bwd + Adam) at one
    clip shape on the host cores; wav2vec2 excluded (pooled features are an input).
    Returns (frames/s, steps, seconds)."""
    import torch.nn.functional as F
    from oracle.fixtures import seeded
    from oracle.unet import (audio_conditioned_input, audio_param_shapes, build_plan,
                             init_params, param_shapes, unet_forward)
    from oracle import schedulers as osch
    B, T, s = 1, shape[0], shape[1]
    plan = build_plan(**cfg, attention_mode=mode)
    P = init_params(param_shapes(plan), 1234)
    P.update(init_params(audio_param_shapes(768, audio_dim, im_cond_output_ch=imc_dim), 77))
    for v in P.values():
        v.requires_grad_(True)
    tab = osch.linear_tables(100, 0.00085, 0.012)
    x0 = seeded((B, 3, T, s, s), 0, "uniform")
    cond = seeded((B, 3, s, s), 1, "uniform")
    eps = seeded((B, 3, T, s, s), 2)
    feat = seeded((B * T, 768), 3)
    t = torch.tensor([37])
    opt = torch.optim.Adam(list(P.values()), lr=1e-2)
    t0, n = time.perf_counter(), 0
    while True:
        xt = osch.q_sample(tab, x0, eps, t)
        x = audio_conditioned_input(P, xt, cond, feat, audio_dim)
        F.mse_loss(unet_forward(P, plan, x, t), eps).backward()
        opt.step()
        opt.zero_grad()
        n += 1
        el = time.perf_counter() - t0
        if el > budget_s or n >= max_steps:
            break
    return n * B * T / el, n, el


def cpu_baseline(args):
    """The oracle (fp32 torch-CPU restatement of the reference path) train step, measured
    on the host cores as BASELINE.md section 3 plans -- no FLOP extrapolation:
      * value: config 2's model (full-width UNet3D, train.py:88-97, dims=3) at 128x128 in
        spatial_temporal mode, on a bounded 2-frame clip (per-frame work is independent of
        T in this mode; the unit is frames/s);
      * config1_tiny3d: BASELINE config 1 (tiny UNet3D, 64x64x8, joint attention).
    Joint attention at 128x128x16 is n/a on a CPU: the reference materialises a 262144^2
    fp32 score matrix (275 GB) per block."""
    from oracle.fixtures import FULL3D, TINY3D
    threads = torch.get_num_threads()
    c2 = {k: v for k, v in FULL3D.items()}
    fps2, n2, el2 = _oracle_train_rate(c2, (args.cpu_frames, args.size), "spatial_temporal",
                                       128, 64, budget_s=8.0, max_steps=3)
    c1 = {k: v for k, v in TINY3D.items()}
    fps1, n1, el1 = _oracle_train_rate(c1, (8, 64), "joint", 16, 16, budget_s=8.0, max_steps=3)
    return {"value": round(fps2, 5), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": (f"oracle fp32 train step (q_sample+cond+fwd+MSE+bwd+Adam, wav2vec2 "
                       f"excluded), config-2 model (full-width UNet3D) at {args.size}x{args.size}"
                       f", spatial_temporal attention, B=1 clip of {args.cpu_frames} frames: "
                       f"{n2} steps in {el2:.1f} s"),
            "joint": "n/a (262144^2 fp32 score matrix = 275 GB per block)",
            "config1_tiny3d": {"value": round(fps1, 4), "unit": "frames/s",
                               "sample": f"tiny UNet3D 64x64x8, joint: {n1} steps in "
                                         f"{el1:.1f} s"}}


def vivit_cpu_baseline(model, B):
    """The oracle (oracle/vivit.py, torch fp32 on the host cores) fine-tune step -- CE +
    backward + AdamW -- on the same config-5 batch shape, with the GPU model's weights."""
    import torch.nn.functional as F
    from oracle.vivit import vivit_classifier
    P = {k: v.detach().float().cpu().clone().requires_grad_(True)
         for k, v in model.state_dict().items()}
    opt = torch.optim.AdamW(list(P.values()), lr=1e-4)
    g = torch.Generator().manual_seed(7)
    x = torch.randn((B, 5, 1, 32, 32), generator=g)
    y = torch.randint(0, 40, (B,), generator=g)
    cfg = model.vit.config

    def step():
        loss = F.cross_entropy(vivit_classifier(P, x, cfg.num_attention_heads,
                                                cfg.num_hidden_layers), y)
        loss.backward()
        opt.step()
        opt.zero_grad()

    step()
    t0, n = time.perf_counter(), 0
    while True:
        step()
        n += 1
        el = time.perf_counter() - t0
        if el > 5.0 or n >= 50:
            break
    return {"value": round(n * B / el, 2), "unit": "clips/s", "cores": torch.get_num_threads(),
            "kind": "port", "sample": f"oracle fp32 fine-tune step (fwd+CE+bwd+AdamW), batch {B}, "
                                      f"{n} steps in {el:.1f} s"}


def vivit_leg(args, rank, world, device):
    """BASELINE config 5: ViViT lipreading fine-tune step (huggingface_vivit_model.py:35-60:
    CE + AdamW 1e-4, batch 16 per GPU, 5x1x32x32 clips, main.py:57 config with 5 frames),
    DDP over the same gradient bucketer; bf16 activations, fp32 master weights."""
    from vdiff.ddp import broadcast_parameters
    from vdiff.vivit import ViViT, VivitModel, VivitTrainer, lipreading_config, vivit_flops
    cfg = lipreading_config(num_frames=5)
    torch.manual_seed(4321)
    model = ViViT(VivitModel(cfg, use_bf16=args.dtype == "bf16"), 40, 5).to(device)
    broadcast_parameters(model)
    # one process: the whole step as one HIP graph.  N > 1: eager with the bucketed
    # all-reduce; --vivit-graph-ddp: forward + backward graph, ONE all-reduce of the flattened
    # gradients, AdamW graph (VivitTrainer) -- not yet run over RCCL (advisor r03)
    graph = not args.vivit_eager and (world == 1 or args.vivit_graph_ddp)
    tr = VivitTrainer(model, graph=graph)
    g = torch.Generator(device=device).manual_seed(300 + rank)
    B = args.vivit_batch
    x = torch.randn((B, 5, 1, 32, 32), generator=g, device=device)
    y = torch.randint(0, 40, (B,), generator=g, device=device)
    for _ in range(3):
        tr.step(x, y)
    barrier_sync(world)
    t0 = time.perf_counter()
    for _ in range(args.vivit_steps):
        loss = tr.step(x, y)
    barrier_sync(world)
    el = max_over_ranks(time.perf_counter() - t0, world, device)
    ms = el / args.vivit_steps * 1e3
    flop = 3 * vivit_flops(cfg, B)
    out = {"metric": "ViViT lipreading fine-tune clips/sec (BASELINE config 5)",
           "value": round(world * B * args.vivit_steps / el, 2), "unit": "clips/s",
           "ms_per_step": round(ms, 3), "batch_per_gpu": B, "clip": [5, 1, 32, 32],
           "tokens": 9, "hidden": cfg.hidden_size, "layers": cfg.num_hidden_layers,
           "heads": cfg.num_attention_heads, "train_tflop_per_step": round(flop / 1e12, 4),
           "model_tflops_per_gpu": round(flop / (el / args.vivit_steps) / 1e12, 2),
           "bound": "launch (9 tokens x 256 hidden: microsecond kernels)",
           "parallelism": f"dp{world}", "loss": _num(loss),
           "hip_graph": graph}
    if rank == 0 and world == 1 and not args.no_cpu:
        try:
            out["cpu_baseline"] = vivit_cpu_baseline(model, B)
        except Exception as e:  # never let the baseline leg kill the GPU numbers
            out["cpu_baseline"] = {"value": None, "error": f"{type(e).__name__}: {e}"}
    log(f"vivit: {ms:.2f} ms/step, {out['value']} clips/s")
    del tr, model
    torch.cuda.empty_cache()
    return out


def xattn_leg(args, rank, world, device, base_ms):
    """Auxiliary: the same train step with the audio cross-attention branches on
    (audio_attention=True, build extension): every attention block also attends from the
    video tokens to the 12 wav2vec2 tokens of each frame's audio window."""
    from vdiff.ddp import broadcast_parameters
    from vdiff.engine import Trainer, synthetic_clip
    from vdiff.flops import unet_forward_work
    from vdiff.schedulers import LinearNoiseScheduler
    seed_host(1234 + rank)
    model = build_model(args, device, audio_attention=True)
    broadcast_parameters(model)
    work = unet_forward_work(model, (args.clips_per_gpu, 195, args.frames, args.size, args.size))
    tr = Trainer(model, LinearNoiseScheduler(100, 0.00085, 0.012), lr=args.lr)
    nsteps = args.steps if args.xattn_steps < 0 else args.xattn_steps
    bank = clip_bank(args, args.warmup + nsteps, device, rank)
    losses = []
    for i in range(args.warmup):
        losses.append(tr.step(bank[i]))
    barrier_sync(world)
    t0 = time.perf_counter()
    for i in range(nsteps):
        losses.append(tr.step(bank[args.warmup + i]))
    barrier_sync(world)
    el = max_over_ranks(time.perf_counter() - t0, world, device)
    ms = el / nsteps * 1e3
    loss = losses[-1]
    out = {"metric": "train-step frames/sec with audio cross-attention (build extension)",
           "value": round(world * args.clips_per_gpu * args.frames * nsteps / el, 4),
           "steps": nsteps, "warmup": args.warmup,
           "train_losses": [_num(x, 5) for x in losses],
           "unit": "frames/s", "ms_per_step": round(ms, 2),
           "overhead_ms_vs_concat_only": round(ms - base_ms, 2) if base_ms else None,
           "fwd_tflop_per_clip": round(work.total / 1e12, 3), "audio_tokens_per_frame": 12,
           "loss": _num(loss)}
    log(f"xattn: {ms:.1f} ms/step")
    del tr, model
    torch.cuda.empty_cache()
    return out


PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 6.29 TB/s measured copy)


def short_attention_roofline(summary):
    """Per-kernel rows of the short-sequence (temporal, <= 32 tokens) attention launches in a
    timer summary: HBM-bound, so achieved = algorithmic bytes per launch
    (vdiff.flops.short_attention_bytes) / average launch time, against the HBM peak; plus the
    executed / algorithmic FLOP ratio (tile padding x recomputed products)."""
    from vdiff.flops import attention_kernel_flops, short_attention_bytes
    rows = []
    for (kind, hd, n, nseq), (cnt, tot_ms) in summary.items():
        if n > 32 or kind not in ("attn_fwd", "attn_bwd"):
            continue
        avg_s = tot_ms / cnt / 1e3
        nb = short_attention_bytes(kind, n, hd, nseq)
        lp = 16 if n <= 16 else 32
        ex = attention_kernel_flops(kind, lp, hd, nseq)
        alg = (2 if kind == "attn_fwd" else 4) * 2.0 * nseq * n * n * hd
        rows.append({"kernel": "short " + kind.replace("attn_", ""), "head_dim": hd, "seq_len": n,
                     "nseq": nseq, "launches": cnt, "total_ms": round(tot_ms, 3),
                     "avg_ms": round(tot_ms / cnt, 4), "alg_bytes": nb,
                     "achieved_gbs": round(nb / avg_s / 1e9, 1),
                     "frac": round(nb / avg_s / 1e9 / PEAK_HBM_GBS, 4),
                     "executed_over_algorithmic_flop": round(ex / alg, 3)})
    rows.sort(key=lambda r: -r["total_ms"])
    return rows


def st_leg(args, rank, world, device):
    """Auxiliary: the same train step in spatial_temporal mode (SURVEY D1 / BASELINE.md
    section 2, 'build default', ~29 TFLOP per step: spatial attention per frame over its
    H*W tokens on the flash kernels + temporal attention per pixel over its T tokens on the
    short-sequence kernels), from the benchmark init at --lr, the headline's step indices.
    Reports frames/s, the spatial attention units (MFMA roofline) and the temporal kernels
    (HBM roofline, short_attention_roofline)."""
    import copy as _copy
    from vdiff import ops
    from vdiff.ddp import broadcast_parameters
    from vdiff.engine import Trainer, synthetic_clip
    from vdiff.flops import unet_forward_work
    from vdiff.schedulers import LinearNoiseScheduler
    a2 = _copy.copy(args)
    a2.mode = "spatial_temporal"
    seed_host(1234 + rank)
    model = build_model(a2, device)
    broadcast_parameters(model)
    work = unet_forward_work(model, (args.clips_per_gpu, 195, args.frames, args.size, args.size))
    tr = Trainer(model, LinearNoiseScheduler(100, 0.00085, 0.012), lr=args.lr)
    nsteps = args.steps if args.st_steps < 0 else args.st_steps
    bank = clip_bank(args, args.warmup + nsteps, device, rank)
    losses = [tr.step(bank[i]) for i in range(args.warmup)]
    barrier_sync(world)
    timer = ops.KernelTimer(attention=True, convs=False)
    ops.set_timer(timer)
    t0 = time.perf_counter()
    for i in range(nsteps):
        losses.append(tr.step(bank[args.warmup + i]))
    barrier_sync(world)
    el = time.perf_counter() - t0
    ops.set_timer(None)
    el = max_over_ranks(el, world, device)
    ms = el / nsteps * 1e3
    summary = timer.summary()
    roof, _, units = pick_roofline(summary, args.dtype, pmc=False)
    short = short_attention_roofline(summary)
    step_flops = 3 * work.total * args.clips_per_gpu
    out = {"metric": "train-step frames/sec, spatial_temporal attention (build default mode)",
           "value": round(world * args.clips_per_gpu * args.frames * nsteps / el, 4),
           "unit": "frames/s", "ms_per_step": round(ms, 2), "steps": nsteps,
           "warmup": args.warmup, "train_losses": [_num(x, 5) for x in losses],
           "fwd_tflop_per_clip": round(work.total / 1e12, 3),
           "train_tflop_per_step": round(step_flops / 1e12, 2),
           "model_tflops_per_gpu": round(step_flops / (el / nsteps) / 1e12, 1),
           "roofline_spatial": roof, "attention_units": units,
           "roofline_temporal": ({"bound": "hbm", "achieved": short[0]["achieved_gbs"],
                                  "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": short[0]["frac"],
                                  "kernel": f"{short[0]['kernel']} (head_dim "
                                            f"{short[0]['head_dim']}, seq {short[0]['seq_len']},"
                                            f" {short[0]['nseq']} seq/launch)",
                                  "traffic": _pmc_traffic([short[0]["kernel"].replace(
                                      "short ", "short_attn_") + f"_d{short[0]['head_dim']}"])}
                                 if short else None),
           "temporal_kernels": short}
    log(f"spatial_temporal: {ms:.1f} ms/step, {out['value']} frames/s")
    for r in short:
        log("  temporal", r)
    del tr, model
    torch.cuda.empty_cache()
    return out


def ddim_st_leg(args, world, device, init_state, sampler, clip, kd):
    """The north-star forward in the factorised mode (VERDICT r05 missing #1): one DDIM
    denoising step (UNet3D forward at 128x128x16 in spatial_temporal mode, SURVEY D1 -- per-frame
    spatial attention over H*W tokens + per-pixel temporal attention over T tokens -- plus the
    DDIM update) replayed as the product's HIP graph, the same weights and inputs as the joint
    `ddim` leg.  frac = the forward's algorithmic FLOP (vdiff.flops.unet_forward_work) per second
    / the bf16 MFMA peak."""
    import copy as _copy
    from vdiff import ops
    from vdiff.flops import unet_forward_work
    a2 = _copy.copy(args)
    a2.mode = "spatial_temporal"
    model = build_model(a2, device)
    with torch.no_grad():
        # the shared weights of the joint leg; the temporal blocks (spatial_temporal only)
        # keep build_model's benchmark init
        miss = model.load_state_dict(init_state, strict=False)
    assert not miss.unexpected_keys and all(".temporal_" in k for k in miss.missing_keys), miss
    model.eval()
    work = unet_forward_work(model, (1, 195, args.frames, args.size, args.size))
    with torch.no_grad(), ops.frozen_weights():
        feats = model.encode_audio(clip.audio)
        xt = torch.randn_like(clip.x0)
        step = ddim_stepper(args, model, sampler, clip.cond, feats, xt)
        step(0)  # warm-up (and, graphed, the capture)
        barrier_sync(world)
        t0 = time.perf_counter()
        for i in range(1, 1 + kd):
            step(i)
        barrier_sync(world)
        el = max_over_ranks(time.perf_counter() - t0, world, device)
        del step
    tf = work.total / (el / kd) / 1e12
    peak = PEAK_BF16_TFLOPS if args.dtype == "bf16" else PEAK_F32_TFLOPS
    out = {"metric": "DDIM steps/sec, 128x128x16 UNet3D, spatial_temporal attention (SURVEY D1)",
           "value": round(world * kd / el, 4), "unit": "steps/s", "steps_timed": kd,
           "ms_per_step": round(el / kd * 1e3, 3),
           "fwd_tflop": round(work.total / 1e12, 3),
           "fwd_tflop_conv": round(work.conv / 1e12, 3),
           "fwd_tflop_attn": round(work.attn / 1e12, 3),
           "model_tflops_per_gpu": round(tf, 1), "peak": peak, "frac": round(tf / peak, 4),
           "hip_graph": not args.ddim_eager,
           "note": "frac = forward algorithmic FLOP / (ms per DDIM step) / peak; the step also "
                   "runs the DDIM update (HBM-bound, a few microseconds)"}
    log(f"ddim_st: {out['ms_per_step']} ms/step, {out['model_tflops_per_gpu']} TFLOP/s, "
        f"frac {out['frac']}")
    del model
    torch.cuda.empty_cache()
    return out


def _num(x, nd=4):
    """A float for the JSON line: None when not finite (NaN / Infinity are not JSON)."""
    x = float(x)
    return round(x, nd) if math.isfinite(x) else None


def graph_leg(args, device):
    """Auxiliary (one process): the train step with the denoiser's forward + backward replayed
    as one HIP graph (Trainer(graph=True), vdiff.engine.TrainStepGraph; wav2vec2 and Adam
    eager around it) against the eager step, PAIRED: two models from the same init, one per
    mode, stepped alternately on the same clip, so both see the same weights (the attention
    kernels' clock follows the operands) and the same box state.  max(3,
    warmup) untimed steps each (graph: two eager, the capture), then --steps timed steps each;
    per-step times are medians.  The headline `value` stays the eager step of the main leg,
    whose per-launch attention events the roofline needs."""
    import statistics
    from vdiff.engine import Trainer, synthetic_clip
    from vdiff.schedulers import LinearNoiseScheduler
    trainers = {}
    os.environ["VDIFF_TRAIN_GRAPH_EXPERIMENTAL"] = "1"  # --train-graph is the explicit opt-in
    for mode in ("eager", "graph"):
        torch.manual_seed(1234)
        model = build_model(args, device)
        # VDIFF_GRAPH_LEG_EAGER=1: both trainers eager (the run-to-run spread of the losses)
        graph = mode == "graph" and not os.environ.get("VDIFF_GRAPH_LEG_EAGER")
        trainers[mode] = Trainer(model, LinearNoiseScheduler(100, 0.00085, 0.012), lr=1e-2,
                                 graph=graph)
    clip = synthetic_clip(args.clips_per_gpu, args.frames, args.size, 100, device, seed=0)
    seq = {m: [] for m in trainers}
    for _ in range(max(3, args.warmup)):
        for m, tr in trainers.items():
            seq[m].append(tr.step(clip))
    times = {m: [] for m in trainers}
    torch.cuda.synchronize()
    for _ in range(args.steps):
        for m, tr in trainers.items():
            t0 = time.perf_counter()
            seq[m].append(tr.step(clip))
            torch.cuda.synchronize()
            times[m].append((time.perf_counter() - t0) * 1e3)
    med = {m: statistics.median(v) for m, v in times.items()}
    out = {"metric": "train-step ms, denoiser fwd+bwd as one HIP graph vs eager (paired)",
           "ms_per_step_graph": round(med["graph"], 2), "ms_per_step_eager": round(med["eager"], 2),
           "ms_saved": round(med["eager"] - med["graph"], 2),
           "value": round(args.clips_per_gpu * args.frames / (med["graph"] / 1e3), 4),
           "unit": "frames/s", "steps_timed": args.steps,
           "losses_graph": [_num(x) for x in seq["graph"]],
           "losses_eager": [_num(x) for x in seq["eager"]]}
    log(f"train graph vs eager (paired): {med['graph']:.1f} vs {med['eager']:.1f} ms/step")
    del trainers
    torch.cuda.empty_cache()
    return out


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n):
    """One process per GPU without an external launcher: run this same command line under
    torch.distributed.run (N local ranks, rendezvous on 127.0.0.1) as a CHILD process and
    return its exit status.  Called before anything in this process touches the GPU."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={free_port()}",
           os.path.abspath(__file__)] + sys.argv[1:]
    log(f"spawning {n} ranks: {' '.join(cmd)}")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def comm_report(trainer, world, device, steps):
    """Gradient exchange of the timed steps: bytes, RCCL world size, the exposed all-reduce
    time per step (end of backward -> averaged buckets, max over ranks), the same exchange
    issued alone, and the fraction of it hidden under the backward."""
    bk = trainer.bucketer
    exposed = bk.comm_times_ms()
    exp_ms = max_over_ranks(sum(exposed) / max(len(exposed), 1), world, device)
    alone = max_over_ranks(bk.standalone_allreduce_ms(), world, device)
    return {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
            "grad_mbytes": round(bk.nbytes / 2 ** 20, 1), "buckets": len(bk.buckets),
            "exposed_ms_per_step": round(exp_ms, 3), "standalone_ms_per_step": round(alone, 3),
            "hidden_frac": round(1.0 - exp_ms / alone, 3) if alone > 0 else None,
            "steps": len(exposed)}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    from vdiff import ops
    from vdiff.ddp import broadcast_parameters, init_from_env
    from vdiff.engine import Trainer, synthetic_clip
    from vdiff.flops import unet_forward_work
    from vdiff.schedulers import DDIMSampler, LinearNoiseScheduler, LinearNoiseSchedulerV2

    rank, world, local = init_from_env()
    if world != args.gpus:
        log(f"error: --gpus {args.gpus} but WORLD_SIZE {world}")
        sys.exit(2)
    if world > 1 and dist.get_world_size() != world:
        log(f"error: process group size {dist.get_world_size()} != WORLD_SIZE {world}")
        sys.exit(2)
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    seed_host(1234 + rank)

    model = build_model(args, device)
    broadcast_parameters(model)
    # the DDIM / config-4 legs time the benchmark init (reinit_nonzero), not the weights the
    # train leg's Adam steps leave behind
    if args.init == "nonzero":
        init_state = {k: v.detach().clone() for k, v in model.state_dict().items()}
    else:
        init_state = build_model(args, device, init="nonzero").state_dict()
    nparams = sum(p.numel() for p in model.parameters())
    in_shape = (args.clips_per_gpu, 195, args.frames, args.size, args.size)
    work = unet_forward_work(model, in_shape)
    frames_per_gpu = args.clips_per_gpu * args.frames
    log(f"world {world}; params {nparams / 1e6:.1f} M; fwd {work.total / 1e12:.2f} TFLOP/clip "
        f"(conv {work.conv / 1e12:.2f}, attn {work.attn / 1e12:.2f})")

    result = {"metric": METRIC, "unit": "frames/s", "n_gpus": world, "steps": args.steps,
              "warmup": args.warmup, "higher_is_better": True, "scaling": "weak",
              "vs_baseline": None, "dtype": args.dtype,
              "data": "synthetic (seeded U[-1,1] frames / N(0,1) noise and audio), random-init "
                      "weights incl. wav2vec2-base"}

    sched = LinearNoiseScheduler(100, 0.00085, 0.012)  # train.py:48-52
    rows = []
    train_losses = []
    if args.only in ("train", "all"):
        trainer = Trainer(model, sched, lr=args.lr)
        bank = clip_bank(args, args.warmup + args.steps, device, rank)
        for i in range(args.warmup):
            loss = trainer.step(bank[i])
            train_losses.append(loss)
            log(f"warmup {i}: loss {float(loss):.4f}")
        barrier_sync(world)
        # attention launches only: the roofline's per-launch times (the conv breakdown comes
        # from one extra untimed step below, so its ~500 event pairs stay out of the timing)
        timer = ops.KernelTimer(attention=True, convs=args.timer_convs)
        ops.set_timer(timer)
        if trainer.bucketer is not None:
            trainer.bucketer.timing = True
        t0 = time.perf_counter()
        for i in range(args.steps):
            loss = trainer.step(bank[args.warmup + i])
            train_losses.append(loss)  # device scalars: read after the timed region
        barrier_sync(world)
        el = time.perf_counter() - t0
        ops.set_timer(None)
        if trainer.bucketer is not None:
            trainer.bucketer.timing = False
            result["allreduce"] = comm_report(trainer, world, device, args.steps)
            log("allreduce", result["allreduce"])
        el = max_over_ranks(el, world, device)
        ms = el / args.steps * 1e3
        result["value"] = round(world * frames_per_gpu * args.steps / el, 4)
        result["ms_per_step"] = round(ms, 2)
        summary = timer.summary()
        roof, rows, units = pick_roofline(summary, args.dtype)
        result["roofline"] = roof
        result["attention_units"] = units
        step_flops = 3 * work.total * args.clips_per_gpu
        result["model_tflops_per_gpu"] = round(step_flops / (el / args.steps) / 1e12, 1)
        # rank 0's MSE losses, warm-up then timed steps (train.py:131-132 prints them)
        result["train_losses"] = [_num(x, 5) for x in train_losses]
        result["train_init"] = {"init": args.init, "lr": args.lr, "reference_lr": 1e-2,
                                "warmup_steps": args.warmup, "timed_steps": args.steps,
                                "note": "not the reference's hyperparameter when lr != 1e-2: "
                                        "train.py:102 trains at 1e-2, where this model's loss "
                                        "spikes and it collapses to outputting 0 (as at 1e-3) "
                                        "-- product-only evidence: the oracle cannot run the "
                                        "config-2 model for hundreds of steps on the host; at "
                                        "1e-4 it learns over ~300 steps (profiles/"
                                        "r05_train_curve.txt), but this short timed window "
                                        "stays on the ~1.0 loss plateau; the kernels run ~4 % "
                                        "slower on its operands than at 1e-3 (DESIGN section 5); "
                                        "five bf16 steps at 1e-4 are pinned to the reference "
                                        "(tests/test_gpu_modules.py)"}
        log(f"train: {ms:.1f} ms/step, {result['value']:.3f} frames/s, loss {float(loss):.4f}, "
            f"model {result['model_tflops_per_gpu']} TFLOP/s/GPU (3x fwd)")
        for r in rows:
            log("  kernel", r)
        ctimer = ops.KernelTimer(attention=False, convs=True)
        ops.set_timer(ctimer)
        trainer.step(bank[-1])  # untimed: per-launch conv times
        ops.set_timer(None)
        conv = ctimer.conv_summary()
        by_kind = {}
        for (kind, key), (cnt, tot, flop) in conv.items():
            a = by_kind.setdefault(kind, [0, 0.0, 0.0])
            a[0] += cnt
            a[1] += tot
            a[2] += flop * cnt
        result["conv_kernels"] = {
            k: {"launches": c, "ms_per_step": round(t, 2),
                "tflops": round(f / (t / 1e3) / 1e12, 1) if t > 0 else None}
            for k, (c, t, f) in sorted(by_kind.items())}
        result["conv_kernels"]["note"] = "one extra untimed train step after the timed ones"
        for (kind, key), (cnt, tot, flop) in sorted(conv.items(), key=lambda kv: -kv[1][1])[:60]:
            log(f"  conv {kind:16s} {key:40s} x{cnt:<3d} {tot:7.2f} ms/step "
                f"{flop * cnt / (tot / 1e3) / 1e12:7.1f} TF/s")
        del trainer, bank
        torch.cuda.empty_cache()

    if args.only == "ddim_st":
        kd = args.ddim_steps or args.steps
        sampler = DDIMSampler(LinearNoiseSchedulerV2(500, 0.00005, 0.015), steps=50)
        clip = synthetic_clip(1, args.frames, args.size, 500, device, seed=100 + rank)
        result["ddim_st"] = ddim_st_leg(args, world, device, init_state, sampler, clip, kd)
        result.update(value=result["ddim_st"]["value"], unit="steps/s",
                      ms_per_step=result["ddim_st"]["ms_per_step"])

    if args.only in ("ddim", "all"):
        with torch.no_grad():
            model.load_state_dict(init_state)
        kd = args.ddim_steps or args.steps
        sampler = DDIMSampler(LinearNoiseSchedulerV2(500, 0.00005, 0.015), steps=50)
        clip = synthetic_clip(1, args.frames, args.size, 500, device, seed=100 + rank)
        model.eval()
        with torch.no_grad(), ops.frozen_weights():
            feats = model.encode_audio(clip.audio)
            xt = torch.randn_like(clip.x0)
            step = ddim_stepper(args, model, sampler, clip.cond, feats, xt)
            step(0)  # warm-up (and, graphed, the capture)
            barrier_sync(world)
            t0 = time.perf_counter()
            for i in range(1, 1 + kd):
                step(i)
            barrier_sync(world)
            el = max_over_ranks(time.perf_counter() - t0, world, device)
            del step
        ddim = {"metric": "DDIM steps/sec (50-step DDIM, B=1 clip, replicas)",
                "value": round(world * kd / el, 4), "unit": "steps/s",
                "ms_per_step": round(el / kd * 1e3, 2),
                "model_tflops_per_gpu": round(work.total / (el / kd) / 1e12, 1)}
        result["ddim"] = ddim
        log(f"ddim: {ddim['ms_per_step']} ms/step, {ddim['value']} steps/s")
        if args.st_steps != 0 and args.mode == "joint":
            try:  # an auxiliary leg: never let it take the headline numbers down
                result["ddim_st"] = ddim_st_leg(args, world, device, init_state, sampler, clip,
                                                kd)
            except Exception as e:
                log(f"ddim_st leg failed: {type(e).__name__}: {e}")
                result["ddim_st"] = {"value": None, "error": f"{type(e).__name__}: {e}"}
        if args.c4_steps > 0:
            # BASELINE config 4: 256x256x25-frame UNet3D, 50-step DDIM (test.py path), one clip
            # per GPU; the same weights (the UNet is size-agnostic), audio encoded once
            T4, S4, k4 = 25, 256, args.c4_steps
            work4 = unet_forward_work(model, (1, 195, T4, S4, S4))
            clip4 = synthetic_clip(1, T4, S4, 500, device, seed=200 + rank)
            with torch.no_grad(), ops.frozen_weights():
                feats4 = model.encode_audio(clip4.audio)
                x4 = torch.randn_like(clip4.x0)
                step4 = ddim_stepper(args, model, sampler, clip4.cond, feats4, x4)
                step4(0)  # warm-up step
                barrier_sync(world)
                t0 = time.perf_counter()
                for i in range(1, 1 + k4):
                    step4(i)
                barrier_sync(world)
                el4 = max_over_ranks(time.perf_counter() - t0, world, device)
                del step4
            result["ddim_config4"] = {
                "metric": "DDIM steps/sec, 256x256x25 UNet3D (BASELINE config 4, test.py path)",
                "value": round(world * k4 / el4, 4), "unit": "steps/s",
                "ms_per_step": round(el4 / k4 * 1e3, 1), "steps_timed": k4,
                "attention_mode": args.mode, "fwd_tflop": round(work4.total / 1e12, 1),
                "model_tflops_per_gpu": round(work4.total / (el4 / k4) / 1e12, 1),
                "sampling_50_steps_s": round(50 * el4 / k4, 1)}
            log(f"ddim config 4 (256x256x25): {result['ddim_config4']['ms_per_step']} ms/step, "
                f"{result['ddim_config4']['model_tflops_per_gpu']} TFLOP/s")
            del clip4, feats4, x4
            torch.cuda.empty_cache()
        if "value" not in result:
            result.update(value=ddim["value"], unit="steps/s", ms_per_step=ddim["ms_per_step"])

    if args.only in ("train", "all") and args.xattn_steps != 0:
        try:  # an auxiliary leg: never let it take the headline numbers down
            result["audio_xattn"] = xattn_leg(args, rank, world, device,
                                              result.get("ms_per_step"))
        except Exception as e:
            log(f"xattn leg failed: {type(e).__name__}: {e}")
            result["audio_xattn"] = {"value": None, "error": f"{type(e).__name__}: {e}"}

    if args.only in ("train", "all") and args.st_steps != 0 and args.mode == "joint":
        try:  # an auxiliary leg: never let it take the headline numbers down
            result["spatial_temporal"] = st_leg(args, rank, world, device)
        except Exception as e:
            log(f"spatial_temporal leg failed: {type(e).__name__}: {e}")
            result["spatial_temporal"] = {"value": None, "error": f"{type(e).__name__}: {e}"}

    if args.only in ("train", "all") and args.train_graph and world == 1:
        try:  # an auxiliary leg: never let it take the headline numbers down
            result["train_graph"] = graph_leg(args, device)
        except Exception as e:
            log(f"train graph leg failed: {type(e).__name__}: {e}")
            result["train_graph"] = {"value": None, "error": f"{type(e).__name__}: {e}"}

    if args.only in ("vivit", "all") and args.vivit_steps > 0:
        try:  # an auxiliary leg: never let it take the headline numbers down
            result["vivit"] = vivit_leg(args, rank, world, device)
        except Exception as e:
            log(f"vivit leg failed: {type(e).__name__}: {e}")
            result["vivit"] = {"value": None, "error": f"{type(e).__name__}: {e}"}

    result["config"] = {
        "workload": f"train step, audio-conditioned UNet3D {args.size}x{args.size}x{args.frames} "
                    f"({args.mode} attention), {args.clips_per_gpu} clip/GPU",
        "clip": [args.clips_per_gpu, 3, args.frames, args.size, args.size],
        "global_batch_clips": world * args.clips_per_gpu,
        "attention_mode": args.mode, "parallelism": f"dp{world}",
        "fwd_tflop_per_clip": round(work.total / 1e12, 3)}
    if rows:
        result["kernels"] = rows
    if rank == 0 and world == 1 and not args.no_cpu:
        try:
            result["cpu_baseline"] = cpu_baseline(args)
        except Exception as e:  # never let the baseline leg kill the GPU numbers
            result["cpu_baseline"] = {"value": None, "error": f"{type(e).__name__}: {e}"}
    else:
        result["cpu_baseline"] = None
    bad = [i for i, x in enumerate(result.get("train_losses", [])) if x is None]
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if bad:  # a diverged step: the line is printed (with the losses) but the run fails
        log(f"error: non-finite training loss at steps {bad}")
        sys.exit(3)


if __name__ == "__main__":
    main()
