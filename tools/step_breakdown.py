"""Where the config-2 train step's time goes, by component (HIP events on the current
stream, bf16, 128x128x16 joint):
  * the whole Trainer.step (q_sample + UNetAudio fwd + MSE + bwd + Adam);
  * wav2vec2 alone (the audio encoder's forward on the clip's 16 windows + its backward);
  * the UNet alone (pooled audio features given, encoder skipped) fwd + bwd;
  * Adam alone.
    python tools/step_breakdown.py [--steps 5]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def timed(fn, steps):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(steps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--bf16-w2v", action="store_true")
    a = ap.parse_args()
    if a.bf16_w2v:
        os.environ["VDIFF_W2V_BF16"] = "1"
    import bench
    from vdiff.engine import Trainer, synthetic_clip
    from vdiff.schedulers import LinearNoiseScheduler
    dev = torch.device("cuda", 0)
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    torch.manual_seed(0)
    model = bench.build_model(args, dev)
    tr = Trainer(model, LinearNoiseScheduler(100, 0.00085, 0.012), lr=1e-2)
    clip = synthetic_clip(1, 16, 128, 100, dev, seed=0)
    res = {"train_step_ms": timed(lambda: tr.step(clip), a.steps)}

    def w2v():
        model.train()
        f = model.encode_audio(clip.audio)
        f.backward(torch.ones_like(f))
    res["wav2vec2_fwd_bwd_ms"] = timed(w2v, a.steps)
    with torch.no_grad():
        feats = model.encode_audio(clip.audio).detach()

    def unet():
        model.train()
        xt = tr.scheduler.add_noise(clip.x0, clip.eps, clip.t)
        F.mse_loss(model(xt, clip.cond, feats, clip.t), clip.eps).backward()
    res["unet_fwd_bwd_ms"] = timed(unet, a.steps)
    res["adam_ms"] = timed(lambda: tr.opt.step(), a.steps)
    tr.opt.zero_grad(set_to_none=True)
    n_w2v = sum(p.numel() for p in model.audio_encoder.parameters())
    res["wav2vec2_params_M"] = round(n_w2v / 1e6, 2)
    print({k: round(v, 2) if isinstance(v, float) else v for k, v in res.items()}, flush=True)


if __name__ == "__main__":
    main()
