"""Does the denoiser learn on the synthetic clips?  (A sanity check of the training path, not
a benchmark.)  x0 ~ U[-1, 1] i.i.d. per pixel, eps ~ N(0, 1), t ~ U{0..99} (a new clip every
step): the best per-pixel linear estimator eps_hat = c(t) x_t already reaches an MSE of about
0.6 averaged over t (1 at t = 0, 0.27 at t = 99 for the linear schedule of train.py:47), so a
trainer that works drives the loss below 1 -- a loss that stays at 1.0 means the network
only learned to output 0.

    python tools/learn_check.py oracle [steps] [lr]        # CPU: oracle/ (fp32 torch)
    python tools/learn_check.py gpu [steps] [lr] [fp32]    # the product Trainer (bf16)

Tiny UNet3D of oracle.fixtures.TINY3D at 32x32x4, random non-zero init, Adam; prints the
mean loss per 25 steps."""
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd"))

import torch  # noqa: E402

T, S, AUD = 4, 32, 16


def floor_mse():
    """The per-pixel linear estimator's MSE averaged over t (x0 variance 1/3)."""
    betas = torch.linspace(0.00085, 0.012, 100, dtype=torch.float64)
    ab = torch.cumprod(1 - betas, 0)
    return float((1 - (1 - ab) / (ab / 3 + 1 - ab)).mean())


def clip(i, device):
    g = torch.Generator(device=device).manual_seed(1000 + i)
    x0 = torch.rand((1, 3, T, S, S), generator=g, device=device) * 2 - 1
    cond = torch.rand((1, 3, S, S), generator=g, device=device) * 2 - 1
    eps = torch.randn((1, 3, T, S, S), generator=g, device=device)
    feat = torch.randn((T, 768), generator=g, device=device)
    t = torch.randint(0, 100, (1,), generator=g, device=device)
    return x0, cond, eps, feat, t


def run_oracle(steps, lr):
    import torch.nn.functional as F
    from oracle import schedulers as osch
    from oracle.fixtures import TINY3D
    from oracle.unet import (audio_conditioned_input, audio_param_shapes, build_plan,
                             init_params, param_shapes, unet_forward)
    plan = build_plan(**TINY3D, attention_mode="joint")
    P = init_params(param_shapes(plan), 1234)
    P.update(init_params(audio_param_shapes(768, AUD, im_cond_output_ch=16), 77))
    for v in P.values():
        v.requires_grad_(True)
    tab = osch.linear_tables(100, 0.00085, 0.012)
    opt = torch.optim.Adam(list(P.values()), lr=lr)
    losses = []
    for i in range(steps):
        x0, cond, eps, feat, t = clip(i, "cpu")
        xt = osch.q_sample(tab, x0, eps, t)
        x = audio_conditioned_input(P, xt, cond, feat, AUD)
        loss = F.mse_loss(unet_forward(P, plan, x, t), eps)
        loss.backward()
        opt.step()
        opt.zero_grad()
        losses.append(float(loss))
    return losses


def run_gpu(steps, lr, fp32):
    from vdiff.engine import Clip, Trainer, reinit_nonzero
    from vdiff.schedulers import LinearNoiseScheduler
    from vdiff.unet_audio import UNetAudio
    from oracle.fixtures import TINY3D
    dev = torch.device("cuda", 0)
    m = UNetAudio(image_size=S, in_channels=3, model_channels=TINY3D["model_channels"],
                  out_channels=3, num_res_blocks=TINY3D["num_res_blocks"],
                  attention_resolutions=TINY3D["attention_resolutions"],
                  channel_mult=TINY3D["channel_mult"], dropout=0.0, dims=3,
                  audio_feature_dim=768, projected_audio_dim=AUD, use_bf16=not fp32,
                  attention_mode="joint", audio_encoder_pretrained=False)
    reinit_nonzero(m, seed=1234)
    m = m.to(dev)
    tr = Trainer(m, LinearNoiseScheduler(100, 0.00085, 0.012), lr=lr)
    losses = []
    for i in range(steps):
        x0, cond, eps, _, t = clip(i, dev)
        audio = {"input_values": torch.randn((T, 4000), device=dev,
                                             generator=torch.Generator(device=dev).manual_seed(i))}
        losses.append(tr.step(Clip(x0, cond, audio, eps, t)))
    return [float(x) for x in losses]


def main():
    which = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    lr = float(sys.argv[3]) if len(sys.argv) > 3 else 1e-3
    fp32 = len(sys.argv) > 4 and sys.argv[4] == "fp32"
    t0 = time.time()
    losses = run_oracle(steps, lr) if which == "oracle" else run_gpu(steps, lr, fp32)
    print(f"{which}{' fp32' if fp32 else ''} lr {lr}: {steps} steps in {time.time() - t0:.0f} s; "
          f"linear-estimator floor {floor_mse():.3f}")
    for k in range(0, steps, 25):
        w = losses[k:k + 25]
        print(f"  steps {k:4d}-{k + len(w) - 1:4d}: mean loss {sum(w) / len(w):.4f}")
    assert all(math.isfinite(x) for x in losses)


if __name__ == "__main__":
    main()
