"""Drop-in modules (vdiff.nn / vdiff.unet_audio) vs the reference golden vectors and the
oracle: fp32 parity mode (north-star bar: rel-L2 <= 1e-3; observed ~1e-6) and bf16
throughput mode (rel-L2 <= 3e-2 vs fp32 reference)."""
import pytest
import torch
import torch.nn.functional as F

from oracle import nn as onn
from oracle.fixtures import FULL2D, FULL2D_SHAPE, TINY3D, TINY3D_SHAPE, rel_l2, seeded
from oracle.unet import audio_param_shapes, build_plan, init_params, param_shapes, unet_forward

from conftest import golden, record_metric

pytestmark = pytest.mark.gpu
dev = "cuda"


def _load(module, seed):
    shapes = {k: tuple(v.shape) for k, v in module.state_dict().items()}
    P = init_params(shapes, seed)
    module.load_state_dict(P)
    return P


def test_state_dict_keys_match_reference_plan():
    from vdiff.nn import UNetModel
    m = UNetModel(image_size=32, **FULL2D)
    ref = param_shapes(build_plan(**FULL2D))
    sd = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    assert list(sd) == list(ref)
    assert sd == dict(ref)


def test_resblock3d_golden():
    from vdiff.nn import ResBlock
    g = golden("blocks.npz")
    rb = ResBlock(64, 256, 0.0, out_channels=128, dims=3)
    _load(rb, 30)
    rb = rb.to(dev)
    x = seeded((2, 64, 2, 6, 6), 31).to(dev).requires_grad_(True)
    emb = seeded((2, 256), 32).to(dev).requires_grad_(True)
    y = rb(x, emb)
    assert rel_l2(y, g["rb_y"]) < 1e-5
    y.backward(seeded(y.shape, 33).to(dev))
    assert rel_l2(x.grad, g["rb_dx"]) < 1e-5
    assert rel_l2(emb.grad, g["rb_demb"]) < 1e-5
    named = dict(rb.named_parameters())
    for k in ("in_layers.2.weight", "skip_connection.weight", "out_layers.0.weight",
              "emb_layers.1.weight", "out_layers.3.bias"):
        assert rel_l2(named[k].grad, g["rb_d_" + k]) < 1e-5, k


def test_resblock2d_identity_skip_golden():
    from vdiff.nn import ResBlock
    g = golden("blocks.npz")
    rb = ResBlock(64, 256, 0.0, dims=2)
    _load(rb, 34)
    rb = rb.to(dev)
    x = seeded((2, 64, 10, 10), 35).to(dev).requires_grad_(True)
    y = rb(x, seeded((2, 256), 36).to(dev))
    assert rel_l2(y, g["rb2_y"]) < 1e-5
    y.backward(seeded(y.shape, 37).to(dev))
    assert rel_l2(x.grad, g["rb2_dx"]) < 1e-5
    assert rel_l2(rb.in_layers[2].weight.grad, g["rb2_d_in_w"]) < 1e-5


def test_attention_block_golden():
    from vdiff.nn import AttentionBlock
    g = golden("blocks.npz")
    ab = AttentionBlock(64, num_heads=1)
    _load(ab, 40)
    ab = ab.to(dev)
    x = seeded((2, 64, 2, 6, 6), 41).to(dev).requires_grad_(True)
    y = ab(x)
    assert rel_l2(y, g["ab_y"]) < 1e-5
    y.backward(seeded(y.shape, 42).to(dev))
    assert rel_l2(x.grad, g["ab_dx"]) < 1e-5
    assert rel_l2(ab.qkv.weight.grad, g["ab_d_qkv_w"]) < 1e-5
    assert rel_l2(ab.proj_out.weight.grad, g["ab_d_proj_w"]) < 1e-5
    assert rel_l2(ab.norm.weight.grad, g["ab_d_norm_w"]) < 1e-5
    for tag, new_order in (("abh", False), ("abn", True)):
        m = AttentionBlock(64, num_heads=2, use_new_attention_order=new_order)
        _load(m, 43)
        m = m.to(dev)
        x = seeded((1, 64, 10, 10), 44).to(dev).requires_grad_(True)
        y = m(x)
        assert rel_l2(y, g[f"{tag}_y"]) < 1e-5, tag
        y.backward(seeded(y.shape, 45).to(dev))
        assert rel_l2(x.grad, g[f"{tag}_dx"]) < 1e-5, tag
        assert rel_l2(m.qkv.weight.grad, g[f"{tag}_d_qkv_w"]) < 1e-5, tag


def test_up_down_golden():
    from vdiff.nn import Downsample, Upsample
    g = golden("blocks.npz")
    up = Upsample(64, True, dims=3)
    _load(up, 50)
    up = up.to(dev)
    x = seeded((1, 64, 2, 5, 5), 51).to(dev).requires_grad_(True)
    y = up(x)
    assert rel_l2(y, g["up_y"]) < 1e-5
    y.backward(seeded(y.shape, 52).to(dev))
    assert rel_l2(x.grad, g["up_dx"]) < 1e-5
    assert rel_l2(up.conv.weight.grad, g["up_dw"]) < 1e-5
    dn = Downsample(64, True, dims=3)
    _load(dn, 53)
    dn = dn.to(dev)
    x = seeded((1, 64, 2, 9, 9), 54).to(dev).requires_grad_(True)
    y = dn(x)
    assert rel_l2(y, g["dn_y"]) < 1e-5
    y.backward(seeded(y.shape, 55).to(dev))
    assert rel_l2(x.grad, g["dn_dx"]) < 1e-5
    assert rel_l2(dn.op.weight.grad, g["dn_dw"]) < 1e-5


def _tiny3d(dtype_bf16=False, mode="joint"):
    from vdiff.nn import UNetModel
    m = UNetModel(image_size=64, **TINY3D, attention_mode=mode, use_bf16=dtype_bf16)
    _load(m, 1234)
    return m.to(dev).eval()


def test_tiny3d_unet_golden_fp32():
    g = golden("unet_tiny3d.npz")
    m = _tiny3d()
    x = seeded(TINY3D_SHAPE, 60, "uniform").to(dev)
    y = m(x, g["t"].to(dev))
    e = rel_l2(y, g["y"])
    assert e < 1e-4, e  # north-star bar is 1e-3
    loss = F.mse_loss(y, seeded((1, 3) + TINY3D_SHAPE[2:], 61).to(dev))
    assert abs(loss.item() - g["loss"].item()) / g["loss"].item() < 1e-5
    loss.backward()
    named = dict(m.named_parameters())
    for k in ("input_blocks.0.0.weight", "out.2.weight", "input_blocks.3.1.qkv.weight",
              "middle_block.0.in_layers.0.weight", "output_blocks.0.0.skip_connection.weight",
              "time_embed.0.weight"):
        assert rel_l2(named[k].grad, g["grad_" + k]) < 1e-4, k


def test_tiny3d_unet_bf16_tolerance():
    g = golden("unet_tiny3d.npz")
    m = _tiny3d(dtype_bf16=True)
    y = m(seeded(TINY3D_SHAPE, 60, "uniform").to(dev), g["t"].to(dev))
    assert y.dtype == torch.float32
    e = rel_l2(y, g["y"])
    assert e < 3e-2, e


def test_full2d_unet_golden_fp32():
    from vdiff.nn import UNetModel
    g = golden("unet_full2d.npz")
    m = UNetModel(image_size=32, **FULL2D)
    _load(m, 1234)
    m = m.to(dev).eval()
    y = m(seeded(FULL2D_SHAPE, 62, "uniform").to(dev), g["t"].to(dev))
    assert rel_l2(y, g["y"]) < 1e-4
    y.backward(seeded(y.shape, 63).to(dev))
    assert rel_l2(m.input_blocks[0][0].weight.grad, g["grad_in"]) < 1e-4
    assert rel_l2(m.input_blocks[1][1].qkv.weight.grad, g["grad_attn"]) < 1e-4
    assert rel_l2(m.out[2].weight.grad, g["grad_out"]) < 1e-4


def test_unet_audio_conditioning_golden():
    from vdiff.unet_audio import UNetAudio
    ga = golden("unet_audio2d.npz")
    m = UNetAudio(image_size=32, in_channels=3, model_channels=64, out_channels=3,
                  num_res_blocks=2, attention_resolutions=(1, 2, 4), audio_feature_dim=768,
                  projected_audio_dim=128, audio_encoder=False)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    P = init_params({k: v for k, v in shapes.items() if not k.startswith(("audio_", "cond_"))},
                    1234)
    P.update(init_params(audio_param_shapes(768, 128), 77))
    m.load_state_dict(P)
    m = m.to(dev).eval()
    y = m(seeded((2, 3, 32, 32), 64, "uniform").to(dev),
          seeded((2, 3, 16, 16), 65, "uniform").to(dev), seeded((2, 768), 66).to(dev),
          ga["t"].to(dev))
    assert rel_l2(y, ga["y"]) < 1e-4


def test_unet_audio_5d_matches_oracle_and_trains():
    """Frame-stack conditioning (build extension D2) vs the oracle restatement, incl. grads
    through the concat kernel into cond_conv_in / audio_transformer."""
    from vdiff.unet_audio import UNetAudio
    cfg = dict(image_size=16, in_channels=3, model_channels=32, out_channels=3,
               num_res_blocks=1, attention_resolutions=(2,), channel_mult=(1, 2), dims=3,
               audio_feature_dim=64, projected_audio_dim=16, im_cond_output_ch=16, dropout=0.0)
    m = UNetAudio(**cfg, audio_encoder=False)
    P = _load(m, 5)
    m = m.to(dev)
    image = seeded((2, 3, 4, 16, 16), 1, "uniform")
    cond = seeded((2, 3, 8, 8), 2, "uniform")
    feat = seeded((8, 64), 3)
    t = torch.tensor([3, 70])
    y = m(image.to(dev), cond.to(dev), feat.to(dev), t.to(dev))
    plan = build_plan(in_channels=3 + 16 + 16, model_channels=32, out_channels=3,
                      num_res_blocks=1, attention_resolutions=(2,), channel_mult=(1, 2), dims=3)
    Pr = {k: v.clone().requires_grad_(True) for k, v in P.items()}
    from oracle.unet import audio_conditioned_input
    xin = audio_conditioned_input(Pr, image, cond, feat, 16)
    yr = unet_forward(Pr, plan, xin, t)
    assert rel_l2(y, yr) < 1e-4
    gy = seeded(yr.shape, 4)
    yr.backward(gy)
    y.backward(gy.to(dev))
    named = dict(m.named_parameters())
    for k in ("cond_conv_in.weight", "audio_transformer.transform.0.weight",
              "input_blocks.0.0.weight"):
        assert rel_l2(named[k].grad, Pr[k].grad) < 1e-4, k


@pytest.mark.parametrize("mode", ["spatial", "temporal"])
def test_factorised_attention_modes_vs_oracle(mode):
    from vdiff.nn import UNetModel
    cfg = dict(TINY3D)
    m = UNetModel(image_size=32, **cfg, attention_mode=mode)
    P = _load(m, 9)
    m = m.to(dev).eval()
    x = seeded((1, 35, 4, 32, 32), 10, "uniform")
    t = torch.tensor([11])
    y = m(x.to(dev), t.to(dev))
    yr = unet_forward(P, build_plan(**cfg), x, t, attn_mode=mode)
    assert rel_l2(y, yr) < 1e-4


def test_spatial_temporal_block_composes_modes():
    from vdiff.nn import AttentionBlock
    ab = AttentionBlock(64, attention_mode="spatial_temporal")
    P = _load(ab, 12)
    ab = ab.to(dev)
    x = seeded((1, 64, 3, 6, 6), 13)
    y = ab(x.to(dev))
    h = onn.attention_block(P, "", x, mode="spatial")
    Pt = {"norm.weight": P["temporal_norm.weight"], "norm.bias": P["temporal_norm.bias"],
          "qkv.weight": P["temporal_qkv.weight"], "qkv.bias": P["temporal_qkv.bias"],
          "proj_out.weight": P["temporal_proj_out.weight"],
          "proj_out.bias": P["temporal_proj_out.bias"]}
    yr = onn.attention_block(Pt, "", h, mode="temporal")
    assert rel_l2(y, yr) < 1e-5


def test_fused_dropout_mask_consistency():
    """Train-mode dropout fused into GN+SiLU: keep rate ~ 1-p and the backward uses the
    same mask as the forward."""
    from vdiff import ops
    p = 0.25
    x = seeded((2, 64, 4, 16, 16), 14)
    w, b = 1 + 0.1 * seeded((64,), 15), 0.1 * seeded((64,), 16)
    xd = ops.to_cl(x.to(dev)).requires_grad_(True)
    y = ops.group_norm_silu(xd, w.to(dev), b.to(dev), dropout=p, seed=1234)
    base = onn.group_norm(x, w, b, silu=True)
    mask = (y.detach().cpu() != 0).float()
    keep = mask.mean().item()
    assert abs(keep - (1 - p)) < 0.01
    assert rel_l2(y, base * mask / (1 - p)) < 1e-5
    g = seeded(x.shape, 17)
    y.backward(ops.to_cl(g.to(dev)))
    xr = x.clone().requires_grad_(True)
    (onn.group_norm(xr, w, b, silu=True) * mask / (1 - p)).backward(g)
    assert rel_l2(xd.grad, xr.grad) < 1e-5
    y2 = ops.group_norm_silu(xd.detach(), w.to(dev), b.to(dev), dropout=p, seed=1234)
    assert torch.equal(y.detach(), y2)


def test_schedulers_module_api():
    from vdiff.schedulers import (CosineNoiseScheduler, DDIMSampler, LinearNoiseScheduler,
                                  LinearNoiseSchedulerV2)
    from oracle import schedulers as osch
    s = LinearNoiseScheduler(100, 0.00085, 0.012)
    ref = osch.linear_tables(100, 0.00085, 0.012)
    assert torch.equal(s.alpha_cum_prod, ref["acp"])
    x0, eps = seeded((2, 3, 4, 8, 8), 1), seeded((2, 3, 4, 8, 8), 2)
    t = torch.tensor([5, 90])
    out = s.add_noise(x0.to(dev), eps.to(dev), t.to(dev))
    assert rel_l2(out, osch.q_sample(ref, x0, eps, t)) < 1e-6
    v2 = LinearNoiseSchedulerV2(500, 0.00005, 0.015)
    z = seeded(x0.shape, 3)
    prev, x0p = v2.sample_prev_timestep(x0.to(dev), eps.to(dev), t.to(dev), z=z.to(dev))
    rp, rx = osch.p_sample_v2(osch.linear_tables(500, 0.00005, 0.015), x0, eps, t, z)
    assert rel_l2(prev, rp) < 1e-6 and rel_l2(x0p, rx) < 1e-6
    c = CosineNoiseScheduler(2000)
    assert torch.equal(c.alphas_cumprod, osch.cosine_tables(2000)["acp"])
    ddim = DDIMSampler(v2, steps=50)
    assert ddim.timesteps[0] == 499 and ddim.timesteps[-1] == 0
    xp, _ = ddim.step(x0.to(dev), eps.to(dev), 0)
    rxp, _ = osch.ddim_step(v2.alpha_cum_prod, x0, eps, torch.tensor([499, 499]),
                            torch.tensor([int(ddim.prev_timesteps[0])] * 2))
    assert rel_l2(xp, rxp) < 1e-5


def test_trainer_step_matches_reference_adam_step():
    """one fp32 Trainer.step (q_sample -> UNetAudio -> MSE -> backward -> fused
    Adam lr 1e-2) with injected eps / t against the reference train step's loss, gradients
    and one-step parameter deltas (tests/golden/train_step_tiny3d.npz, config 1's shape)."""
    from oracle.fixtures import adam_delta_close, train_step_inputs
    from vdiff.engine import Clip, Trainer
    from vdiff.schedulers import LinearNoiseScheduler
    from vdiff.unet_audio import UNetAudio
    g = golden("train_step_tiny3d.npz")
    m = UNetAudio(image_size=64, in_channels=3, model_channels=32, out_channels=3,
                  num_res_blocks=1, attention_resolutions=(2,), channel_mult=(1, 2), dims=3,
                  audio_feature_dim=64, projected_audio_dim=16, im_cond_output_ch=16,
                  dropout=0.0, audio_encoder=False)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    P = init_params({k: v for k, v in shapes.items() if not k.startswith(("audio_", "cond_"))},
                    1234)
    P.update(init_params(audio_param_shapes(64, 16, im_cond_output_ch=16), 77))
    m.load_state_dict(P)
    m = m.to(dev)
    before = {k: v.detach().clone() for k, v in m.named_parameters()}
    x0, cond, feat, eps = (u.to(dev) for u in train_step_inputs())
    tr = Trainer(m, LinearNoiseScheduler(100, 0.00085, 0.012), lr=1e-2)
    grads = {}
    hooks = [p.register_post_accumulate_grad_hook(
        lambda p, n=n: grads.__setitem__(n, p.grad.detach().clone()))
        for n, p in m.named_parameters()]
    loss = tr.step(Clip(x0, cond, feat, eps, g["t"].to(dev)))
    for h in hooks:
        h.remove()
    assert abs(float(loss) - float(g["loss"])) < 1e-5 * float(g["loss"])
    named = dict(m.named_parameters())
    keys = [k[len("delta_"):] for k in g if k.startswith("delta_")]
    assert len(keys) == 9
    for k in keys:
        assert rel_l2(grads[k], g["grad_" + k]) < 1e-4, k
        d = named[k].detach() - before[k]
        assert adam_delta_close(d, g["delta_" + k], g["grad_" + k]) < 1e-6, k


def _five_steps(bf16, lr=1e-2, fixture="train_steps5_tiny3d.npz"):
    """Five steps of the DEFAULT Trainer (conv operands packed per call in step 1, by the
    batched launch from step 2 on; fused Adam lr 1e-2 whose moments carry over) on the
    inputs of the five-step reference fixture (train.py:107-134,
    tests/golden/train_steps5_tiny3d.npz).  Returns {"loss": max rel error of the five
    losses, name: (step-1 grad, step-5 grad, five-step delta) rel-L2} for nine parameters."""
    from oracle.fixtures import TRAIN5_T, train5_inputs
    from vdiff.engine import Clip, Trainer
    from vdiff.schedulers import LinearNoiseScheduler
    from vdiff.unet_audio import UNetAudio
    g = golden(fixture)
    if "lr" in g:
        assert abs(float(g["lr"]) - lr) <= 1e-6 * lr, (float(g["lr"]), lr)  # stored fp32
    m = UNetAudio(image_size=64, in_channels=3, model_channels=32, out_channels=3,
                  num_res_blocks=1, attention_resolutions=(2,), channel_mult=(1, 2), dims=3,
                  audio_feature_dim=64, projected_audio_dim=16, im_cond_output_ch=16,
                  dropout=0.0, audio_encoder=False)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    P = init_params({k: v for k, v in shapes.items() if not k.startswith(("audio_", "cond_"))},
                    1234)
    P.update(init_params(audio_param_shapes(64, 16, im_cond_output_ch=16), 77))
    m.load_state_dict(P)
    if bf16:
        m.convert_to_fp16()   # the bench's mode: bf16 activations, fp32 master weights
    m = m.to(dev)
    before = {k: v.detach().clone() for k, v in m.named_parameters()}
    tr = Trainer(m, LinearNoiseScheduler(100, 0.00085, 0.012), lr=lr)
    assert tr.packs.__class__.__name__ == "step_packed_weights"  # the default path
    grads = {}
    step = [0]
    hooks = [p.register_post_accumulate_grad_hook(
        lambda p, n=n: grads.__setitem__((step[0], n), p.grad.detach().float().clone()))
        for n, p in m.named_parameters()]
    losses = []
    for k, t in enumerate(TRAIN5_T):
        step[0] = k
        x0, cond, feat, eps = (u.to(dev) for u in train5_inputs(k))
        losses.append(tr.step(Clip(x0, cond, feat, eps, torch.tensor([t], device=dev))))
    for h in hooks:
        h.remove()
    assert tr.packs.plans  # steps 2-5 ran on the batched pack
    losses = torch.stack(losses).float().cpu()
    assert torch.isfinite(losses).all()
    err_l = float(((losses - g["losses"]).abs() / g["losses"]).max())
    named = dict(m.named_parameters())
    names = [k[len("delta5_"):] for k in g if k.startswith("delta5_")]
    assert len(names) == 9
    rep = {"loss": err_l}
    for k in names:
        e1 = rel_l2(grads[(0, k)], g["grad1_" + k])
        e5 = rel_l2(grads[(4, k)], g["grad5_" + k])
        ed = rel_l2(named[k].detach().float() - before[k].float(), g["delta5_" + k])
        rep[k] = (e1, e5, ed)
    worst = {"grad1": max(v[0] for k, v in rep.items() if k != "loss"),
             "grad5": max(v[1] for k, v in rep.items() if k != "loss"),
             "delta5": max(v[2] for k, v in rep.items() if k != "loss")}
    record_metric(test="trainer_five_steps_vs_reference", mode="bf16" if bf16 else "fp32",
                  lr=lr, loss_max_rel=err_l, worst=worst,
                  per_param={k: v for k, v in rep.items() if k != "loss"})
    print("five-step parity", "bf16" if bf16 else "fp32", worst, rep)
    return rep, worst


def test_trainer_five_steps_match_reference():
    """five fp32 (parity mode) steps against the five
    reference steps.  Bars: the GPU's fp32 reductions differ from the CPU's in order only,
    so losses and step-1 gradients agree to 1e-4 and step-5 gradients (after four Adam
    updates) to 1e-3 (measured round 5: 2.6e-5, 1.9e-6, 7.2e-4).  The five-step parameter
    change is held to 3x its measured value (1.6e-4 -> 5e-4): Adam's g / (sqrt(v) + eps) turns
    order-level gradient differences into steps of up to lr where a gradient component is ~0
    (oracle.fixtures.adam_delta_close), so it sits above the step-1 gradients'."""
    rep, worst = _five_steps(bf16=False)
    assert rep["loss"] < 1e-4, rep
    assert worst["grad1"] < 1e-4 and worst["grad5"] < 1e-3, rep
    assert worst["delta5"] < 5e-4, rep


def _autocast_five_steps():
    """The same five steps of the ORACLE (the reference's math restated in torch, pinned bit
    for bit to the fixture on the CPU) on the GPU under torch.autocast(bfloat16): what bf16
    operands alone cost against the fp32 reference -- the peer the bf16 Trainer is held to.
    Returns the same error summary as _five_steps."""
    from oracle.fixtures import TRAIN5_T, train5_inputs
    from oracle.train import train_steps
    g = golden("train_steps5_tiny3d.npz")
    plan = build_plan(**TINY3D)
    P = init_params(param_shapes(plan), 1234)
    P.update(init_params(audio_param_shapes(64, 16, im_cond_output_ch=16), 77))
    P = {k: v.to(dev) for k, v in P.items()}
    P0 = {k: v.clone() for k, v in P.items()}
    batches = [tuple(u.to(dev) for u in train5_inputs(k)) + (torch.tensor([t], device=dev),)
               for k, t in enumerate(TRAIN5_T)]
    prev = torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32
    torch.backends.cuda.matmul.allow_tf32 = torch.backends.cudnn.allow_tf32 = False
    try:
        with torch.autocast("cuda", dtype=torch.bfloat16):
            losses, kept = train_steps(P, plan, batches, 16, keep_grads=(0, 4))
    finally:
        torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32 = prev
    losses = losses.float().cpu()
    names = [k[len("delta5_"):] for k in g if k.startswith("delta5_")]
    rep = {k: (rel_l2(kept[0][k], g["grad1_" + k]), rel_l2(kept[4][k], g["grad5_" + k]),
               rel_l2(P[k] - P0[k], g["delta5_" + k])) for k in names}
    worst = {"loss": float(((losses - g["losses"]).abs() / g["losses"]).max()),
             "grad1": max(v[0] for v in rep.values()), "grad5": max(v[1] for v in rep.values()),
             "delta5": max(v[2] for v in rep.values())}
    record_metric(test="oracle_autocast_bf16_five_steps_vs_reference", worst=worst,
                  per_param=rep)
    return worst


def test_trainer_five_steps_bf16_match_reference():
    """VERDICT r04 missing #2: the bf16 Trainer -- the path bench.py times (bf16 activations
    and conv / attention operands, fp32 master weights, fp32 accumulation, fused Adam) --
    against the same five fp32 reference steps.  Stated bf16 bars: every one of the five
    losses within 3e-2 relative and the step-1 gradients within 5e-2 rel-L2 (measured
    round 5: 8.3e-3 and 1.3e-2).  After four Adam updates at the reference lr 1e-2 the
    trajectories separate: Adam's g / (sqrt(v) + eps) turns every bf16-level gradient
    difference on a near-zero component into a full +-lr step, and at this lr the loss
    itself jumps 1.27 -> 2.23 -> 1.54.  So the step-5 gradients and the five-step parameter
    change are held to fixed bars 1.5x above the measured values (1.07 and 0.24 -> 1.6 and
    0.36) AND to the reference's own math run in bf16 -- the oracle under torch.autocast
    (_autocast_five_steps), which measured loss 0.43, step-1 gradients 0.15, step-5
    gradients 3.76, five-step change 2.70: the bf16 Trainer must stay at or below that peer
    on every figure."""
    rep, worst = _five_steps(bf16=True)
    auto = _autocast_five_steps()
    print("autocast-bf16 oracle five-step parity", auto)
    assert rep["loss"] < 3e-2, rep
    assert worst["grad1"] < 5e-2, rep
    assert worst["grad5"] < 1.6 and worst["delta5"] < 0.36, (worst, auto)
    for k in ("grad1", "grad5", "delta5"):
        assert worst[k] <= auto[k], (k, worst, auto)
    assert rep["loss"] <= auto["loss"], (rep["loss"], auto)


def test_trainer_five_steps_bf16_at_bench_lr_match_reference():
    """the bf16 Trainer -- the path bench.py times -- at bench.py's Adam lr
    1e-4 against five fp32 steps of the imported reference at that lr
    (train_steps5_tiny3d_lr1e-4.npz).  At this lr the trajectories do not separate after step
    1 (every Adam step is 1e-4, not 1e-2), so every figure constrains the kernels.  Measured
    round 6 (profiles/r06_parity_metrics.jsonl): losses 2.3e-4, step-1 gradients 1.3e-2,
    step-5 gradients 1.5e-2, five-step change 5.9e-2.  Bars about 3x those, capped at the bars
    VERDICT r05 set (3e-2 / 1e-1 / 1e-1): 1e-3, 4e-2, 5e-2, 1e-1.  The five-step change sits
    above the gradients because Adam's g / (sqrt(v) + eps) turns bf16-level differences on
    near-zero gradient components into steps of up to lr (oracle.fixtures.adam_delta_close)."""
    rep, worst = _five_steps(bf16=True, lr=1e-4, fixture="train_steps5_tiny3d_lr1e-4.npz")
    assert rep["loss"] < 1e-3, rep
    assert worst["grad1"] < 4e-2 and worst["grad5"] < 5e-2, (worst, rep)
    assert worst["delta5"] < 1e-1, (worst, rep)


def test_trainer_five_steps_fp32_at_bench_lr_match_reference():
    """The fp32 parity-mode Trainer against the same lr-1e-4 fixture: the bars of the lr-1e-2
    fp32 pin (the GPU's fp32 reductions differ from the CPU's in order only; measured round 6:
    losses 9.4e-8, step-1 / step-5 gradients 1.9e-6 / 5.0e-6, five-step change 1.8e-5)."""
    rep, worst = _five_steps(bf16=False, lr=1e-4, fixture="train_steps5_tiny3d_lr1e-4.npz")
    assert rep["loss"] < 1e-4, rep
    assert worst["grad1"] < 1e-4 and worst["grad5"] < 1e-3, rep
    assert worst["delta5"] < 5e-4, rep


def _pack_runs(m, modes, lr, steps=3):
    """Train copies of m for `steps` bf16 steps, one per entry of modes (batch_pack flags);
    returns per run (losses, per-step gradients by name, final parameters) and the last
    trainer.  Asserts that from the second step on no per-call pack runs for a Parameter."""
    import copy
    from vdiff import ops
    from vdiff.engine import Clip, Trainer
    from vdiff.schedulers import LinearNoiseScheduler
    runs, tr = [], None
    for batch_pack in modes:
        mm = copy.deepcopy(m)
        tr = Trainer(mm, LinearNoiseScheduler(100, 0.00085, 0.012), lr=lr, batch_pack=batch_pack)
        calls, grads = [], []
        hooks = [p.register_post_accumulate_grad_hook(
            lambda p, n=n: grads[-1].__setitem__(n, p.grad.detach().clone()))
            for n, p in mm.named_parameters()]
        orig = ops._pack_weight_now
        ops._pack_weight_now = lambda w, *a, _o=orig: calls.append(w) or _o(w, *a)
        try:
            losses = []
            for s in range(steps):
                gen = torch.Generator(device=dev).manual_seed(s)
                x0 = torch.rand((1, 3, 4, 32, 32), generator=gen, device=dev) * 2 - 1
                cond = torch.rand((1, 3, 32, 32), generator=gen, device=dev) * 2 - 1
                feat = torch.randn((4, 64), generator=gen, device=dev)
                eps = torch.randn(x0.shape, generator=gen, device=dev)
                n0 = len(calls)
                grads.append({})
                losses.append(tr.step(Clip(x0, cond, feat, eps, torch.tensor([7 + s], device=dev))))
                if batch_pack and s > 0:
                    assert not any(isinstance(w, torch.nn.Parameter) for w in calls[n0:])
        finally:
            ops._pack_weight_now = orig
            for h in hooks:
                h.remove()
        runs.append((torch.stack(losses), grads, [p.detach().clone() for p in mm.parameters()]))
    return runs, tr


def _pack_model():
    from vdiff.unet_audio import UNetAudio
    m = UNetAudio(image_size=32, in_channels=3, model_channels=32, out_channels=3,
                  num_res_blocks=1, attention_resolutions=(2,), channel_mult=(1, 2), dims=3,
                  audio_feature_dim=64, projected_audio_dim=16, im_cond_output_ch=16,
                  dropout=0.0, audio_encoder=False)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    m.load_state_dict(init_params(shapes, 5))
    m.convert_to_fp16()
    return m.to(dev)


def test_trainer_batched_pack_equals_per_call_pack():
    """the conv operands re-packed once per step in one launch
    (ops.step_packed_weights, vd_conv_pack_weights) are bit-identical to per-call packs of the
    same weights, from the second step on no per-call pack runs for a Parameter, and -- every
    reduction of the step being fixed-order since round 4 (conv weight gradients, GroupNorm
    backward sums, conditioning backward) -- three bf16 train steps at lr 1e-3 give
    bit-identical losses, gradients and parameters with the batched pack and with per-call
    packs, and two per-call runs are bit-identical to each other."""
    from vdiff import ops
    runs, tr = _pack_runs(_pack_model(), (False, False, True), lr=1e-3)
    sp = tr.packs
    assert len(sp.bufs) >= 20
    with sp:
        for k, (w, Co, Ci, taps, Cip, Cop, trn, dt) in sp.want.items():
            assert torch.equal(sp.bufs[k], ops._pack_weight_now(w, Co, Ci, taps, Cip, Cop, trn, dt))
    for other in (runs[1], runs[2]):
        assert torch.equal(other[0], runs[0][0]), (other[0], runs[0][0])
        for s, (ga, gb) in enumerate(zip(runs[0][1], other[1])):
            assert ga.keys() == gb.keys()
            for n in ga:
                assert torch.equal(ga[n], gb[n]), (s, n)
        for a, b in zip(runs[0][2], other[2]):
            assert torch.equal(a, b)


def test_trainer_lr0_gradients_bit_identical():
    """At lr 0 the weights never move, so all three steps see the same operands: the batched
    pack's gradients equal the per-call run's bit for bit at every step (the localisation
    VERDICT r03 item 1 asked for, kept as a test)."""
    runs, _ = _pack_runs(_pack_model(), (False, True), lr=0.0)
    for s, (ga, gb) in enumerate(zip(runs[0][1], runs[1][1])):
        for n in ga:
            assert torch.equal(ga[n], gb[n]), (s, n)
    assert torch.equal(runs[0][0], runs[1][0])


def test_batched_pack_plan_survives_moved_weights():
    """A weight whose storage is replaced between steps (here .data = a new tensor) drops
    the batched-pack plan before its launch (the old pointer is never read) and the step
    still packs the current weights: the conv output equals a fresh per-call pack's."""
    from vdiff import ops
    w = torch.nn.Parameter(torch.randn(64, 32, 3, 3, 3, device=dev) * 0.05)
    x = ops.to_cl(torch.randn(1, 32, 4, 16, 16, device=dev).bfloat16())
    sp = ops.step_packed_weights()
    with sp:
        ops.conv(x, w, padding=1)
    assert sp.dirty is False and sp.plans  # plan built at the end of the first step
    w.data = torch.randn_like(w) * 0.05      # new storage
    with sp:
        y = ops.conv(x, w, padding=1)
    y0 = ops.conv(x, w, padding=1)          # no plan: per-call pack
    assert torch.equal(y, y0)
