"""Audio cross-attention (north_star build extension): video tokens attend to the wav2vec2
tokens of their frame's audio window.  No reference counterpart exists (the reference
conditions on audio by concatenation, unet_audio.py:52-61), so parity is pinned through the
oracle (oracle.nn.cross_attention), which is itself pinned to the reference's QKVAttention
math (tests/test_oracle_golden.py::test_cross_attention_oracle_reduces_to_reference).
Tolerances: fp32 2e-5 (kernels) / 1e-4 (models), bf16 2e-2 (outputs) / 4e-2 (gradients)."""
import pytest
import torch

from oracle import nn as onn
from oracle.fixtures import rel_l2, seeded
from oracle.unet import audio_conditioned_input, build_plan, init_params, unet_forward

pytestmark = pytest.mark.gpu
dev = "cuda"


def _check(B, C, heads, T, HW, L, per_frame, dtype, seed):
    from vdiff import ops
    q = seeded((B, C, T * HW), seed)
    kv = seeded((B * T, L, 2 * C), seed + 1)
    if dtype == torch.bfloat16:
        q, kv = q.bfloat16().float(), kv.bfloat16().float()
    qr, kvr = q.clone().requires_grad_(True), kv.clone().requires_grad_(True)
    ref = onn.cross_attention(qr, kvr, heads, T, per_frame)
    g = seeded(ref.shape, seed + 2)
    ref.backward(g)
    qd = ops.to_cl(q.to(dev, dtype)).requires_grad_(True)
    kvd = kv.to(dev, dtype).requires_grad_(True)
    out = ops.cross_attention(qd, kvd, heads, T, per_frame)
    out.backward(ops.to_cl(g.to(dev, dtype)))
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    e = (rel_l2(out, ref), rel_l2(qd.grad, qr.grad), rel_l2(kvd.grad, kvr.grad))
    assert e[0] < tol and e[1] < 2 * tol and e[2] < 2 * tol, e


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("C", [32, 64, 128, 256])
def test_per_frame_head_dims(C, dtype):
    _check(2, C, 1, 3, 67, 12, True, dtype, 100 + C)  # ragged query tiles, 12 audio tokens


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_clip_level_and_heads(dtype):
    _check(2, 128, 2, 4, 36, 12, False, dtype, 200)   # all T*HW tokens onto all T*12
    _check(1, 128, 4, 2, 50, 7, True, dtype, 201)


def test_query_split_and_long_kv():
    """bf16: a key grid too small for the chip splits the queries (fp32 dK/dV partials);
    more than one 64-key tile of audio tokens."""
    _check(1, 64, 1, 1, 3000, 12, True, torch.bfloat16, 300)
    _check(1, 64, 1, 2, 700, 150, True, torch.bfloat16, 301)
    _check(1, 64, 1, 2, 700, 150, True, torch.float32, 302)


def test_attention_block_with_audio_matches_oracle():
    from vdiff.nn import AttentionBlock
    ab = AttentionBlock(64, attention_mode="joint", audio_attention=True, audio_context_dim=48)
    shapes = {k: tuple(v.shape) for k, v in ab.state_dict().items()}
    P = init_params(shapes, 17)
    ab.load_state_dict(P)
    ab = ab.to(dev)
    x = seeded((2, 64, 3, 6, 6), 18)
    ctx = seeded((6, 12, 48), 19)
    Pr = {k: v.clone().requires_grad_(True) for k, v in P.items()}
    xr, cr = x.clone().requires_grad_(True), ctx.clone().requires_grad_(True)
    yr = onn.attention_block(Pr, "", xr, context=cr)
    xd = x.to(dev).requires_grad_(True)
    cd = ctx.to(dev).requires_grad_(True)
    y = ab(xd, context=cd)
    assert rel_l2(y, yr) < 1e-5
    g = seeded(y.shape, 20)
    yr.backward(g)
    y.backward(g.to(dev))
    assert rel_l2(xd.grad, xr.grad) < 1e-5
    assert rel_l2(cd.grad, cr.grad) < 1e-5
    named = dict(ab.named_parameters())
    for k in ("audio_q.weight", "audio_kv.weight", "audio_proj_out.weight", "audio_norm.weight"):
        assert rel_l2(named[k].grad, Pr[k].grad) < 1e-5, k


def test_unet_audio_with_cross_attention_matches_oracle():
    """The 5-D audio-conditioned UNet3D with audio_attention=True: tokens [B*T, 12, F] feed
    the cross-attention branches and, mean-pooled, the concat conditioning."""
    from vdiff.unet_audio import UNetAudio
    cfg = dict(image_size=16, in_channels=3, model_channels=32, out_channels=3,
               num_res_blocks=1, attention_resolutions=(2,), channel_mult=(1, 2), dims=3,
               audio_feature_dim=64, projected_audio_dim=16, im_cond_output_ch=16, dropout=0.0)
    m = UNetAudio(**cfg, audio_encoder=False, audio_attention=True)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    P = init_params(shapes, 23)
    m.load_state_dict(P)
    m = m.to(dev)
    image = seeded((2, 3, 4, 16, 16), 24, "uniform")
    cond = seeded((2, 3, 8, 8), 25, "uniform")
    tokens = seeded((8, 12, 64), 26)
    t = torch.tensor([3, 70])
    y = m(image.to(dev), cond.to(dev), tokens.to(dev), t.to(dev))
    plan = build_plan(in_channels=35, model_channels=32, out_channels=3, num_res_blocks=1,
                      attention_resolutions=(2,), channel_mult=(1, 2), dims=3, audio_attention=64)
    Pr = {k: v.clone().requires_grad_(True) for k, v in P.items()}
    xin = audio_conditioned_input(Pr, image, cond, tokens.mean(1), 16)
    yr = unet_forward(Pr, plan, xin, t, context=tokens)
    assert rel_l2(y, yr) < 1e-4
    g = seeded(yr.shape, 27)
    yr.backward(g)
    y.backward(g.to(dev))
    named = dict(m.named_parameters())
    for k in ("input_blocks.3.1.audio_kv.weight", "input_blocks.3.1.audio_q.weight",
              "middle_block.1.audio_proj_out.weight", "audio_transformer.transform.0.weight"):
        assert rel_l2(named[k].grad, Pr[k].grad) < 1e-4, k
    # bf16 throughput mode against the same fp32 oracle
    m.convert_to_fp16()
    y16 = m(image.to(dev), cond.to(dev), tokens.to(dev), t.to(dev))
    assert rel_l2(y16, yr) < 3e-2
