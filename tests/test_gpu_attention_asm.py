"""The hand-scheduled head_dim-64 kernels (csrc/asm/gen_attn_asm.py, gen_fwd.py; attention
config "asm", the head_dim-64 default) against the compiler-scheduled kernels and a
materialised fp32 reference of QKVAttentionLegacy (unet.py:349-366).

Backward (vd_attn_bwd_dq_d64, vd_attn_bwd_dkdv_d64): the same products in the same
accumulation order as the pipelined kernels (config "p8"), so with the SAME forward (the
forward runs under one config, the backward under the other) dQ, dK and dV agree to fp32
rounding (bound 1e-6 rel-L2).
Forward (vd_attn_fwd_d64): the deferred-check forward's algorithm (lagged max, bf16 P,
fp32 row sums) with a different summation order and rare-path timing, so O agrees with the
deferred-check kernel (config "p8" selects it) to bf16 rounding (rel-L2 <= 4e-3, lse to
2e-5 absolute) and with the fp32 reference as closely as it does.
Shapes: joint attention with whole and ragged last tiles (the masked last iteration), a
batch of two sequences, spatial grouping (4 frames x 1024 tokens: groups on grid.y), late
logit jumps (the rare path past the first tile) -- the kernels take N >= 1024."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


def _run(qkv, g, fwd_cfg, bwd_cfg=None, **kw):
    from vdiff import ops
    x = qkv.detach().clone().requires_grad_(True)
    with ops.attention_config(fwd_cfg):
        y = ops.attention(x, 1, **kw)
    lse = y.grad_fn.saved_tensors[2].detach().clone()
    if bwd_cfg is None:
        return y.detach(), lse
    with ops.attention_config(bwd_cfg):
        y.backward(g)
    torch.cuda.synchronize()
    return y.detach(), x.grad.detach()


def _inputs(B, N, seed, spatial=None):
    from vdiff import ops
    gen = torch.Generator(device=dev).manual_seed(seed)
    shape = (B, 192, N if spatial is None else math.prod(spatial))
    qkv = torch.randn(shape, generator=gen, device=dev) * 1.3
    gout = torch.randn((B, 64, shape[2]), generator=gen, device=dev)
    return ops.to_cl(qkv.bfloat16()), ops.to_cl(gout.bfloat16())


def _reference(qkv, C=64):
    t = qkv.float()[0].detach()                       # logical [3C, N]
    q, k, v = t[:C].T, t[C:2 * C].T, t[2 * C:].T      # [N, C]
    s = (q @ k.T) / math.sqrt(C)
    return torch.softmax(s, -1) @ v, torch.logsumexp(s, -1)


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm())


@pytest.mark.parametrize("B,N,seed", [(1, 1024, 0), (1, 4096, 1), (1, 5000, 2), (2, 3000, 3),
                                      (1, 65536 + 17, 4)])
def test_asm_bwd_equals_pipelined_kernels(B, N, seed):
    qkv, g = _inputs(B, N, seed)
    y0, g0 = _run(qkv, g, "asm", "p8")
    y1, g1 = _run(qkv, g, "asm", "asm")
    assert torch.equal(y0, y1)
    assert torch.isfinite(g1.float()).all()
    for name, sl in (("dq", slice(0, 64)), ("dk", slice(64, 128)), ("dv", slice(128, 192))):
        a, b = g0[:, sl].float(), g1[:, sl].float()
        assert b.abs().max() > 0, name
        err = float((a - b).norm() / a.norm())
        assert err <= 1e-6, (name, err)


def test_asm_bwd_spatial_groups():
    qkv, g = _inputs(1, None, 5, spatial=(4, 32, 32))
    kw = dict(mode="spatial", spatial=(4, 32, 32))
    _, g0 = _run(qkv, g, "asm", "p8", **kw)
    _, g1 = _run(qkv, g, "asm", "asm", **kw)
    assert _rel(g1, g0) <= 1e-6


def test_asm_bwd_against_fp32_reference():
    N, C = 4096, 64
    qkv, g = _inputs(1, N, 6)
    _, gr = _run(qkv, g, "asm", "asm")
    t = qkv.float()[0].detach()
    q, k, v = t[:C].T, t[C:2 * C].T, t[2 * C:].T
    q, k, v = (u.clone().requires_grad_(True) for u in (q, k, v))
    s = (q @ k.T) / math.sqrt(C)
    o = torch.softmax(s, -1) @ v
    o.backward(g.float()[0].T)
    for got, ref in ((gr[0, :C], q.grad), (gr[0, C:2 * C], k.grad), (gr[0, 2 * C:], v.grad)):
        e = float((got.float().T - ref).norm() / ref.norm())
        assert e < 2e-2, e


@pytest.mark.parametrize("B,N,seed", [(1, 1024, 10), (1, 1500, 11), (1, 4096, 12),
                                      (2, 3000, 13), (1, 65536 + 17, 14)])
def test_asm_fwd_against_deferred_check_kernel(B, N, seed):
    qkv, _ = _inputs(B, N, seed)
    y0, l0 = _run(qkv, None, "p8")
    y1, l1 = _run(qkv, None, "asm")
    assert torch.isfinite(y1.float()).all() and torch.isfinite(l1).all()
    assert _rel(y1, y0) <= 4e-3
    assert float((l1 - l0).abs().max()) <= 2e-5


def test_asm_fwd_against_fp32_reference():
    qkv, _ = _inputs(1, 4096, 15)
    y, lse = _run(qkv, None, "asm")
    yd, ld = _run(qkv, None, "p8")
    ref, lref = _reference(qkv)
    e, ed = _rel(y[0].T, ref), _rel(yd[0].T, ref)
    assert e <= max(1.25 * ed, 4e-3), (e, ed)
    # both kernels score with Q' = bf16(Q * scale * log2 e): lse carries its rounding
    el, eld = float((lse - lref).abs().max()), float((ld - lref).abs().max())
    assert el <= 1.25 * eld + 1e-5, (el, eld)


def test_asm_fwd_late_logit_jumps():
    """Keys far above every earlier score in late tiles and a query with a large max of its
    own: the rare path (true max, O / l rescale, S(t+1) recompute) past the first tile, in
    the unmasked iterations and in the masked last one."""
    from vdiff import ops
    N, C = 3000, 64
    gen = torch.Generator(device=dev).manual_seed(16)
    qkv = torch.randn((1, 3 * C, N), generator=gen, device=dev) * 3.0
    qkv[:, C:2 * C, 700] *= 12     # a jump in an unmasked iteration
    qkv[:, C:2 * C, 2900] *= 14    # ... and in the masked last one
    qkv[:, :C, 1300] *= 10
    qkv = ops.to_cl(qkv.bfloat16())
    y, lse = _run(qkv, None, "asm")
    yd, ld = _run(qkv, None, "p8")
    ref, lref = _reference(qkv)
    assert torch.isfinite(y.float()).all()
    assert _rel(y[0].T, ref) < 2e-2
    assert _rel(y, yd) <= 1e-2
    el, eld = float((lse - lref).abs().max()), float((ld - lref).abs().max())
    assert el <= 1.25 * eld + 1e-5, (el, eld)


def test_asm_fwd_spatial_groups():
    qkv, _ = _inputs(1, None, 17, spatial=(4, 32, 32))
    kw = dict(mode="spatial", spatial=(4, 32, 32))
    y0, l0 = _run(qkv, None, "p8", **kw)
    y1, l1 = _run(qkv, None, "asm", **kw)
    assert _rel(y1, y0) <= 4e-3
    assert float((l1 - l0).abs().max()) <= 2e-5


def test_asm_is_the_d64_default():
    qkv, g = _inputs(1, 2048, 7)
    y0, g0 = _run(qkv, g, "auto", "auto")
    y1, g1 = _run(qkv, g, "asm", "asm")
    assert torch.equal(y0, y1)
    assert torch.equal(g0, g1)
