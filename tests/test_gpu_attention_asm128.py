"""The hand-scheduled head_dim-128 backward kernels (csrc/asm/gen_d128.py,
vd_attn_bwd_dq_d128 and vd_attn_bwd_dkdv_d128; attention config "asm" at D = 128) against the
compiler-scheduled kernels and a materialised fp32 reference of QKVAttentionLegacy's backward
(unet.py:349-366 at C = 128).

With the same forward, the hand-scheduled kernels run the products of the 4-wave pipelined
kernels (config "p4": one 32-row block per wave, tiles in order) in the same accumulation
order, so dQ, dK and dV agree with them to fp32 rounding (bound 1e-6 rel-L2); against the
defaults (8-wave dQ, paired dK/dV whose SIMD partners sum half-tile partials at the end) they
agree to bf16 output rounding.  Shapes: whole and ragged last tiles, a batch of two sequences, the
spatial grouping of the 64x64 level (groups on grid.y), N = 65536 + 17 (config-2 size and
a ragged tail); the kernel takes N >= 1024."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"
C = 128


def _grads(qkv, g, fwd_cfg, bwd_cfg, **kw):
    from vdiff import ops
    x = qkv.detach().clone().requires_grad_(True)
    with ops.attention_config(fwd_cfg):
        y = ops.attention(x, 1, **kw)
    with ops.attention_config(bwd_cfg):
        y.backward(g)
    torch.cuda.synchronize()
    return x.grad.detach()


def _inputs(B, N, seed, spatial=None):
    from vdiff import ops
    gen = torch.Generator(device=dev).manual_seed(seed)
    n = N if spatial is None else math.prod(spatial)
    qkv = torch.randn((B, 3 * C, n), generator=gen, device=dev) * 1.3
    gout = torch.randn((B, C, n), generator=gen, device=dev)
    return ops.to_cl(qkv.bfloat16()), ops.to_cl(gout.bfloat16())


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm())


@pytest.mark.parametrize("B,N,seed", [(1, 1024, 0), (1, 4096, 1), (1, 5000, 2), (2, 3000, 3),
                                      (1, 65536 + 17, 4)])
def test_asm128_bwd_equals_pipelined_kernels(B, N, seed):
    qkv, g = _inputs(B, N, seed)
    g0 = _grads(qkv, g, "auto", "p4")
    g1 = _grads(qkv, g, "auto", "asm")
    assert torch.isfinite(g1.float()).all()
    for name, sl in (("dq", slice(0, C)), ("dk", slice(C, 2 * C)), ("dv", slice(2 * C, 3 * C))):
        a, b = g0[:, sl].float(), g1[:, sl].float()
        assert b.abs().max() > 0, name
        err = float((a - b).norm() / a.norm())
        assert err <= 1e-6, (name, err)


@pytest.mark.parametrize("B,N,seed", [(1, 4096, 5), (1, 65536, 6)])
def test_asm128_bwd_against_default_kernels(B, N, seed):
    qkv, g = _inputs(B, N, seed)
    g0 = _grads(qkv, g, "auto", "w8")    # dQ: the 8-wave kernel (the default)
    g1 = _grads(qkv, g, "auto", "asm")
    assert _rel(g1[:, :C], g0[:, :C]) <= 4e-3
    g0 = _grads(qkv, g, "auto", "pair")  # dK / dV: the paired kernel (the default)
    assert _rel(g1[:, C:], g0[:, C:]) <= 4e-3


def test_asm128_spatial_groups():
    qkv, g = _inputs(1, None, 7, spatial=(4, 32, 32))
    kw = dict(mode="spatial", spatial=(4, 32, 32))
    g0 = _grads(qkv, g, "auto", "p4", **kw)
    g1 = _grads(qkv, g, "auto", "asm", **kw)
    assert _rel(g1, g0) <= 1e-6


def test_asm128_against_fp32_reference():
    N = 4096
    qkv, g = _inputs(1, N, 8)
    gr = _grads(qkv, g, "auto", "asm")
    t = qkv.float()[0].detach()
    q, k, v = t[:C].T, t[C:2 * C].T, t[2 * C:].T
    q, k, v = (u.clone().requires_grad_(True) for u in (q, k, v))
    o = torch.softmax((q @ k.T) / math.sqrt(C), -1) @ v
    o.backward(g.float()[0].T)
    for got, ref in ((gr[0, :C], q.grad), (gr[0, C:2 * C], k.grad), (gr[0, 2 * C:], v.grad)):
        e = float((got.float().T - ref).norm() / ref.norm())
        assert e < 2e-2, e


# ------------------------------------------------------------------ forward (gen_fwd128.py)
def _fwd(qkv, cfg, **kw):
    from vdiff import ops
    x = qkv.detach().clone().requires_grad_(True)
    with ops.attention_config(cfg):
        y = ops.attention(x, 1, **kw)
    lse = y.grad_fn.saved_tensors[2].detach().clone()
    torch.cuda.synchronize()
    return y.detach(), lse


def _reference(qkv):
    t = qkv.float()[0].detach()
    q, k, v = t[:C].T, t[C:2 * C].T, t[2 * C:].T
    s = (q @ k.T) / math.sqrt(C)
    return torch.softmax(s, -1) @ v, torch.logsumexp(s, -1)


@pytest.mark.parametrize("B,N,seed", [(1, 1024, 20), (1, 1500, 21), (1, 4096, 22),
                                      (2, 3000, 23), (1, 65536 + 17, 24)])
def test_asm128_fwd_against_deferred_check_kernel(B, N, seed):
    """vd_attn_fwd_d128 runs the deferred-check forward's algorithm (lagged max, bf16 P,
    fp32 row sums) with 32-key tiles and another summation order: O to bf16 rounding, lse
    to 2e-5."""
    qkv, _ = _inputs(B, N, seed)
    y0, l0 = _fwd(qkv, "d8n")
    y1, l1 = _fwd(qkv, "asm")
    assert torch.isfinite(y1.float()).all() and torch.isfinite(l1).all()
    assert _rel(y1, y0) <= 4e-3
    assert float((l1 - l0).abs().max()) <= 2e-5


def test_asm128_fwd_against_fp32_reference():
    qkv, _ = _inputs(1, 4096, 25)
    y, lse = _fwd(qkv, "asm")
    yd, ld = _fwd(qkv, "d8n")
    ref, lref = _reference(qkv)
    e, ed = _rel(y[0].T, ref), _rel(yd[0].T, ref)
    assert e <= max(1.25 * ed, 4e-3), (e, ed)
    el, eld = float((lse - lref).abs().max()), float((ld - lref).abs().max())
    assert el <= 1.25 * eld + 1e-5, (el, eld)


def test_asm128_fwd_late_logit_jumps():
    """Keys far above every earlier score in late tiles (the rare path past the first tile,
    in an unmasked iteration and in the masked last one) and a query with a large max."""
    from vdiff import ops
    N = 3000
    gen = torch.Generator(device=dev).manual_seed(26)
    qkv = torch.randn((1, 3 * C, N), generator=gen, device=dev) * 2.0
    qkv[:, C:2 * C, 700] *= 12
    qkv[:, C:2 * C, 2900] *= 14
    qkv[:, :C, 1300] *= 10
    qkv = ops.to_cl(qkv.bfloat16())
    y, lse = _fwd(qkv, "asm")
    yd, ld = _fwd(qkv, "d8n")
    ref, lref = _reference(qkv)
    assert torch.isfinite(y.float()).all()
    assert _rel(y[0].T, ref) < 2e-2
    assert _rel(y, yd) <= 1e-2
    el, eld = float((lse - lref).abs().max()), float((ld - lref).abs().max())
    assert el <= 1.25 * eld + 1e-5, (el, eld)


def test_asm128_fwd_spatial_groups():
    qkv, _ = _inputs(1, None, 27, spatial=(4, 32, 32))
    kw = dict(mode="spatial", spatial=(4, 32, 32))
    y0, l0 = _fwd(qkv, "d8n", **kw)
    y1, l1 = _fwd(qkv, "asm", **kw)
    assert _rel(y1, y0) <= 4e-3
    assert float((l1 - l0).abs().max()) <= 2e-5


def test_asm128_is_the_d128_default():
    qkv, g = _inputs(1, 2048, 28)
    y0, l0 = _fwd(qkv, "auto")
    y1, l1 = _fwd(qkv, "asm")
    assert torch.equal(y0, y1) and torch.equal(l0, l1)
    assert torch.equal(_grads(qkv, g, "auto", "auto"), _grads(qkv, g, "asm", "asm"))
