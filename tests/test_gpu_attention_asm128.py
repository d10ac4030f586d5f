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
