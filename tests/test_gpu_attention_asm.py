"""The hand-scheduled head_dim-64 backward kernels (vd_attn_bwd_dq_d64 and
vd_attn_bwd_dkdv_d64, csrc/asm/gen_attn_asm.py, attention config "asm", the head_dim-64 backward default) against the compiler-scheduled
pipelined kernels (config "p8", whose forward is the default deferred-check forward) on the
same bf16 inputs, and against a materialised fp32 reference of QKVAttentionLegacy's backward
(unet.py:349-366).  The asm kernel runs the same products in the same accumulation order,
so dQ, dK and dV agree with the pipelined kernels' to fp32 rounding (bound 1e-6 rel-L2).
Shapes: joint attention with whole and ragged last tiles, a batch of two sequences, and
spatial grouping (4 frames x 1024 tokens: groups on grid.y) -- the kernel takes N >= 1024."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


def _grads(qkv, g, cfg, **kw):
    from vdiff import ops
    x = qkv.detach().clone().requires_grad_(True)
    with ops.attention_config(cfg):
        y = ops.attention(x, 1, **kw)
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


@pytest.mark.parametrize("B,N,seed", [(1, 1024, 0), (1, 4096, 1), (1, 5000, 2), (2, 3000, 3),
                                      (1, 65536 + 17, 4)])
def test_asm_bwd_equals_pipelined_kernels(B, N, seed):
    qkv, g = _inputs(B, N, seed)
    y0, g0 = _grads(qkv, g, "p8")
    y1, g1 = _grads(qkv, g, "asm")
    assert torch.equal(y0, y1)                     # the forward is not affected
    assert torch.isfinite(g1.float()).all()
    for name, sl in (("dq", slice(0, 64)), ("dk", slice(64, 128)), ("dv", slice(128, 192))):
        a, b = g0[:, sl].float(), g1[:, sl].float()
        assert b.abs().max() > 0, name
        err = float((a - b).norm() / a.norm())
        assert err <= 1e-6, (name, err)


def test_asm_bwd_spatial_groups():
    qkv, g = _inputs(1, None, 5, spatial=(4, 32, 32))
    kw = dict(mode="spatial", spatial=(4, 32, 32))
    _, g0 = _grads(qkv, g, "p8", **kw)
    _, g1 = _grads(qkv, g, "asm", **kw)
    err = float((g0.float() - g1.float()).norm() / g0.float().norm())
    assert err <= 1e-6, err


def test_asm_is_the_d64_backward_default():
    qkv, g = _inputs(1, 2048, 7)
    _, g0 = _grads(qkv, g, "auto")
    _, g1 = _grads(qkv, g, "asm")
    assert torch.equal(g0, g1)


def test_asm_bwd_against_fp32_reference():
    N, C = 4096, 64
    qkv, g = _inputs(1, N, 6)
    _, gr = _grads(qkv, g, "asm")
    t = qkv.float()[0].detach()                       # logical [3C, N]
    q, k, v = t[:C].T, t[C:2 * C].T, t[2 * C:].T      # [N, C]
    q, k, v = (u.clone().requires_grad_(True) for u in (q, k, v))
    s = (q @ k.T) / math.sqrt(C)
    o = torch.softmax(s, -1) @ v
    o.backward(g.float()[0].T)
    for got, ref in ((gr[0, :C], q.grad), (gr[0, C:2 * C], k.grad), (gr[0, 2 * C:], v.grad)):
        e = float((got.float().T - ref).norm() / ref.norm())
        assert e < 2e-2, e
