"""Short-sequence attention (attn_short.hip: one wave per sequence of <= 32 tokens, 16x16
MFMA tiles, a fused dQ / dK / dV backward) -- the temporal half of the spatial_temporal
mode (T = 16 at config 2, 25 at config 4, one sequence per pixel) and the ViViT encoder's
9-token heads -- against the oracle's materialised softmax attention (oracle.nn.qkv_attention,
pinned to the reference QKVAttentionLegacy / QKVAttention by the golden regroupings) in fp32
on the same bf16-rounded inputs, and against the flash kernels (vd_attention_set_short(0)).
Bars: bf16 output rel-L2 <= 1e-2 and gradients <= 2e-2 against fp32 (P and dS are rounded to
bf16 once, as in the flash kernels); lse within 1e-3 + 1e-4 |lse|."""
import math

import pytest
import torch

from oracle import nn as onn
from oracle.fixtures import rel_l2, seeded

from conftest import record_metric

pytestmark = pytest.mark.gpu
dev = "cuda"


def _run(B, C, heads, T, HW, mode, legacy, seed, amp=1.0):
    from vdiff import ops
    N = T * HW
    qkv = (seeded((B, 3 * C, N), seed) * amp).bfloat16().float()
    qr = qkv.clone().requires_grad_(True)
    ref = onn.qkv_attention(qr, heads, legacy=legacy, mode=mode, spatial=(T, HW, 1))
    g = seeded(ref.shape, seed + 1)
    ref.backward(g)
    qd = ops.to_cl(qkv.to(dev, torch.bfloat16)).requires_grad_(True)
    out = ops.attention(qd, heads=heads, mode=mode, spatial=(T, HW, 1), legacy=legacy)
    out.backward(ops.to_cl(g.to(dev, torch.bfloat16)))
    return rel_l2(out, ref), rel_l2(qd.grad, qr.grad), out.detach(), qd.grad.detach()


def _uses_short(B, C, heads, T, HW, mode, legacy):
    from vdiff import _lib, ops
    d = ops._attn_desc(B, T * HW, C, heads, C // heads, mode, (T, HW, 1), _lib.VD_BF16, legacy)
    return all(_lib.lib().vd_attention_short_path(x[0]) for x in d)


@pytest.mark.parametrize("C", [64, 128, 256])
@pytest.mark.parametrize("T", [16, 25])
def test_temporal_bf16_vs_oracle(C, T):
    """The temporal mode at the two BASELINE frame counts and the three level widths."""
    B, HW = 2, 48
    assert _uses_short(B, C, 1, T, HW, "temporal", True)
    e_o, e_g, _, _ = _run(B, C, 1, T, HW, "temporal", True, 100 + C + T)
    record_metric(test="short_attention_temporal", C=C, T=T, out=e_o, grad=e_g)
    assert e_o < 1e-2 and e_g < 2e-2, (e_o, e_g)


@pytest.mark.parametrize("T", [1, 2, 5, 9, 15, 17, 31, 32])
def test_ragged_lengths(T):
    """Every padding case of the 16 / 32-token tiles: masked keys, masked queries."""
    e_o, e_g, _, _ = _run(1, 64, 1, T, 37, "temporal", True, 200 + T)
    assert e_o < 1e-2 and e_g < 2e-2, (T, e_o, e_g)


@pytest.mark.parametrize("legacy", [True, False])
def test_multi_head_and_joint_short(legacy):
    """Heads as sequence groups (QKVAttentionLegacy and QKVAttention orders), and joint mode
    over 9 tokens with 8 heads of 32 channels (the ViViT encoder's attention shape)."""
    e_o, e_g, _, _ = _run(2, 128, 2, 16, 20, "temporal", legacy, 300)
    assert e_o < 1e-2 and e_g < 2e-2, (e_o, e_g)
    assert _uses_short(16, 256, 8, 1, 9, "joint", legacy)
    e_o, e_g, _, _ = _run(16, 256, 8, 1, 9, "joint", legacy, 301)
    assert e_o < 1e-2 and e_g < 2e-2, (e_o, e_g)


def test_large_logits_and_lse():
    """Peaked softmax (|logit| up to ~60): the max subtraction, and the saved lse against
    the fp32 log-sum-exp."""
    from vdiff import _lib, ops
    B, C, T, HW = 1, 64, 16, 64
    e_o, e_g, _, _ = _run(B, C, 1, T, HW, "temporal", True, 400, amp=4.0)
    assert e_o < 1e-2 and e_g < 3e-2, (e_o, e_g)
    qkv = (seeded((B, 3 * C, T * HW), 401) * 3.0).bfloat16()
    x = ops.to_cl(qkv.to(dev))
    (d, qo, ko, vo, oo), = ops._attn_desc(B, T * HW, C, 1, C, "temporal", (T, HW, 1),
                                          _lib.VD_BF16, True)
    out = ops.empty_cl([B, C, T * HW], torch.bfloat16, dev)
    lse = torch.empty(d.nseq * d.seq_len, dtype=torch.float32, device=dev)
    base = x.data_ptr()
    _lib.call("vd_attention_fwd_ws", d, base + qo * 2, base + ko * 2, base + vo * 2,
              out.data_ptr(), lse.data_ptr(), None, 0, torch.cuda.current_stream().cuda_stream)
    q, k, _ = qkv.float().reshape(B, 3, C, T, HW).unbind(1)
    s = torch.einsum("ctp,cup->ptu", q[0], k[0]) / math.sqrt(C)   # [pixel, query t, key u]
    ref = torch.logsumexp(s, dim=-1).reshape(-1)
    err = (lse.cpu() - ref).abs()
    assert bool((err <= 1e-3 + 1e-4 * ref.abs()).all()), float(err.max())


def test_short_equals_flash_kernels():
    """The same temporal launch on the short kernels and on the flash kernels (the previous
    path, vd_attention_set_short(0)): two bf16 evaluations of one fp32 reference."""
    from vdiff import _lib
    lib = _lib.lib()
    prev = lib.vd_attention_set_short(0)
    try:
        _, _, o_f, g_f = _run(2, 64, 1, 16, 40, "temporal", True, 500)
    finally:
        lib.vd_attention_set_short(prev)
    _, _, o_s, g_s = _run(2, 64, 1, 16, 40, "temporal", True, 500)
    assert rel_l2(o_s.float(), o_f.float()) < 1e-2
    assert rel_l2(g_s.float(), g_f.float()) < 2e-2


def test_short_path_predicate():
    """vd_attention_short_path: bf16 with <= 32 tokens only; fp32 (parity mode) and longer
    sequences keep the flash kernels."""
    from vdiff import _lib, ops
    lib = _lib.lib()
    for T, dt, want in ((16, _lib.VD_BF16, 1), (32, _lib.VD_BF16, 1), (33, _lib.VD_BF16, 0),
                        (16, _lib.VD_F32, 0)):
        (d, *_), = ops._attn_desc(1, T * 8, 64, 1, 64, "temporal", (T, 8, 1), dt, True)
        assert lib.vd_attention_short_path(d) == want, (T, dt)


def test_backward_with_misaligned_gradient_falls_back_to_flash():
    """Advisor r05: the backward decides on the real buffers.  With aligned q / k / v / o (the
    forward on the short kernel) but a dout that is not 16-B aligned, vd_attention_bwd_short_path
    says 0 and vd_attention_bwd runs the flash dQ + dK/dV kernels with a workspace, giving the
    gradients of the aligned call (which takes the fused short kernel) within bf16 rounding."""
    from vdiff import _lib, ops
    lib = _lib.lib()
    B, C, T, HW = 1, 64, 16, 24
    N = T * HW
    (d, qo, ko, vo, oo), = ops._attn_desc(B, N, C, 1, C, "temporal", (T, HW, 1), _lib.VD_BF16,
                                          True)
    g = torch.Generator(device=dev).manual_seed(3)
    qkv = (torch.randn(B, N, 3 * C, generator=g, device=dev)).bfloat16()
    out = torch.empty(B, N, C, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(d.nseq * d.seq_len, dtype=torch.float32, device=dev)
    es = 2
    base = qkv.data_ptr()
    st = ops._stream(qkv)
    _lib.call("vd_attention_fwd_ws", d, base + qo * es, base + ko * es, base + vo * es,
              out.data_ptr(), lse.data_ptr(), None, 0, st)
    dsrc = torch.randn(B * N * C, generator=g, device=dev).bfloat16()
    dout_buf = torch.zeros(B * N * C + 8, dtype=torch.bfloat16, device=dev)
    grads = {}
    for name, off in (("aligned", 0), ("misaligned", 1)):
        dout = dout_buf[off:off + B * N * C]
        dout.copy_(dsrc)
        dq = torch.zeros(B, N, 3 * C, dtype=torch.bfloat16, device=dev)
        ptrs = (base + qo * es, base + ko * es, base + vo * es, out.data_ptr(), dout.data_ptr(),
                dq.data_ptr() + qo * es, dq.data_ptr() + ko * es, dq.data_ptr() + vo * es)
        short = lib.vd_attention_bwd_short_path(d, *ptrs)
        assert short == (1 if off == 0 else 0), (name, short)
        ws = torch.empty(max(1, lib.vd_attention_bwd_workspace_size(d)), dtype=torch.uint8,
                         device=dev)
        _lib.call("vd_attention_bwd", d, ptrs[0], ptrs[1], ptrs[2], ptrs[3], ptrs[4],
                  lse.data_ptr(), ptrs[5], ptrs[6], ptrs[7], ws.data_ptr(), st)
        grads[name] = dq.float()
    torch.cuda.synchronize()
    assert grads["aligned"].abs().max() > 0
    assert rel_l2(grads["misaligned"], grads["aligned"]) < 2e-2
