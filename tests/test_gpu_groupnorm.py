"""Fused GroupNorm(+SiLU) HIP kernels vs the reference golden vectors and the oracle."""
import pytest
import torch

from oracle import nn as onn
from oracle.fixtures import rel_l2, seeded

from conftest import golden

pytestmark = pytest.mark.gpu
dev = "cuda"


def _run(x, w, b, silu, dtype, g):
    from vdiff import ops
    xd = ops.to_cl(x.to(dev, dtype)).requires_grad_(True)
    wd = w.to(dev).clone().requires_grad_(True)
    bd = b.to(dev).clone().requires_grad_(True)
    y = ops.group_norm_silu(xd, wd, bd, 32, 1e-5, silu)
    y.backward(ops.to_cl(g.to(dev, dtype)))
    return y.float().cpu(), xd.grad.float().cpu(), wd.grad.cpu(), bd.grad.cpu()


def test_gn_silu_golden_fp32():
    gg = golden("blocks.npz")
    x = seeded((2, 64, 2, 6, 6), 20)
    g = seeded(x.shape, 22)
    y, dx, dw, db = _run(x, gg["gn_w"], gg["gn_b"], True, torch.float32, g)
    torch.testing.assert_close(y, gg["gn_y"], atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(dx, gg["gn_dx"], atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(dw, gg["gn_dw"], atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(db, gg["gn_db"], atol=1e-4, rtol=1e-4)


def test_gn_plain_golden_fp32_offset_mean():
    gg = golden("blocks.npz")
    x = seeded((2, 128, 40), 23) * 3 + 1.5
    g = seeded(x.shape, 25)
    y, dx, dw, db = _run(x, gg["gn2_w"], gg["gn2_b"], False, torch.float32, g)
    torch.testing.assert_close(y, gg["gn2_y"], atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(dx, gg["gn2_dx"], atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(dw, gg["gn2_dw"], atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("C,shape", [(64, (1, 64, 16, 128, 128)), (192, (2, 192, 3, 9, 11)),
                                     (384, (1, 384, 2, 8, 8)), (512, (2, 512, 1, 4, 4)),
                                     (256, (3, 256, 16, 32, 32))])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gn_silu_vs_oracle_shapes(C, shape, dtype):
    x = seeded(shape, 3) * 2 + 10.0  # |mean| >> std: exercises the Chan combine
    w = 1 + 0.1 * seeded((C,), 4)
    b = 0.1 * seeded((C,), 5)
    g = seeded(shape, 6)
    xr = x.clone().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = onn.group_norm(xr, wr, br, silu=True)
    yr.backward(g)
    if dtype == torch.bfloat16:  # compare to the oracle fed the same rounded input
        x = x.to(dtype).float()
    y, dx, dw, db = _run(x, w, b, True, dtype, g)
    tol_y = 1e-5 if dtype == torch.float32 else 1e-2
    assert rel_l2(y, yr) < tol_y * 3
    if dtype == torch.float32:
        assert rel_l2(dx, xr.grad) < 1e-4
        assert rel_l2(dw, wr.grad) < 1e-4
        assert rel_l2(db, br.grad) < 1e-4


@pytest.mark.parametrize("shape", [(1, 64, 16, 128, 128), (1, 256, 16, 32, 32), (3, 192, 5, 9, 11)])
def test_gn_bwd_bit_reproducible(shape):
    """the backward's per-channel sums are added in a fixed order (chunk
    partials -> ksplit slices -> ordered finalize; round 3 used float atomics across the
    slices), so dx / dgamma / dbeta are bit-identical run to run at config-2 sizes."""
    C = shape[1]
    x = seeded(shape, 30)
    w = 1 + 0.1 * seeded((C,), 31)
    b = 0.1 * seeded((C,), 32)
    g = seeded(shape, 33)
    r1 = _run(x, w, b, True, torch.bfloat16, g)
    r2 = _run(x, w, b, True, torch.bfloat16, g)
    for a, c in zip(r1, r2):
        assert torch.equal(a, c)


@pytest.mark.parametrize("silu", [True, False])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(1, 64, 4, 32, 32), (2, 192, 3, 9, 11)])
def test_gn_passthrough_adds_residual_gradient(shape, dtype, silu):
    """Round 6: group_norm_silu_pass returns (GN(x), x'); the gradient reaching x' (a residual
    branch) is added inside the GN backward (vd_groupnorm_silu_bwd_add) instead of by an
    autograd add.  Against GN alone + the residual gradient added in fp32: fp32 to rounding,
    bf16 to one rounding of the sum (the fused form rounds once, autograd's add twice)."""
    from vdiff import ops
    C = shape[1]
    x = seeded(shape, 40)
    w, b = 1 + 0.1 * seeded((C,), 41), 0.1 * seeded((C,), 42)
    g, gr = seeded(shape, 43), seeded(shape, 44)
    xd = ops.to_cl(x.to(dev, dtype)).requires_grad_(True)
    wd, bd = w.to(dev).requires_grad_(True), b.to(dev).requires_grad_(True)
    y, xs = ops.group_norm_silu_pass(xd, wd, bd, 32, 1e-5, silu)
    assert xs.data_ptr() == xd.data_ptr()
    torch.autograd.backward([y, xs], [ops.to_cl(g.to(dev, dtype)), ops.to_cl(gr.to(dev, dtype))])
    _, dx0, dw0, db0 = _run(x, w, b, silu, torch.float32 if dtype == torch.float32 else dtype, g)
    want = dx0 + gr.to(dtype).float()
    tol = 1e-6 if dtype == torch.float32 else 8e-3
    assert rel_l2(xd.grad.float().cpu(), want) < tol
    torch.testing.assert_close(wd.grad.cpu(), dw0)
    torch.testing.assert_close(bd.grad.cpu(), db0)
    # no gradient through the alias: plain GN backward
    xd2 = ops.to_cl(x.to(dev, dtype)).requires_grad_(True)
    y2, _ = ops.group_norm_silu_pass(xd2, wd.detach(), bd.detach(), 32, 1e-5, silu)
    y2.backward(ops.to_cl(g.to(dev, dtype)))
    assert torch.equal(xd2.grad.float().cpu(), dx0)


@pytest.mark.parametrize("shape", [(1, 64, 16, 128, 128), (1, 256, 16, 32, 32), (2, 192, 3, 9, 11)])
def test_gn_unroll_bit_identical(shape):
    """vd_groupnorm_set_unroll (rows whose loads each thread keeps in flight) changes only the
    load schedule: the sums are added in the same order, so y, dx, dgamma, dbeta are
    bit-identical for U = 1, 2, 4."""
    from vdiff import _lib
    C = shape[1]
    x = seeded(shape, 50)
    w, b = 1 + 0.1 * seeded((C,), 51), 0.1 * seeded((C,), 52)
    g = seeded(shape, 53)
    lib = _lib.lib()
    outs = []
    try:
        for u in (1, 2, 4):
            assert lib.vd_groupnorm_set_unroll(u) in (1, 2, 4)
            outs.append(_run(x, w, b, True, torch.bfloat16, g))
    finally:
        lib.vd_groupnorm_set_unroll(2)
    assert lib.vd_groupnorm_set_unroll(3) == -2
    for o in outs[1:]:
        for a, c in zip(outs[0], o):
            assert torch.equal(a, c)
