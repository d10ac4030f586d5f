"""Implicit-GEMM conv kernels (fwd, bwd-data, bwd-weight) vs the oracle (torch CPU conv)."""
import pytest
import torch

from oracle import nn as onn
from oracle.fixtures import rel_l2, seeded

pytestmark = pytest.mark.gpu
dev = "cuda"

CASES = [
    # (x shape, Co, kernel, stride, padding)
    ((2, 64, 3, 9, 11), 64, 3, 1, 1),
    ((1, 195, 2, 8, 8), 64, 3, 1, 1),          # unpadded input channels (UNetAudio concat)
    ((2, 64, 2, 6, 7), 3, 3, 1, 1),            # model out conv: Co = 3
    ((1, 64, 2, 9, 9), 64, 3, (1, 2, 2), 1),   # Downsample
    ((2, 64, 2, 5, 5), 128, 1, 1, 0),          # ResBlock skip
    ((1, 384, 2, 4, 4), 256, 1, 1, 0),
    ((1, 512, 2, 4, 6), 256, 3, 1, 1),         # N > 128: two column tiles
    ((2, 64, 200), 192, 1, 1, 0),              # AttentionBlock qkv (Conv1d)
    ((2, 64, 10, 10), 64, 3, 1, 1),            # dims = 2
    ((1, 32, 4, 16, 16), 32, 3, 1, 1),
    ((1, 64, 2, 16, 24), 64, 3, 1, 1),         # bf16 tap-outer kernel: 256 x 64 tiles, ragged M
    ((1, 128, 3, 12, 12), 256, 3, 1, 1),       # 64 x 128 tiles (few workgroups)
    ((1, 128, 4, 128, 128), 128, 1, 1, 0),     # 128 x 128 tiles
    ((1, 128, 3, 10, 10), 128, 3, (1, 2, 2), 1),  # strided: transposed gather with stride 2
    ((2, 64, 3, 4, 32), 64, 3, 1, 1),          # bf16 kw-strip wgrad: 2 rows / step, t and b carry
    ((1, 64, 2, 3, 64), 128, 3, 1, 1),         # kw-strip wgrad: one 64-pixel row / step
    ((1, 96, 2, 5, 7), 48, 1, 1, 0),           # streaming 1x1: K = 96 (odd K step count)
    ((1, 256, 2, 6, 6), 768, 1, 1, 0),         # streaming 1x1: weight in 12 LDS slices
    ((1, 64, 1, 3, 7), 40, 1, 1, 0),           # 1x1 with N % 16 != 0: igemm fallback
    ((2, 96, 3, 5, 32), 80, 3, 1, 1),          # halo tile: 2 channel steps, partial t / h, ragged N
    ((1, 64, 2, 4, 16), 64, 3, 1, 1),          # halo tile: exact fit
    ((2, 96, 3, 5, 64), 80, 3, 1, 1),          # 64-pixel rows: wgrad planes, 2 ci tiles, ragged Co
    ((1, 64, 2, 2, 128), 64, 3, 1, 1),         # two 64-pixel steps per row
]


def _weights(Ci, Co, k, nd, seed):
    ks = (k,) * nd if isinstance(k, int) else k
    w = seeded((Co, Ci) + ks, seed) / (Ci * (k ** nd if isinstance(k, int) else 1)) ** 0.5
    b = 0.1 * seeded((Co,), seed + 1)
    return w, b


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_conv_fwd_bwd_vs_oracle(case, dtype):
    _conv_vs_oracle(case, dtype)


# every 3x3x3 stride-1 case that fits the halo tile (W % 16 == 0), on both kernels whatever
# the default selection picks for it
HALO_CASES = [i for i, c in enumerate(CASES)
              if len(c[0]) == 5 and c[2] == 3 and c[3] == 1 and c[4] == 1 and c[0][-1] % 16 == 0]


@pytest.mark.parametrize("mode", [0, 1, 3, 5])
@pytest.mark.parametrize("case", HALO_CASES)
def test_conv_halo_modes(case, mode):
    from vdiff import ops
    with ops.conv_halo(mode):
        _conv_vs_oracle(case, torch.bfloat16)


def test_conv_halo_hook_rejects_unknown():
    from vdiff import _lib, ops
    assert _lib.lib().vd_conv_set_halo(6) == -2
    with pytest.raises(ValueError):
        ops.conv_halo(7)


# (Ci, Co, T, H = W): the train step's halo shapes at both channel steps, the one that showed a
# nondeterministic result while the ring's stage reads could still be in flight across the
# per-tap barrier (round 6: 192 -> 128 at 64x64, 64-channel steps), and ragged tiles
DETERMINISM = [(64, 64, 16, 128), (192, 128, 16, 64), (256, 256, 16, 32), (200, 64, 4, 128),
               (96, 80, 5, 32)]


@pytest.mark.parametrize("mode", [2, 3, 5])
@pytest.mark.parametrize("shape", DETERMINISM)
def test_halo_conv_is_deterministic(shape, mode):
    """Bit-identical outputs over repeated launches (fwd and bwd-data) at full train-step sizes:
    every LDS read of a ring stage or halo returns before a barrier lets another wave's DMA refill
    it (vm_lgk_wait_barrier), so no launch may differ from another."""
    from vdiff import _lib, ops
    Ci, Co, T, H = shape
    g = torch.Generator(device=dev).manual_seed(Ci + Co + H)
    x = (torch.rand(1, T, H, H, Ci, generator=g, device=dev) * 2 - 1).bfloat16()
    dy = (torch.rand(1, T, H, H, Co, generator=g, device=dev) * 2 - 1).bfloat16()
    w = torch.randn(Co, Ci, 3, 3, 3, generator=g, device=dev) / (27 * Ci) ** 0.5
    wf = ops._pack_weight_now(w, Co, Ci, 27, Ci, Co, False, torch.bfloat16)
    wb = ops._pack_weight_now(w, Co, Ci, 27, Ci, Co, True, torch.bfloat16)
    d = ops._desc(1, [T, H, H], Ci, [T, H, H], Co, [3, 3, 3], [1, 1, 1], [1, 1, 1],
                  ops._DT[torch.bfloat16])
    st = ops._stream(x)
    for name, src, wt, shp in (("vd_conv3d_fwd", x, wf, Co), ("vd_conv3d_bwd_data", dy, wb, Ci)):
        with ops.conv_halo(mode):
            outs = []
            for _ in range(12):
                o = torch.empty(1, T, H, H, shp, dtype=torch.bfloat16, device=dev)
                if name == "vd_conv3d_fwd":
                    _lib.call(name, d, src.data_ptr(), wt.data_ptr(), None, None, None, o.data_ptr(), st)
                else:
                    _lib.call(name, d, src.data_ptr(), wt.data_ptr(), o.data_ptr(), st)
                outs.append(o)
            torch.cuda.synchronize()
            bad = [i for i, o in enumerate(outs) if not torch.equal(o, outs[0])]
            assert not bad, (name, shape, bad)


def _conv_vs_oracle(case, dtype):
    from vdiff import ops
    shape, Co, k, stride, pad = CASES[case]
    nd = len(shape) - 2
    Ci = shape[1]
    x = seeded(shape, 100 + case)
    w, b = _weights(Ci, Co, k, nd, 200 + case)
    if dtype == torch.bfloat16:  # oracle sees the same rounded operands
        x = x.bfloat16().float()
        w = w.bfloat16().float()
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    yr = onn.conv(xr, wr, br, stride=stride, padding=pad)
    g = seeded(yr.shape, 300 + case)
    yr.backward(g)

    xd = ops.to_cl(x.to(dev, dtype)).requires_grad_(True)
    wd = w.to(dev).requires_grad_(True)
    bd = b.to(dev).requires_grad_(True)
    y = ops.conv(xd, wd, bd, stride=stride, padding=pad)
    assert list(y.shape) == list(yr.shape)
    assert ops.is_cl(y)
    y.backward(ops.to_cl(g.to(dev, dtype)))
    tol = 2e-6 if dtype == torch.float32 else 1e-2
    assert rel_l2(y, yr) < tol, rel_l2(y, yr)
    assert rel_l2(xd.grad, xr.grad) < tol * 2, rel_l2(xd.grad, xr.grad)
    assert rel_l2(wd.grad, wr.grad) < tol * 2, rel_l2(wd.grad, wr.grad)
    assert rel_l2(bd.grad, br.grad) < (1e-5 if dtype == torch.float32 else 1e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("spatial", [(2, 7, 9), (3, 5, 16)])  # gathered tiles / halo tiles
def test_conv_fused_epilogue(dtype, spatial):
    """y = conv(x) + bias + chan_add[b, co] + residual (the ResBlock emb-add and skip-add)."""
    from vdiff import ops
    x = seeded((2, 64) + spatial, 1)
    w, b = _weights(64, 128, 3, 3, 2)
    ca = seeded((2, 128), 4)
    res = seeded((2, 128) + spatial, 5)
    if dtype == torch.bfloat16:
        x, w, res = x.bfloat16().float(), w.bfloat16().float(), res.bfloat16().float()
    leaves = [t.clone().requires_grad_(True) for t in (x, w, b, ca, res)]
    yr = onn.conv(leaves[0], leaves[1], leaves[2], padding=1) + leaves[3][:, :, None, None, None] \
        + leaves[4]
    g = seeded(yr.shape, 6)
    yr.backward(g)
    dl = [x.to(dev, dtype), w.to(dev), b.to(dev), ca.to(dev), res.to(dev, dtype)]
    dl[0] = ops.to_cl(dl[0])
    dl[4] = ops.to_cl(dl[4])
    dl = [t.requires_grad_(True) for t in dl]
    y = ops.conv(dl[0], dl[1], dl[2], padding=1, chan_add=dl[3], residual=dl[4])
    y.backward(ops.to_cl(g.to(dev, dtype)))
    tol = 2e-6 if dtype == torch.float32 else 1e-2
    assert rel_l2(y, yr) < tol
    for a, r in zip(dl, leaves):
        assert rel_l2(a.grad, r.grad) < 2 * tol + 1e-5


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_conv1x1_fused_epilogue(dtype):
    """The streaming 1x1 kernel's fused store: bias + chan_add[b, co] + residual, over a
    ragged pixel count (B = 2, 5 x 7 x 3 = 105 pixels per batch, not a multiple of 16)."""
    from vdiff import ops
    x = seeded((2, 64, 3, 5, 7), 11)
    w, b = _weights(64, 192, 1, 3, 12)
    ca = seeded((2, 192), 14)
    res = seeded((2, 192, 3, 5, 7), 15)
    if dtype == torch.bfloat16:
        x, w, res = x.bfloat16().float(), w.bfloat16().float(), res.bfloat16().float()
    leaves = [t.clone().requires_grad_(True) for t in (x, w, b, ca, res)]
    yr = onn.conv(leaves[0], leaves[1], leaves[2]) + leaves[3][:, :, None, None, None] + leaves[4]
    g = seeded(yr.shape, 16)
    yr.backward(g)
    dl = [x.to(dev, dtype), w.to(dev), b.to(dev), ca.to(dev), res.to(dev, dtype)]
    dl[0] = ops.to_cl(dl[0])
    dl[4] = ops.to_cl(dl[4])
    dl = [t.requires_grad_(True) for t in dl]
    y = ops.conv(dl[0], dl[1], dl[2], chan_add=dl[3], residual=dl[4])
    y.backward(ops.to_cl(g.to(dev, dtype)))
    tol = 2e-6 if dtype == torch.float32 else 1e-2
    assert rel_l2(y, yr) < tol
    for a, r in zip(dl, leaves):
        assert rel_l2(a.grad, r.grad) < 2 * tol + 1e-5


def _wgrad(x, w, dy, stride, pad, atomic):
    from vdiff import ops
    old = ops._WGRAD_ATOMIC
    ops._WGRAD_ATOMIC = atomic
    try:
        xd = x.detach().requires_grad_(False)
        wd = w.detach().clone().requires_grad_(True)
        y = ops.conv(xd, wd, None, stride=stride, padding=pad)
        y.backward(dy)
        return wd.grad
    finally:
        ops._WGRAD_ATOMIC = old


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_conv_wgrad_fixed_order(case, dtype):
    """the default weight gradient (per-split partials + one ordered pass,
    vd_conv3d_bwd_weight_det) is bit-identical run to run and equals round 3's atomic split-K
    kernel up to fp32 summation order (both are checked against the oracle above)."""
    from vdiff import ops
    shape, Co, k, stride, pad = CASES[case]
    nd = len(shape) - 2
    x = ops.to_cl(seeded(shape, 100 + case).to(dev, dtype))
    w, _ = _weights(shape[1], Co, k, nd, 200 + case)
    w = w.to(dev)
    y = ops.conv(x, w, None, stride=stride, padding=pad)
    dy = ops.to_cl(seeded(tuple(y.shape), 300 + case).to(dev, dtype))
    a = _wgrad(x, w, dy, stride, pad, False)
    b = _wgrad(x, w, dy, stride, pad, False)
    c = _wgrad(x, w, dy, stride, pad, True)
    assert torch.equal(a, b)
    assert rel_l2(a, c) < 1e-6, rel_l2(a, c)


@pytest.mark.parametrize("shape,Co,k", [((1, 64, 16, 128, 128), 64, 3),
                                       ((1, 256, 16, 32, 32), 256, 3),
                                       ((1, 64, 16, 128, 128), 192, 1)])
def test_conv_wgrad_fixed_order_config2(shape, Co, k):
    """Config-2 weight-gradient shapes, where the split-K has 8-256 pixel splits (the atomic
    kernel's sums then depend on arrival order): two fixed-order runs are bit-identical, and
    they agree with the atomic kernel and with a torch fp32 conv weight gradient of the same
    bf16 operands."""
    from vdiff import ops
    x = ops.to_cl(seeded(shape, 7).to(dev, torch.bfloat16))
    w = (seeded((Co, shape[1]) + (k,) * 3, 8) / (shape[1] * k ** 3) ** 0.5).to(dev)
    pad = k // 2
    y = ops.conv(x, w, None, padding=pad)
    dy = ops.to_cl(seeded(tuple(y.shape), 9).to(dev, torch.bfloat16))
    a = _wgrad(x, w, dy, 1, pad, False)
    b = _wgrad(x, w, dy, 1, pad, False)
    c = _wgrad(x, w, dy, 1, pad, True)
    assert torch.equal(a, b)
    assert rel_l2(a, c) < 1e-5, rel_l2(a, c)
    ref = torch.nn.grad.conv3d_weight(x.float().cpu().contiguous(), w.shape,
                                      dy.float().cpu().contiguous(), padding=pad)
    assert rel_l2(a, ref) < 1e-4, rel_l2(a, ref)


@pytest.mark.parametrize("shape,Co,k", [((1, 128, 16, 64, 64), 128, 3),    # 128-wide kw-strip tiles
                                       ((1, 384, 16, 64, 64), 128, 3),
                                       ((1, 512, 16, 32, 32), 256, 3),
                                       ((1, 128, 16, 32, 32), 256, 3),    # 64-wide (grid < a round)
                                       ((2, 128, 8, 64, 64), 128, 3),     # two clips
                                       ((1, 64, 16, 128, 128), 3, 3),     # the 64->3 output conv
                                       ((1, 256, 1, 128, 128), 768, 1),   # qkv 1x1, 64-wide tiles
                                       ((1, 200, 16, 64, 64), 64, 3)])    # padded Ci
def test_conv_wgrad_round4_split_rule(shape, Co, k):
    """The round-4 weight-gradient launch choices (occupancy-round pixel splits, 128-wide
    kw-strip tiles where their grid fills the chip, 64-wide 1x1 tiles): bit-identical run to
    run and within fp32 summation order of the fp32 parity-mode weight gradient
    (conv_wgrad_kernel<float>, exact-fp32 MFMA, itself checked against the oracle and torch
    above) of the same bf16 values."""
    from vdiff import ops
    x = ops.to_cl(seeded(shape, 17).to(dev, torch.bfloat16))
    w = (seeded((Co, shape[1]) + (k,) * 3, 18) / (shape[1] * k ** 3) ** 0.5).to(dev)
    pad = k // 2
    y = ops.conv(x, w, None, padding=pad)
    dy = ops.to_cl(seeded(tuple(y.shape), 19).to(dev, torch.bfloat16))
    a = _wgrad(x, w, dy, 1, pad, False)
    b = _wgrad(x, w, dy, 1, pad, False)
    assert torch.equal(a, b)
    ref = _wgrad(ops.to_cl(x.float()), w, ops.to_cl(dy.float()), 1, pad, False)
    assert rel_l2(a, ref) < 1e-5, rel_l2(a, ref)


@pytest.mark.parametrize("shape,Co,k", [((1, 64, 16, 128, 128), 64, 3),   # one 64-px row / step
                                       ((1, 256, 16, 32, 32), 256, 3),    # two rows / step
                                       ((2, 32, 4, 16, 16), 32, 3),       # four rows, two clips
                                       ((1, 64, 3, 5, 32), 64, 3),        # H % rows != 0: round 5
                                       ((1, 2 * 64, 4, 8, 128), 128, 3),  # two steps per row
                                       ((1, 64, 16, 64, 64), 192, 1),     # 1x1
                                       ((1, 96, 2, 5, 7), 48, 1)])        # 1x1, short last step
def test_wgrad_strip_equals_round5_kernel(shape, Co, k):
    """Round 6: the stage-unrolled weight-gradient kernel (vd_conv_set_wgrad(1), the default)
    runs the round-5 kernel's tiles, DMA pieces and summation order, so the two are
    bit-identical (tools/wgrad3_bench.py checks the same on every shape of the step)."""
    from vdiff import _lib, ops
    x = ops.to_cl(seeded(shape, 27).to(dev, torch.bfloat16))
    w = (seeded((Co, shape[1]) + (k,) * 3, 28) / (shape[1] * k ** 3) ** 0.5).to(dev)
    pad = k // 2
    y = ops.conv(x, w, None, padding=pad)
    dy = ops.to_cl(seeded(tuple(y.shape), 29).to(dev, torch.bfloat16))
    lib = _lib.lib()
    prev = lib.vd_conv_set_wgrad(0)
    try:
        a = _wgrad(x, w, dy, 1, pad, False)
        lib.vd_conv_set_wgrad(1)
        b = _wgrad(x, w, dy, 1, pad, False)
    finally:
        lib.vd_conv_set_wgrad(prev)
    assert torch.equal(a, b)
    assert lib.vd_conv_set_wgrad(3) == -2
