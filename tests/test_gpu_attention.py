"""Flash attention (fwd + bwd) vs the oracle's materialised softmax attention and the
reference golden vectors.  Modes: joint (reference), spatial, temporal."""
import pytest
import torch

from oracle import nn as onn
from oracle.fixtures import rel_l2, seeded

from conftest import golden

pytestmark = pytest.mark.gpu
dev = "cuda"


def _check(B, C, heads, T, HW, mode, legacy, dtype, seed):
    from vdiff import ops
    N = T * HW
    qkv = seeded((B, 3 * C, N), seed)
    if dtype == torch.bfloat16:
        qkv = qkv.bfloat16().float()
    qr = qkv.clone().requires_grad_(True)
    ref = onn.qkv_attention(qr, heads, legacy=legacy, mode=mode, spatial=(T, HW, 1))
    g = seeded(ref.shape, seed + 1)
    ref.backward(g)
    qd = ops.to_cl(qkv.to(dev, dtype)).requires_grad_(True)
    out = ops.attention(qd, heads=heads, mode=mode, spatial=(T, HW, 1), legacy=legacy)
    out.backward(ops.to_cl(g.to(dev, dtype)))
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    e_out, e_grad = rel_l2(out, ref), rel_l2(qd.grad, qr.grad)
    assert e_out < tol, (e_out, e_grad)
    assert e_grad < 2 * tol, (e_out, e_grad)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("C", [32, 64, 128, 256])
def test_joint_head_dims(C, dtype):
    _check(2, C, 1, 3, 67, "joint", True, dtype, 10 + C)  # N = 201: ragged tiles


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("mode", ["spatial", "temporal"])
def test_spatial_temporal(mode, dtype):
    _check(2, 64, 1, 5, 130, mode, True, dtype, 20)


@pytest.mark.parametrize("legacy", [True, False])
def test_multi_head_orders(legacy):
    _check(2, 128, 2, 1, 300, "joint", legacy, torch.float32, 30)
    _check(1, 128, 4, 2, 64, "temporal", legacy, torch.float32, 31)


def test_single_token_and_long_sequence():
    _check(1, 64, 1, 1, 1, "joint", True, torch.float32, 40)
    _check(1, 64, 1, 1, 4096, "joint", True, torch.bfloat16, 41)


def test_scores_with_large_logits():
    """Large |q.k| forces the online-softmax rescale branch on many tiles."""
    from vdiff import ops
    B, C, N = 1, 64, 777
    qkv = seeded((B, 3 * C, N), 50) * 4.0
    qkv[:, :C, 500] *= 8  # one query row with a far larger max late in the sequence
    ref = onn.qkv_attention(qkv, 1)
    out = ops.attention(ops.to_cl(qkv.to(dev)), heads=1)
    assert rel_l2(out, ref) < 2e-5


CONFIGS = ["auto", "base", "nb2", "w8", "p8", "p4", "d8", "d8n", "d4", "pair", "p4n2", "role",
           "sp", "asm"]


@pytest.mark.parametrize("cfg", CONFIGS)
@pytest.mark.parametrize("C", [32, 64, 128, 256])
def test_bf16_kernel_shapes(cfg, C):
    """Every bf16 kernel shape (4/8 waves, 1/2 row blocks, software-pipelined ring) on a
    ragged sequence (N = 201: partial last tile and block) and a sequence shorter than
    one tile; shapes a head_dim does not support fall back inside the library."""
    from vdiff import ops
    with ops.attention_config(cfg):
        _check(2, C, 1, 3, 67, "joint", True, torch.bfloat16, 60 + C)
        _check(1, C, 1, 1, 21, "joint", True, torch.bfloat16, 61 + C)


@pytest.mark.parametrize("cfg", CONFIGS)
@pytest.mark.parametrize("C", [64, 128, 256])
def test_bf16_long_ragged_ring(cfg, C):
    """A sequence long enough for the stage-unrolled ring loops (>= 16 tiles) whose tile
    count is not a multiple of the 4 ring stages (N = 1157: 19 tiles, the last partial), so
    the padded tail tiles (zero rows) and the remainder loop both run, fwd and bwd."""
    from vdiff import ops
    with ops.attention_config(cfg):
        _check(1, C, 1, 1, 1157, "joint", True, torch.bfloat16, 70 + C)


@pytest.mark.parametrize("cfg", CONFIGS)
def test_bf16_lagged_max_rescale(cfg):
    """bf16 forward with logits that jump late in the sequence: exercises the lagged-max
    rare path (p reaching 2^16 forces a recompute against the true max)."""
    from vdiff import ops
    B, C, N = 1, 64, 1500
    qkv = seeded((B, 3 * C, N), 52) * 3.0
    qkv[:, C:2 * C, 1100] *= 12  # one key far above every earlier score, seen late
    qkv[:, :C, 700] *= 10        # and one query row with a large max of its own
    qkv = qkv.bfloat16().float()
    ref = onn.qkv_attention(qkv, 1)
    with ops.attention_config(cfg):
        out = ops.attention(ops.to_cl(qkv.to(dev, torch.bfloat16)), heads=1)
    assert torch.isfinite(out.float()).all()
    assert rel_l2(out, ref) < 2e-2


@pytest.mark.parametrize("C", [64, 128])
def test_bf16_lagged_max_rescale_default_shapes(C):
    """The default forward (deferred check) at both head dims it serves: a key far above
    every earlier score in a later tile, a query row with a large max, N not a multiple of
    the 64-key tile."""
    from vdiff import ops
    B, N = 1, 1337
    qkv = seeded((B, 3 * C, N), 53) * 3.0
    qkv[:, C:2 * C, 1100] *= 12
    qkv[:, :C, 700] *= 10
    qkv = qkv.bfloat16().float()
    ref = onn.qkv_attention(qkv, 1)
    out = ops.attention(ops.to_cl(qkv.to(dev, torch.bfloat16)), heads=1)
    assert torch.isfinite(out.float()).all()
    assert rel_l2(out, ref) < 2e-2


def test_config_hook_rejects_unknown():
    from vdiff import _lib, ops
    assert _lib.lib().vd_attention_set_config(13) == -2
    with pytest.raises(ValueError):
        ops.attention_config("fast")


def test_golden_regroupings():
    from vdiff import ops
    g = golden("blocks.npz")
    B, C, T, HW = 2, 64, 3, 36
    qkv = ops.to_cl(seeded((B, 3 * C, T * HW), 46).to(dev))
    for mode, key in (("joint", "st_joint"), ("spatial", "st_spatial"),
                      ("temporal", "st_temporal")):
        out = ops.attention(qkv, heads=1, mode=mode, spatial=(T, 6, 6))
        assert rel_l2(out, g[key]) < 2e-5, mode


@pytest.mark.parametrize("C,T,HW", [(256, 4, 256), (64, 1, 1000)])
def test_kv_split(C, T, HW):
    """KV-split forward / dQ (flash-decoding partials + merge): the 4-wave shape splits the keys
    when its query grid is too small for the chip (bf16, head_dim 256 by default)."""
    from vdiff import ops
    with ops.attention_config("base"):
        _check(1, C, 1, T, HW, "joint", True, torch.bfloat16, 80 + C)
