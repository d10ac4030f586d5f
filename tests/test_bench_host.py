"""Host-side logic of bench.py and the FLOP models (CPU): the roofline object's
arithmetic, the attention FLOP counts the roofline uses, and the JSON contract keys."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_attention_kernel_flops():
    from vdiff.flops import attention_kernel_flops
    n, d = 262144, 64
    # fwd 4 N^2 D (QK^T, PV); dQ 6 (S, dP, dQ); dK/dV 8 (S, dP, dV, dK)
    assert attention_kernel_flops("attn_fwd", n, d, 1) == pytest.approx(4 * n * n * d)
    assert attention_kernel_flops("attn_bwd_dq", n, d, 1) == pytest.approx(6 * n * n * d)
    assert attention_kernel_flops("attn_bwd_dkdv", n, d, 2) == pytest.approx(2 * 8 * n * n * d)


def test_attention_unit_flops_are_algorithmic():
    """backward = 2x forward (4 products), no credit for the recomputed S / dP."""
    from vdiff.flops import attention_kernel_flops, attention_unit_flops
    n, d = 262144, 64
    assert attention_unit_flops("fwd", n, d, 1) == pytest.approx(4 * n * n * d)
    assert attention_unit_flops("bwd", n, d, 1) == pytest.approx(8 * n * n * d)
    executed = (attention_kernel_flops("attn_bwd_dq", n, d, 1)
                + attention_kernel_flops("attn_bwd_dkdv", n, d, 1))
    assert executed / attention_unit_flops("bwd", n, d, 1) == pytest.approx(7 / 4)


def test_pick_roofline_takes_the_longest_unit():
    b = _bench()
    summary = {("attn_fwd", 64, 262144, 1): [15, 250.0],
               ("attn_bwd_dkdv", 64, 262144, 1): [15, 420.0],
               ("attn_bwd_dq", 64, 262144, 1): [15, 300.0],
               ("attn_bwd_dq", 128, 65536, 1): [15, 37.0]}
    roof, rows, units = b.pick_roofline(summary, "bf16")
    assert [r["kernel"] for r in rows] == ["attn_bwd_dkdv", "attn_bwd_dq", "attn_fwd",
                                           "attn_bwd_dq"]
    assert [u["unit"] for u in units] == ["bwd", "fwd"]  # the unpaired dQ is no unit
    f = 8 * 262144 ** 2 * 64  # algorithmic backward: 4 products
    t = (420.0 + 300.0) / 15 / 1e3
    assert roof["achieved"] == pytest.approx(f / t / 1e12, rel=1e-3)
    assert roof["frac"] == pytest.approx(f / t / 1e12 / 2500.0, rel=1e-3)
    assert roof["executed_frac"] == pytest.approx(roof["frac"] * 7 / 4, rel=1e-3)
    assert roof["peak"] == 2500.0 and roof["unit"] == "TFLOP/s" and roof["bound"] == "mfma"
    assert roof["traffic"] is None or roof["traffic"] > 0


def test_unet_forward_flops_match_survey():
    """103.95 TFLOP per 128x128x16 clip forward (joint attention)."""
    import torch
    from vdiff.flops import unet_forward_work
    from vdiff.nn import UNetModel
    with torch.device("meta"):
        m = UNetModel(image_size=128, in_channels=195, model_channels=64, out_channels=3,
                      num_res_blocks=2, attention_resolutions=(1, 2, 4), channel_mult=(1, 2, 4),
                      dims=3)
    w = unet_forward_work(m, (1, 195, 16, 128, 128))
    assert w.total / 1e12 == pytest.approx(103.95, abs=0.01)


def test_bench_cli_defaults():
    b = _bench()
    import sys
    argv = sys.argv
    try:
        sys.argv = ["bench.py"]
        a = b.parse()
    finally:
        sys.argv = argv
    assert (a.gpus, a.steps, a.warmup, a.frames, a.size, a.dtype) == (1, 3, 1, 16, 128, "bf16")
    assert a.vivit_batch == 16 and a.only == "all"
