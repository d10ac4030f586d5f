"""The oracle along a sampling trajectory (CPU): oracle.unet + oracle.schedulers.p_sample_v2
with the injected seeded noise reproduce tests/golden/trajectory.npz (the reference loop of
test.py:56-65 over the imported UNetModel / LinearNoiseSchedulerV2) -- pins the oracle the
GPU trajectory test's tolerances are reasoned against."""
import pytest
import torch

from conftest import golden
from oracle import schedulers as osch
from oracle.fixtures import FULL2D, TINY3D, rel_l2, seeded
from oracle.unet import (audio_conditioned_input, audio_param_shapes, build_plan, init_params,
                         param_shapes, unet_forward)


@pytest.mark.parametrize("case,dims,n_t,seed", [("tiny3d_500", 3, 500, 900),
                                                ("full2d_10", 2, 10, 940)])
def test_oracle_trajectory_matches_reference(case, dims, n_t, seed):
    cfg = TINY3D if dims == 3 else FULL2D
    plan = build_plan(**cfg)
    P = init_params(param_shapes(plan), 1234)
    if dims == 3:
        P.update(init_params(audio_param_shapes(64, 16, im_cond_output_ch=16), 77))
        cond, feat, proj = seeded((1, 3, 32, 32), 80, "uniform"), seeded((8, 64), 81), 16
        shape = (1, 3, 8, 64, 64)
    else:
        P.update(init_params(audio_param_shapes(768, 128), 77))
        cond, feat, proj = seeded((1, 3, 48, 48), 82, "uniform"), seeded((1, 768), 83), 128
        shape = (1, 3, 64, 64)
    tab = osch.linear_tables(500, 0.00005, 0.015)
    g = golden("trajectory.npz")
    xt = seeded(shape, seed)
    with torch.no_grad():
        for k, i in enumerate(reversed(range(n_t))):
            if k == 10:
                break
            t = torch.tensor([i])
            eps = unet_forward(P, plan, audio_conditioned_input(P, xt, cond, feat, proj), t)
            xt, x0 = osch.p_sample_v2(tab, xt, eps, t, seeded(shape, seed + 1 + k))
            if k + 1 in (1, 5, 10):
                assert rel_l2(xt, g[f"{case}_xt_{k + 1}"]) < 1e-5, (case, k)
                assert rel_l2(x0, g[f"{case}_x0_{k + 1}"]) < 1e-5, (case, k)
