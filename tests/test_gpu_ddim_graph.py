"""DDIM sampling as a replayed HIP graph (vdiff.engine.DDIMGraph, the default of
engine.sample_ddim on a GPU) against the eager loop: the graph replays the same kernels on
the same operands, so the samples agree bit for bit, in bf16 and fp32, 4-D and 5-D."""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


def _model(dims, bf16):
    from vdiff.engine import reinit_nonzero
    from vdiff.unet_audio import UNetAudio
    torch.manual_seed(4321)
    m = UNetAudio(image_size=32, in_channels=3, model_channels=32, out_channels=3,
                  num_res_blocks=1, attention_resolutions=(2,), channel_mult=(1, 2),
                  audio_feature_dim=64, projected_audio_dim=32, dims=dims, use_bf16=bf16,
                  audio_encoder=False)
    reinit_nonzero(m, seed=4321)
    return m.to(dev).eval()


@pytest.mark.parametrize("dims,bf16", [(3, True), (3, False), (2, True)])
def test_ddim_graph_matches_eager(dims, bf16, monkeypatch):
    from vdiff.engine import sample_ddim
    from vdiff.schedulers import DDIMSampler, LinearNoiseSchedulerV2
    m = _model(dims, bf16)
    T = 4 if dims == 3 else 1
    shape = (1, 3, T, 32, 32) if dims == 3 else (1, 3, 32, 32)
    cond = torch.rand((1, 3, 32, 32), device=dev) * 2 - 1
    feats = torch.randn((T, 64), device=dev)
    sampler = DDIMSampler(LinearNoiseSchedulerV2(500, 0.00005, 0.015), steps=5)
    out, traj = {}, {}
    for mode in ("0", "1"):
        monkeypatch.setenv("VDIFF_DDIM_GRAPH", mode)
        g = torch.Generator(device=dev).manual_seed(9)
        seen = traj[mode] = []
        out[mode] = sample_ddim(m, sampler, cond, feats, shape, generator=g,
                                callback=lambda i, xt, x0: seen.append((xt, x0)))
    for a, b in zip(out["0"], out["1"]):
        assert torch.isfinite(a).all() and a.abs().max() > 0
        assert torch.equal(a, b)
    # a callback that keeps references sees every step's own values on both paths (the
    # graph path hands out copies of its static buffers, advisor r2)
    assert len(traj["0"]) == len(traj["1"]) == 5
    for (xa, x0a), (xb, x0b) in zip(traj["0"], traj["1"]):
        assert torch.equal(xa, xb) and torch.equal(x0a, x0b)
    assert not torch.equal(traj["1"][0][1], traj["1"][-1][1])


def test_ddim_graph_matches_eager_config2(monkeypatch):
    """the full-size sampling graph (BASELINE config 2: 128x128x16, joint
    attention, bf16, the bench's model -- the default sampling path and the bench's DDIM
    legs) against the eager loop over 3 DDIM steps: the same kernels on the same operands,
    so bit-equal (this size runs the asm D = 64 / 128 kernels and the D = 256 KV split with
    its in-capture workspaces, which the 32x32 tests above never reach)."""
    import argparse
    import bench
    from vdiff.engine import sample_ddim, synthetic_clip
    from vdiff import ops
    from vdiff.schedulers import DDIMSampler, LinearNoiseSchedulerV2
    ns = argparse.Namespace(size=128, frames=16, dtype="bf16", mode="joint", init="nonzero")
    m = bench.build_model(ns, torch.device(dev)).eval()
    clip = synthetic_clip(1, 16, 128, 500, dev, seed=5)
    sampler = DDIMSampler(LinearNoiseSchedulerV2(500, 0.00005, 0.015), steps=3)
    seen = {}
    with torch.no_grad(), ops.frozen_weights():
        feats = m.encode_audio(clip.audio)
        for mode in ("0", "1"):
            monkeypatch.setenv("VDIFF_DDIM_GRAPH", mode)
            g = torch.Generator(device=dev).manual_seed(9)
            seen[mode] = []
            sample_ddim(m, sampler, clip.cond, feats, tuple(clip.x0.shape), generator=g,
                        callback=lambda i, xt, x0, s=seen[mode]: s.append(xt.float()))
    assert len(seen["0"]) == len(seen["1"]) == 3
    for e, gr in zip(seen["0"], seen["1"]):
        assert torch.isfinite(e).all() and e.abs().max() > 0
        assert torch.equal(e, gr), float((gr - e).norm() / e.norm())


def _host_work_callback(seen):
    """test.py:205-207's callback does eager GPU work between replays (save_frame: clamp,
    scale, copy to the host); this one keeps clones and runs torch reductions and a device ->
    host copy after every replay, the trigger of the round-5 replay defect."""
    def cb(i, xt, x0):
        seen.append((xt.clone(), x0.clone()))
        s = (x0.float().clamp(-1, 1) * 0.5 + 0.5).mean() + xt.float().abs().sum()
        if i % 10 == 0:
            assert torch.isfinite(s.cpu())
    return cb


def test_ddim_graph_50_steps_with_host_work_matches_eager(monkeypatch):
    """one full 50-step graphed DDIM sample (the product default, the
    replay count of test.py's sampler) with eager GPU work between the replays equals the
    eager loop bit for bit at every step, and the captured step holds no memset node."""
    from vdiff import ops
    from vdiff.engine import DDIMGraph, sample_ddim
    from vdiff.schedulers import DDIMSampler, LinearNoiseSchedulerV2
    m = _model(3, True)
    shape = (1, 3, 4, 32, 32)
    cond = torch.rand((1, 3, 32, 32), device=dev) * 2 - 1
    feats = torch.randn((4, 64), device=dev)
    sampler = DDIMSampler(LinearNoiseSchedulerV2(500, 0.00005, 0.015), steps=50)
    seen = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("VDIFF_DDIM_GRAPH", mode)
        g = torch.Generator(device=dev).manual_seed(11)
        seen[mode] = []
        sample_ddim(m, sampler, cond, feats, shape, generator=g,
                    callback=_host_work_callback(seen[mode]))
    assert len(seen["0"]) == len(seen["1"]) == 50
    for i, ((xa, x0a), (xb, x0b)) in enumerate(zip(seen["0"], seen["1"])):
        assert torch.equal(xa, xb) and torch.equal(x0a, x0b), i
    assert torch.isfinite(seen["1"][-1][0]).all()
    with torch.no_grad(), ops.frozen_weights():
        gr = DDIMGraph(m, sampler, cond, feats, torch.randn(shape, device=dev))
        gr.capture()
        types = gr.node_types()
    assert types.get("memset", 0) == 0 and types.get("kernel", 0) > 20, types


@pytest.mark.parametrize("frames,size", [(16, 128), (25, 256)])
def test_ddim_graph_holds_no_memset_node_full_size(frames, size):
    """the default sampling graph at BASELINE config 2 (128x128x16) and
    config 4 (256x256x25, joint attention: the D = 256 key split with its in-capture
    workspaces) holds no memset node, and its first replays equal the eager steps."""
    import argparse
    import bench
    from vdiff import ops
    from vdiff.engine import DDIMGraph, synthetic_clip
    from vdiff.schedulers import DDIMSampler, LinearNoiseSchedulerV2
    ns = argparse.Namespace(size=128, frames=16, dtype="bf16", mode="joint", init="nonzero")
    m = bench.build_model(ns, torch.device(dev)).eval()
    clip = synthetic_clip(1, frames, size, 500, dev, seed=5)
    sampler = DDIMSampler(LinearNoiseSchedulerV2(500, 0.00005, 0.015), steps=50)
    with torch.no_grad(), ops.frozen_weights():
        feats = m.encode_audio(clip.audio)
        xt = torch.randn_like(clip.x0)
        gr = DDIMGraph(m, sampler, clip.cond, feats, xt)
        gr.capture()
        types = gr.node_types()
        assert types.get("memset", 0) == 0 and types.get("kernel", 0) > 100, types
        got, _ = gr.step(0)
        t = torch.full((1,), int(sampler.timesteps[0]), dtype=torch.int64, device=dev)
        want, _ = sampler.step(xt, m(xt, clip.cond, feats, t), 0)
        assert torch.equal(got, want.view_as(got)), float((got - want).norm() / want.norm())
