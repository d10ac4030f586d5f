"""Data path on the GPU: the frame transform kernel against PIL (the resampler torchvision's
Resize hands PIL images to: bit-identical uint8, hence identical normalised values), the
TalkingFaceFrameDataset item against the oracle, the ClipBatcher's frame stacks, and
train.py reading a frame index (BASELINE config 1 shape)."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import DROPIN
from oracle import data as od

pytestmark = pytest.mark.gpu
dev = "cuda"


def _frames(n, H, W, seed):
    g = np.random.default_rng(seed)
    # smooth content plus noise: exercises rounding at every level
    yy, xx = np.meshgrid(np.linspace(0, 1, H), np.linspace(0, 1, W), indexing="ij")
    base = (np.stack([yy, xx, (yy + xx) / 2], -1) * 255)[None]
    return np.clip(base + g.integers(-40, 40, (n, H, W, 3)), 0, 255).astype(np.uint8)


@pytest.mark.parametrize("H,W", [(160, 160), (224, 224), (100, 181), (64, 64), (128, 128),
                                 (96, 200)])
def test_frame_transform_matches_pil_bit_for_bit(H, W):
    from vdiff import data as vd
    fr = _frames(3, H, W, H + W)
    got = vd.transform_frames(torch.from_numpy(fr).to(dev), 128).cpu().numpy()
    ref = np.stack([od.frame_transform(f, 128) for f in fr])
    assert got.shape == ref.shape == (3, 3, 128, 128)
    np.testing.assert_array_equal(got, ref)
    got16 = vd.transform_frames(torch.from_numpy(fr).to(dev), 128, dtype=torch.bfloat16)
    np.testing.assert_array_equal(got16.float().cpu().numpy(),
                                  torch.from_numpy(ref).bfloat16().float().numpy())


def _store(tmp_path, name, F=30, H=160, W=160, fps=30.0, sr=16000, seed=0):
    from vdiff import data as vd
    g = np.random.default_rng(seed)
    audio = (0.3 * np.sin(np.arange(int(sr * F / fps)) * 0.05) +
             0.05 * g.standard_normal(int(sr * F / fps))).astype(np.float32)[None]
    p = str(tmp_path / f"{name}.vdclip")
    vd.write_clip(p, _frames(F, H, W, seed), fps, audio, sr)
    return p


def test_dataset_item_matches_oracle(tmp_path):
    from vdiff import data as vd
    p = _store(tmp_path, "v0", seed=3)
    items = vd.build_frame_items([p])
    ds = vd.TalkingFaceFrameDataset(items, gpu_transform=True, device=dev)
    c = vd.ClipFile(p)
    for idx in (0, 7, len(items) - 1):
        inp, outp, aud = ds[idx]
        out_idx = min(items[idx].frame_end, len(c) - 1)
        np.testing.assert_array_equal(inp.cpu().numpy(), od.frame_transform(np.asarray(c.frames[0])))
        np.testing.assert_array_equal(outp.cpu().numpy(),
                                      od.frame_transform(np.asarray(c.frames[out_idx])))
        ref = od.audio_window(np.asarray(c.audio), c.sr, c.fps, out_idx)
        assert aud["input_values"].shape == (1, 4000)
        np.testing.assert_allclose(aud["input_values"].numpy(), ref, atol=2e-4)
    # a missing file: the reference prints and returns (None, None) (dataset.py:137-139)
    bad = vd.TalkingFaceFrameDataset([vd.FrameItem(str(tmp_path / "missing.vdclip"), 0, 1)])
    assert bad[0] == (None, None)


def test_clip_batcher_frame_stacks(tmp_path):
    from vdiff import data as vd
    paths = [_store(tmp_path, f"v{i}", F=24, seed=10 + i) for i in range(3)]
    items = vd.build_frame_items(paths)
    b = vd.ClipBatcher(items, batch=2, frames=4, num_timesteps=100, device=dev, size=64, seed=5)
    clip = b.next()
    assert clip.x0.shape == (2, 3, 4, 64, 64) and clip.cond.shape == (2, 3, 64, 64)
    assert clip.audio["input_values"].shape == (8, 4000)
    assert clip.eps.shape == clip.x0.shape and clip.t.shape == (2,)
    # replay the same picks on the host: same frames through PIL
    rng = np.random.default_rng(5)
    picks = rng.integers(0, len(items), size=2)
    for bi, i in enumerate(picks):
        it = items[i]
        c = vd.ClipFile(it.video_path)
        s = b._sample(it)
        np.testing.assert_array_equal(clip.cond[bi].cpu().numpy(),
                                      od.frame_transform(np.asarray(c.frames[0]), 64))
        for k, fi in enumerate(s.out_idx):
            np.testing.assert_array_equal(clip.x0[bi, :, k].cpu().numpy(),
                                          od.frame_transform(np.asarray(c.frames[fi]), 64))
    b.close()


def test_clip_batcher_prefetch_gives_the_same_batches(tmp_path):
    """The background host thread (prefetch > 0) draws and prepares batches in order: the
    batches equal the synchronous batcher's, frame for frame and window for window."""
    from vdiff import data as vd
    paths = [_store(tmp_path, f"v{i}", F=24, H=96 + 32 * (i % 2), W=96, seed=40 + i)
             for i in range(3)]
    items = vd.build_frame_items(paths)
    got = {}
    for pf in (0, 3):
        b = vd.ClipBatcher(items, batch=2, frames=3, num_timesteps=100, device=dev, size=32,
                           seed=11, prefetch=pf)
        got[pf] = [b.next() for _ in range(5)]
        b.close()
    for a, c in zip(got[0], got[3]):
        for k in ("x0", "cond", "eps", "t"):
            assert torch.equal(getattr(a, k), getattr(c, k)), k
        assert torch.equal(a.audio["input_values"], c.audio["input_values"])


def test_train_entry_reads_a_frame_index(tmp_path):
    from vdiff import data as vd
    paths = [_store(tmp_path, f"v{i}", F=20, H=96, W=96, seed=20 + i) for i in range(2)]
    idx = str(tmp_path / "index.jsonl")
    vd.save_frame_items(vd.build_frame_items(paths), idx)
    args = ["--dims", "3", "--frames", "4", "--image-size", "32", "--model-channels", "32",
            "--channel-mult", "1", "2", "--num-res-blocks", "1", "--attention-resolutions", "2",
            "--random-audio-encoder", "--batch-size", "1", "--epochs", "1",
            "--steps-per-epoch", "2", "--data", idx, "--ckpt", str(tmp_path / "m.pth")]
    out = subprocess.run([sys.executable, os.path.join(DROPIN, "train.py")] + args, cwd=tmp_path,
                         capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    assert "Finished epoch 1" in out.stdout
