"""train.py / test.py drop-in entry points run end to end on the GPU (BASELINE config 1
shape: tiny UNet3D at 64x64x8, one DDPM train step; sampling with DDPM-V2 and DDIM)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import DROPIN

pytestmark = pytest.mark.gpu

TINY = ["--dims", "3", "--frames", "8", "--image-size", "64", "--model-channels", "32",
        "--channel-mult", "1", "2", "--num-res-blocks", "1", "--attention-resolutions", "2",
        "--random-audio-encoder"]


def _run(script, args, cwd):
    out = subprocess.run([sys.executable, os.path.join(DROPIN, script)] + args, cwd=cwd,
                         capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    return out.stdout


def test_train_entry_one_step(tmp_path):
    ck = str(tmp_path / "m.pth")
    out = _run("train.py", TINY + ["--batch-size", "1", "--epochs", "1", "--steps-per-epoch",
                                   "1", "--ckpt", ck], tmp_path)
    assert "Finished epoch 1" in out and os.path.exists(ck)
    # resume from the saved model/optimizer state for one more epoch
    out = _run("train.py", TINY + ["--batch-size", "1", "--epochs", "2", "--steps-per-epoch",
                                   "1", "--ckpt", ck, "--resume", ck + ".resume"], tmp_path)
    assert "Finished epoch 2" in out


@pytest.mark.parametrize("sampler,steps", [("ddim", "3"), ("ddpm-v2", "4")])
def test_sampling_entry(tmp_path, sampler, steps):
    out_dir = tmp_path / "imgs"
    _run("test.py", ["--dims", "3", "--frames", "4", "--image-size", "32", "--sampler", sampler,
                     "--steps", steps, "--save-every", "1", "--out-dir", str(out_dir),
                     "--random-init"], tmp_path)
    files = sorted(p for p in os.listdir(out_dir) if p.endswith(".npy"))
    assert files
    x0 = np.load(out_dir / files[0])
    assert x0.shape == (1, 3, 4, 32, 32) and np.isfinite(x0).all()


def test_train_entry_requires_audio_weights_or_flag(tmp_path):
    """Without pretrained wav2vec2 weights (none exist offline) train.py refuses to start
    unless --random-audio-encoder is given (the reference loads them, unet_audio.py:14)."""
    args = [a for a in TINY if a != "--random-audio-encoder"]
    out = subprocess.run([sys.executable, os.path.join(DROPIN, "train.py")] + args +
                         ["--batch-size", "1", "--epochs", "1", "--steps-per-epoch", "1",
                          "--ckpt", str(tmp_path / "m.pth")], cwd=tmp_path,
                         capture_output=True, text=True, timeout=900)
    assert out.returncode != 0


def test_reference_sampling_api(tmp_path):
    """test.py's reference API called as the reference script calls it (test.py:116, 152):
    load_model_and_scheduler(config) then sample_images(model, scheduler, img_cond,
    audio_cond, n_timesteps) -- here 3 DDPM-V2 steps on a 32x32 2-D model."""
    code = f"""
import os, sys, numpy as np, torch
sys.path.insert(0, {DROPIN!r})
os.chdir({str(tmp_path)!r})
import test
test.config["dataset_params"]["im_size"] = 32
model, scheduler = test.load_model_and_scheduler(test.config)
img_cond = torch.rand(1, 3, 32, 32, device=test.device) * 2 - 1
audio_cond = {{"input_values": torch.randn(1, 4000, device=test.device)}}
x0 = test.sample_images(model, scheduler, img_cond, audio_cond, n_timesteps=3)
assert x0.shape == (1, 3, 32, 32) and torch.isfinite(x0).all()
files = sorted(os.listdir("lipreading_generated_images"))
assert "x0_0.png" in files or "x0_0.npy" in files, files
print("OK", type(scheduler).__name__)
"""
    out = subprocess.run([sys.executable, "-c", code], cwd=tmp_path, capture_output=True,
                         text=True, timeout=900)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    assert "OK LinearNoiseSchedulerV2" in out.stdout


def test_sampling_entry_with_audio_cross_attention(tmp_path):
    """test.py --audio-attention: the wav2vec2 tokens (not pooled) reach the cross-attention
    branches of every attention block (build extension)."""
    out_dir = tmp_path / "imgs"
    _run("test.py", ["--dims", "3", "--frames", "2", "--image-size", "32", "--sampler", "ddim",
                     "--steps", "2", "--save-every", "1", "--out-dir", str(out_dir),
                     "--random-init", "--audio-attention"], tmp_path)
    files = sorted(p for p in os.listdir(out_dir) if p.endswith(".npy"))
    x0 = np.load(out_dir / files[0])
    assert x0.shape == (1, 3, 2, 32, 32) and np.isfinite(x0).all()
