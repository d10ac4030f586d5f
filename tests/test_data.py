"""Data path: the .vdclip store, the frame index, the host audio-window
DSP in libvdiff (vd_audio_window, vd_resize_plan: host code, no GPU) against the oracle,
and the oracle's restatements against the third-party implementations present here
(scipy.signal.lfilter for torchaudio's biquad, transformers' Wav2Vec2FeatureExtractor for the
processor).  torchaudio is absent: its Resample is pinned by known answers only.  CPU."""
import math

import numpy as np
import pytest

from oracle import data as od
from vdiff import data as vd


def _wave(C, n, sr, seed=0):
    g = np.random.default_rng(seed)
    t = np.arange(n) / sr
    base = 0.3 * np.sin(2 * math.pi * 220 * t) + 0.2 * np.sin(2 * math.pi * 40 * t)
    return (base[None] + 0.05 * g.standard_normal((C, n))).astype(np.float32)


def test_biquad_matches_scipy_lfilter():
    from scipy.signal import lfilter
    x = _wave(2, 3000, 16000, 1) * 4  # large enough that the clamp bites
    sr, w0 = 16000, 2 * math.pi * 300 / 16000
    alpha = math.sin(w0) / 2 / 0.707
    b = [(1 + math.cos(w0)) / 2, -1 - math.cos(w0), (1 + math.cos(w0)) / 2]
    a = [1 + alpha, -2 * math.cos(w0), 1 - alpha]
    ref = np.clip(lfilter(b, a, x.astype(np.float64), axis=-1), -1, 1)
    np.testing.assert_allclose(od.highpass_biquad(x, sr), ref, atol=1e-12)


def test_resample_known_answers():
    x = _wave(1, 800, 16000, 2)
    np.testing.assert_array_equal(od.sinc_resample(x, 16000, 16000), x.astype(np.float64))
    c = np.full((1, 400), 0.7, np.float32)
    y = od.sinc_resample(c, 44100, 16000)
    assert y.shape == (1, math.ceil(160 * 400 / 441))
    assert np.abs(y[0, 20:-20] - 0.7).max() < 5e-3      # passband gain ~1 away from the edges
    # the reference's bug (orig_freq = channel count): 1 -> 16000, keep 4000
    yb = od.sinc_resample(x, 1, 16000, keep=4000)
    assert yb.shape == (1, 4000) and np.isfinite(yb).all()


def test_processor_normalisation_matches_transformers():
    from transformers import Wav2Vec2FeatureExtractor
    fe = Wav2Vec2FeatureExtractor(feature_size=1, sampling_rate=16000, padding_value=0.0,
                                  do_normalize=True, return_attention_mask=False)
    x = _wave(1, 4000, 16000, 3)[0] * 3 + 0.2
    ref = fe(x, sampling_rate=16000, return_tensors="np")["input_values"][0]
    np.testing.assert_allclose(od.processor_normalize(x[None].astype(np.float64))[0], ref,
                               rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("C,sr,bug", [(1, 16000, True), (1, 16000, False), (2, 16000, True),
                                      (1, 44100, False), (1, 22050, True)])
def test_audio_window_abi_matches_oracle(C, sr, bug):
    fps = 25.0
    wave = _wave(C, sr * 2, sr, 4)
    for out_frame in (0, 3, 17, 49):
        got = vd.audio_window(wave, sr, fps, out_frame, bug_compatible=bug)
        assert got.shape == (C, 4000)
        if out_frame == 0:  # empty window: the reference's normalisation of nothing -> zeros
            assert np.allclose(got, 0)
            continue
        ref = od.audio_window(wave, sr, fps, out_frame, bug_compatible=bug)
        # fp32 filter / kernel arithmetic (torchaudio's dtype) against the float64 oracle:
        # measured max |diff| 3e-6 .. 6e-5 on unit-variance outputs
        np.testing.assert_allclose(got, ref, rtol=0, atol=2e-4)


def test_resize_plan_coefficients():
    from vdiff import _lib
    for n_in, n_out in ((160, 128), (224, 128), (64, 128), (128, 128), (181, 128)):
        cap = 2 * -(-n_in // n_out) + 1
        b = np.zeros((n_out, 2), np.int32)
        c = np.zeros((n_out, cap), np.int32)
        _lib.call("vd_resize_plan", n_in, n_out, b.ctypes.data, c.ctypes.data, cap)
        s = c.sum(1)
        assert np.abs(s - (1 << 22)).max() <= cap  # normalised weights, 22-bit fixed point
        assert (b[:, 0] >= 0).all() and (b.sum(1) <= n_in).all()


def test_clip_store_and_frame_index(tmp_path):
    frames = np.random.default_rng(5).integers(0, 256, (40, 20, 24, 3), dtype=np.uint8)
    audio = _wave(1, 16000, 16000, 6)
    p = str(tmp_path / "a.vdclip")
    vd.write_clip(p, frames, 60.0, audio, 16000)
    c = vd.ClipFile(p)
    assert len(c) == 40 and c.fps == 60.0 and c.sr == 16000
    np.testing.assert_array_equal(np.asarray(c.frames), frames)
    np.testing.assert_array_equal(np.asarray(c.audio), audio)
    items = vd.build_frame_items([p])
    ref = od.frame_items(40, 60.0)  # step = 2 at 60 fps
    assert [(i.frame_start, i.frame_end) for i in items] == ref
    idx = str(tmp_path / "index.jsonl")
    vd.save_frame_items(items, idx)
    back = vd.load_frame_items(idx)
    assert [(i.video_path, i.frame_start, i.frame_end) for i in back] == \
        [(i.video_path, i.frame_start, i.frame_end) for i in items]
    # an unreadable file yields no items, as process_video's except branch
    bad = tmp_path / "bad.vdclip"
    bad.write_bytes(b"nope" * 20)
    assert vd.build_frame_items([str(bad)]) == []


def test_dataset_returns_raw_frames_without_transforms(tmp_path):
    """frame_transforms=None returns the raw uint8 frames, as the reference does (dataset.py:
    105-107), with no GPU call (usable from DataLoader workers); a host transform is applied
    per frame; data errors give (None, None) (dataset.py:137-139).  CPU."""
    frames = np.random.default_rng(8).integers(0, 256, (12, 20, 24, 3), dtype=np.uint8)
    p = str(tmp_path / "r.vdclip")
    vd.write_clip(p, frames, 30.0, _wave(1, 8000, 16000, 9), 16000)
    items = vd.build_frame_items([p])
    ds = vd.TalkingFaceFrameDataset(items)
    inp, outp, aud = ds[3]
    out_idx = min(items[3].frame_end, 11)
    assert inp.dtype == np.uint8 and inp.shape == (20, 24, 3)
    np.testing.assert_array_equal(inp, frames[0])
    np.testing.assert_array_equal(outp, frames[out_idx])
    assert tuple(aud["input_values"].shape) == (1, 4000)
    ds2 = vd.TalkingFaceFrameDataset(items, frame_transforms=lambda f: f[::2, ::2].copy())
    np.testing.assert_array_equal(ds2[3][1], frames[out_idx][::2, ::2])
    assert vd.TalkingFaceFrameDataset([vd.FrameItem(str(tmp_path / "no.vdclip"), 0, 1)])[0] \
        == (None, None)


def test_device_error_markers():
    """Advisor r03: only real HIP / CUDA / libvdiff failures propagate out of a dataset item;
    an ordinary data error whose message merely contains "hip" / "cuda" (a path such as
    /data/ship/clip.vdclip) is a per-item error (None, None) as in the reference."""
    from vdiff.data import _device_error
    assert _device_error(RuntimeError("HIP error: invalid device function"))
    assert _device_error(RuntimeError("CUDA error: out of memory"))
    assert _device_error(RuntimeError("libvdiff vd_frames_resize_normalize failed (code 3): x"))
    assert not _device_error(RuntimeError("cannot open /data/ship/clip_0001.vdclip"))
    assert not _device_error(RuntimeError("bad header in /mnt/barracuda/x.vdclip"))
    assert not _device_error(ValueError("HIP error"))
