"""Oracle restatement of the data path (TEST INFRASTRUCTURE ONLY -- never imported by the
product path): TalkingFaceFrameDataset.__getitem__ (reference video-generation/dataset.py:
78-139) and the frame index of preprocessing/extract_video_frames.py:21-39, 84-90.

Third-party pieces the reference calls, restated from their published algorithms (the
libraries themselves are absent here except where noted):
  * torchaudio.functional.highpass_biquad + lfilter(clamp=True) (torchaudio absent): the
    RBJ biquad high-pass, direct-form recursion, output clamped to [-1, 1]; pinned in the
    tests against scipy.signal.lfilter;
  * torchaudio.transforms.Resample (sinc_interp_hann, lowpass_filter_width 6, rolloff 0.99;
    torchaudio absent): restated from its kernel construction; pinned by known answers
    (identity at equal rates, constants stay constant away from the edges);
  * Wav2Vec2Processor's feature extractor (transformers, present): zero-mean unit-variance
    normalisation, pinned against transformers' own Wav2Vec2FeatureExtractor;
  * torchvision Resize on a PIL image = PIL's bilinear resample (PIL present): the oracle IS
    PIL (Image.resize), no restatement.
"""
from __future__ import annotations

import math

import numpy as np


def frame_items(total_frames: int, fps: float):
    """extract_video_frames.py:31-33: (i, i + step) pairs stepping at ~30 fps."""
    step = max(1, int(fps / 30))
    return [(i, i + step) for i in range(0, total_frames - step, step)]


def highpass_biquad(x: np.ndarray, sr: int, cutoff: float = 300.0, Q: float = 0.707):
    """torchaudio highpass_biquad -> lfilter(clamp=True) on each row of x [C, n] (float64
    arithmetic; torchaudio computes in the waveform dtype)."""
    w0 = 2 * math.pi * cutoff / sr
    alpha = math.sin(w0) / 2.0 / Q
    b = np.array([(1 + math.cos(w0)) / 2, -1 - math.cos(w0), (1 + math.cos(w0)) / 2])
    a = np.array([1 + alpha, -2 * math.cos(w0), 1 - alpha])
    b, a = b / a[0], a / a[0]
    y = np.zeros_like(x, dtype=np.float64)
    for c in range(x.shape[0]):
        x1 = x2 = y1 = y2 = 0.0
        for i, xi in enumerate(x[c].astype(np.float64)):
            yi = b[0] * xi + b[1] * x1 + b[2] * x2 - a[1] * y1 - a[2] * y2
            x2, x1, y2, y1 = x1, xi, y1, yi
            y[c, i] = yi
    return np.clip(y, -1.0, 1.0)


def sinc_resample(x: np.ndarray, orig: int, new: int, keep: int | None = None):
    """torchaudio.functional.resample (sinc_interp_hann, width 6, rolloff 0.99) of each row
    of x [C, n]; returns the first `keep` samples (default: all ceil(new * n / orig))."""
    g = math.gcd(orig, new)
    n = x.shape[-1]
    if orig == new:
        out = x.astype(np.float64)
        return out if keep is None else np.pad(out, ((0, 0), (0, max(0, keep - n))))[:, :keep]
    of, nf = orig // g, new // g
    base = min(of, nf) * 0.99
    width = math.ceil(6 * of / base)
    idx = np.arange(-width, width + of, dtype=np.float64)[None] / of
    t = np.arange(0, -nf, -1, dtype=np.float64)[:, None] / nf + idx
    t = np.clip(t * base, -6, 6)
    window = np.cos(t * math.pi / 6 / 2) ** 2
    t = t * math.pi
    with np.errstate(invalid="ignore", divide="ignore"):
        kern = np.where(t == 0, 1.0, np.sin(t) / t)
    kern = (kern * window * base / of).astype(np.float32).astype(np.float64)  # [nf, klen]
    target = math.ceil(nf * n / of)
    keep = target if keep is None else keep
    out = np.zeros((x.shape[0], keep))
    padded = np.pad(x.astype(np.float64), ((0, 0), (width, width + of)))
    for j in range(min(keep, target)):
        pos, ph = divmod(j, nf)
        out[:, j] = padded[:, pos * of: pos * of + kern.shape[1]] @ kern[ph]
    return out


def processor_normalize(x: np.ndarray):
    """Wav2Vec2FeatureExtractor.zero_mean_unit_var_norm on each row."""
    m = x.mean(-1, keepdims=True)
    v = x.var(-1, keepdims=True)
    return (x - m) / np.sqrt(v + 1e-7)


def audio_window(wave: np.ndarray, sr: int, fps: float, out_frame: int, buffer_frames=5,
                 target_len=4000, target_sr=16000, bug_compatible=True):
    """dataset.py:113-130 for one output frame; wave [C, n] -> input_values [C, target_len]."""
    fd = 1.0 / fps
    start_sec = max(0.0, (out_frame - buffer_frames) * fd)
    end_sec = out_frame * fd
    s0, s1 = int(sr * start_sec), int(sr * end_sec)
    seg = wave[:, s0:s1]
    seg = highpass_biquad(seg, sr)
    seg = (seg - seg.mean()) / seg.std(ddof=1)          # normalize_waveform (torch .std())
    orig = seg.shape[0] if bug_compatible else sr        # dataset.py:53 compares size(0)
    seg = sinc_resample(seg, orig, target_sr, keep=target_len)
    return processor_normalize(seg)


def frame_transform(frame_u8: np.ndarray, size: int = 128):
    """ToPILImage -> Resize((size, size)) -> ToTensor -> Normalize(0.5, 0.5) (train.py:70-75):
    [H, W, 3] uint8 -> [3, size, size] float32 in [-1, 1].  PIL does the resampling."""
    from PIL import Image
    im = Image.fromarray(frame_u8).resize((size, size), Image.BILINEAR)
    a = np.asarray(im, dtype=np.float32) / 255.0
    return ((a - 0.5) / 0.5).transpose(2, 0, 1)
