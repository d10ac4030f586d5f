"""Data path: the reference's TalkingFaceFrameDataset (video-generation/dataset.py:43-139) and
frame index (preprocessing/extract_video_frames.py:21-111) on this build.

The reference decodes mp4 files with decord and torchaudio at every __getitem__; neither
exists in this image, so clips are stored decoded, once, in a flat binary format that the
loader memory-maps (no decode, no pickle):

  <name>.vdclip = 64-byte header (magic b"VDCLIP01", frames, height, width, channels = 3,
                  fps f64, audio sample rate, audio channels, audio samples)
                  + frames uint8 [F][H][W][3] + audio fp32 [C][S]

A frame index is JSON lines {"video_path", "frame_start", "frame_end"} (the reference pickles
FrameItem objects; pickles are never loaded here).  Per item the reference takes frame 0 as
the conditioning image, frame min(frame_end, F - 1) as the target, and the audio of the 5
frames before the target (dataset.py:98-130).  The frame transform (PIL bilinear resize +
normalise) runs on the GPU (vd_frames_resize_normalize, bit-identical to PIL's uint8
resample); the audio window DSP runs on the host (vd_audio_window).
"""
from __future__ import annotations

import json
import os
import struct
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib

MAGIC = b"VDCLIP01"
_HDR = struct.Struct("<8siiiidiiq")  # 48 bytes, padded to 64
HEADER_BYTES = 64


def write_clip(path: str, frames: np.ndarray, fps: float, audio: np.ndarray, sr: int) -> None:
    """Store one decoded video: frames uint8 [F, H, W, 3], audio fp32 [C, S] at `sr` Hz."""
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    audio = np.ascontiguousarray(np.atleast_2d(audio), dtype=np.float32)
    if frames.ndim != 4 or frames.shape[3] != 3:
        raise ValueError(f"frames must be [F, H, W, 3] uint8, got {frames.shape}")
    F, H, W, _ = frames.shape
    hdr = _HDR.pack(MAGIC, F, H, W, 3, float(fps), int(sr), audio.shape[0], audio.shape[1])
    with open(path, "wb") as f:
        f.write(hdr.ljust(HEADER_BYTES, b"\0"))
        f.write(frames.tobytes())
        f.write(audio.tobytes())


class ClipFile:
    """Memory-mapped .vdclip: .frames uint8 [F, H, W, 3], .audio fp32 [C, S], .fps, .sr."""

    def __init__(self, path: str):
        with open(path, "rb") as f:
            raw = f.read(HEADER_BYTES)
        magic, F, H, W, C3, fps, sr, ac, an = _HDR.unpack(raw[:_HDR.size])
        if magic != MAGIC or C3 != 3:
            raise ValueError(f"{path}: not a VDCLIP01 file")
        self.path, self.fps, self.sr = path, fps, sr
        self.frames = np.memmap(path, np.uint8, "r", HEADER_BYTES, (F, H, W, 3))
        off = HEADER_BYTES + F * H * W * 3
        self.audio = np.memmap(path, np.float32, "r", off, (ac, an))

    def __len__(self):
        return self.frames.shape[0]


_open_cache: dict = {}


def open_clip(path: str) -> ClipFile:
    c = _open_cache.get(path)
    if c is None:
        if len(_open_cache) > 256:
            _open_cache.clear()
        c = _open_cache[path] = ClipFile(path)
    return c


class FrameItem:
    """dataset.py:43-47."""

    def __init__(self, video_path, frame_start, frame_end):
        self.video_path = video_path
        self.frame_start = frame_start
        self.frame_end = frame_end

    def __repr__(self):
        return f"FrameItem({self.video_path!r}, {self.frame_start}, {self.frame_end})"


def process_video(video_path: str):
    """extract_video_frames.py:21-39: (path, [(i, i + step)]) with step = max(1, int(fps/30));
    an unreadable file yields no items (the reference prints and returns [])."""
    try:
        c = open_clip(video_path)
    except (OSError, ValueError) as e:
        print(f"Error processing video {video_path}: {e}")
        return video_path, []
    if c.fps == 0:
        print(f"Error processing video {video_path}: FPS is zero")
        return video_path, []
    step = max(1, int(c.fps / 30))
    return video_path, [(i, i + step) for i in range(0, len(c) - step, step)]


def build_frame_items(paths) -> list:
    """extract_video_frames.py main() + extract_instances (:41-49, 84-90)."""
    items = []
    for p in paths:
        _, idx = process_video(p)
        items.extend(FrameItem(p, s, e) for s, e in idx)
    return items


def save_frame_items(items, path: str) -> None:
    with open(path, "w") as f:
        for it in items:
            f.write(json.dumps({"video_path": it.video_path, "frame_start": it.frame_start,
                                "frame_end": it.frame_end}) + "\n")


def load_frame_items(path: str) -> list:
    base = os.path.dirname(os.path.abspath(path))
    out = []
    with open(path) as f:
        for line in f:
            if line.strip():
                d = json.loads(line)
                vp = d["video_path"]
                out.append(FrameItem(vp if os.path.isabs(vp) else os.path.join(base, vp),
                                     int(d["frame_start"]), int(d["frame_end"])))
    return out


# ----------------------------------------------------------------- frame transform (GPU)
_plans: dict = {}


def _plan(in_size: int, out_size: int, device):
    key = (in_size, out_size, str(device))
    if key not in _plans:
        cap = 2 * -(-in_size // out_size) + 1
        bounds = np.zeros((out_size, 2), np.int32)
        coef = np.zeros((out_size, cap), np.int32)
        _lib.call("vd_resize_plan", in_size, out_size, bounds.ctypes.data, coef.ctypes.data, cap)
        _plans[key] = (torch.from_numpy(bounds).to(device), torch.from_numpy(coef).to(device), cap)
    return _plans[key]


def transform_frames(frames: torch.Tensor, size: int = 128, dtype=torch.float32,
                     out: torch.Tensor | None = None) -> torch.Tensor:
    """ToPILImage -> Resize((size, size)) -> ToTensor -> Normalize(0.5, 0.5) (train.py:70-75)
    on the GPU: uint8 [n, H, W, 3] (device) -> [n, 3, size, size] in [-1, 1]."""
    if not frames.is_cuda:
        raise RuntimeError("transform_frames runs on the GPU only (no CPU fallback)")
    frames = frames.contiguous()
    n, H, W, _ = frames.shape
    xb, xc, xk = _plan(W, size, frames.device)
    yb, yc, yk = _plan(H, size, frames.device)
    tmp = torch.empty((n, H, size, 3), dtype=torch.uint8, device=frames.device)
    if out is None:
        out = torch.empty((n, 3, size, size), dtype=dtype, device=frames.device)
    dt = {torch.float32: _lib.VD_F32, torch.bfloat16: _lib.VD_BF16}[out.dtype]
    _lib.call("vd_frames_resize_normalize", frames.data_ptr(), n, H, W, size, size,
              xb.data_ptr(), xc.data_ptr(), xk, yb.data_ptr(), yc.data_ptr(), yk, tmp.data_ptr(),
              out.data_ptr(), dt, 3 * size * size, 0,
              torch.cuda.current_stream(frames.device).cuda_stream)
    return out


def audio_window(wave: np.ndarray, sr: int, fps: float, out_frame: int, buffer_frames: int = 5,
                 target_len: int = 4000, target_sr: int = 16000,
                 bug_compatible: bool = True) -> np.ndarray:
    """dataset.py:113-130 (host DSP in libvdiff): input_values fp32 [C, target_len]."""
    wave = np.ascontiguousarray(np.atleast_2d(wave), dtype=np.float32)
    out = np.empty((wave.shape[0], target_len), np.float32)
    _lib.call("vd_audio_window", wave.ctypes.data, wave.shape[0], wave.shape[1], int(sr),
              float(fps), int(out_frame), int(buffer_frames), int(target_len), int(target_sr),
              int(bool(bug_compatible)), out.ctypes.data)
    return out


def _device_error(e: BaseException) -> bool:
    """A HIP/CUDA initialisation or launch failure: never swallowed into (None, None) (a
    forked DataLoader worker cannot re-initialise the GPU; hiding that only moves the error
    to collate)."""
    if not isinstance(e, RuntimeError):
        return False
    msg = str(e)
    # specific markers only: a bare "hip" / "cuda" substring also matches paths such as
    # .../ship/... or .../barracuda/... of an ordinary per-item data error
    markers = ("HIP error", "hipError", "CUDA error", "CUDA driver", "CUDA out of memory",
               "HIP out of memory", "Cannot re-initialize CUDA", "no CUDA GPUs",
               "Found no NVIDIA driver", "libvdiff ", "libvdiff.so", "device-side assert")
    return any(k in msg for k in markers)


class TalkingFaceFrameDataset(torch.utils.data.Dataset):
    """dataset.py:68-139 over .vdclip files: (input_frame, output_frame,
    {"input_values": [C, 4000]}); on a data error it prints and returns (None, None) like the
    reference.  Frames are what the reference returns: the raw uint8 [H, W, 3] frames when
    `frame_transforms` is None, else frame_transforms(frame) (the reference's torchvision
    Compose, on the host).  gpu_transform=True (opt-in, main process only) instead runs
    ToPILImage -> Resize -> ToTensor -> Normalize on `device` (vd_frames_resize_normalize)
    and returns [3, S, S] tensors there; device errors are raised, not swallowed.
    bug_compatible: reproduce process_audio's resample from orig_freq = channel count
    (dataset.py:53); False resamples from the track's rate (identity at 16 kHz)."""

    def __init__(self, frame_items, frame_transforms=None, frame_rate=30, audio_transforms=None,
                 *, image_size=128, gpu_transform=False, device="cuda", bug_compatible=True):
        self.frame_items = frame_items
        self.frame_transforms = frame_transforms
        self.frame_rate = frame_rate
        self.audio_transforms = audio_transforms
        self.image_size = image_size
        self.gpu_transform = gpu_transform
        self.device = device
        self.bug_compatible = bug_compatible

    def __len__(self):
        return len(self.frame_items)

    def __getitem__(self, idx):
        it = self.frame_items[idx]
        try:
            c = open_clip(it.video_path)
            if c.fps == 0:
                raise ValueError("FPS is zero, which may indicate an issue with the video file")
            out_idx = min(it.frame_end, len(c) - 1)
            pair = np.stack([c.frames[0], c.frames[out_idx]])  # input_frame_idx = 0 (:98)
            if self.gpu_transform:
                f = transform_frames(torch.from_numpy(pair).to(self.device), self.image_size)
                inp, outp = f[0], f[1]
            elif self.frame_transforms is not None:
                inp, outp = self.frame_transforms(pair[0]), self.frame_transforms(pair[1])
            else:
                inp, outp = pair[0], pair[1]
            a = audio_window(c.audio, c.sr, c.fps, out_idx, bug_compatible=self.bug_compatible)
            a = torch.from_numpy(a)
            if self.audio_transforms is not None:
                a = self.audio_transforms(a)
            return inp, outp, {"input_values": a}
        except Exception as e:  # the reference's contract (dataset.py:137-139)
            if _device_error(e):
                raise
            print(f"Error processing video {it.video_path}: {e}")
            return None, None


@dataclass
class _Sample:
    clip: ClipFile
    out_idx: list


@dataclass
class _HostBatch:
    frames: torch.Tensor | None   # pinned uint8 [B*(T+1), H, W, 3] (one frame size), or None
    per_clip: list | None         # [uint8 [T+1, H, W, 3]] when the frame sizes differ
    audio: torch.Tensor           # pinned fp32 [B*T, 4000]


class ClipBatcher:
    """Training batches for the frame-stack denoiser from a frame index: per item the
    conditioning image is frame 0, the targets are `frames` consecutive output frames from
    min(frame_end, F - 1) on (stepping like the index, clipped to the last frame), each with
    its own audio window (frames = 1 is the reference's per-frame sample).

    The host half of a batch (item draws, memory-mapped frame reads, the audio-window DSP,
    pinned staging) runs on a background thread `prefetch` batches ahead -- the reference's
    DataLoader(num_workers=4) (train.py:82) in one process, with no GPU context in a
    worker.  The libvdiff DSP releases the GIL (ctypes), so it overlaps the host's kernel
    launches.  next() takes the prepared batch, uploads it on the current stream (pinned,
    asynchronous) and runs the resize kernel; eps and t are drawn on the device.  Draws are
    sequential on one thread, so batches are the same as prefetch=0.  Returns
    vdiff.engine.Clip."""

    def __init__(self, items, batch, frames, num_timesteps, device, size=128, seed=0,
                 bug_compatible=True, dims=3, prefetch=2):
        self.items, self.batch, self.frames, self.size = list(items), batch, frames, size
        self.num_timesteps, self.device, self.dims = num_timesteps, device, dims
        self.bug_compatible = bug_compatible
        self.rng = np.random.default_rng(seed)
        self.gen = torch.Generator(device=device).manual_seed(seed)
        if not self.items:
            raise ValueError("empty frame index")
        self.prefetch = int(prefetch)
        self._pool = None
        self._pending = []
        if self.prefetch > 0:
            from concurrent.futures import ThreadPoolExecutor
            self._pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="vdclip")

    def _sample(self, it):
        c = open_clip(it.video_path)
        step = max(1, it.frame_end - it.frame_start)
        o = min(it.frame_end, len(c) - 1)
        return _Sample(c, [min(o + k * step, len(c) - 1) for k in range(self.frames)])

    def _host_batch(self) -> _HostBatch:
        B = self.batch
        picks = [self._sample(self.items[i])
                 for i in self.rng.integers(0, len(self.items), size=B)]
        stacks = [np.stack([p.clip.frames[0]] + [p.clip.frames[i] for i in p.out_idx])
                  for p in picks]
        audio = [audio_window(p.clip.audio, p.clip.sr, p.clip.fps, i,
                              bug_compatible=self.bug_compatible)[0]  # mono: channel 0
                 for p in picks for i in p.out_idx]
        pin = torch.cuda.is_available()
        audio = torch.from_numpy(np.stack(audio))
        audio = audio.pin_memory() if pin else audio
        if len({s.shape for s in stacks}) == 1:  # one upload and two launches for the batch
            fr = torch.from_numpy(np.concatenate(stacks))
            return _HostBatch(fr.pin_memory() if pin else fr, None, audio)
        return _HostBatch(None, [torch.from_numpy(s) for s in stacks], audio)

    def _fill(self):
        while len(self._pending) < self.prefetch:
            self._pending.append(self._pool.submit(self._host_batch))

    def next(self):
        from .engine import Clip
        if self._pool is None:
            hb = self._host_batch()
        else:
            self._fill()
            hb = self._pending.pop(0).result()
            self._fill()  # the next batch's host work starts now, beside this step
        B, T, S = self.batch, self.frames, self.size
        x0 = torch.empty((B, T, 3, S, S), device=self.device)
        cond = torch.empty((B, 3, S, S), device=self.device)
        if hb.frames is not None:
            dev = hb.frames.to(self.device, non_blocking=True)
            f = transform_frames(dev, S).reshape(B, T + 1, 3, S, S)
            cond.copy_(f[:, 0])
            x0.copy_(f[:, 1:])
        else:
            for b, fr in enumerate(hb.per_clip):
                f = transform_frames(fr.to(self.device), S)
                cond[b], x0[b] = f[0], f[1:]
        audio = hb.audio.to(self.device, non_blocking=True)
        x0 = x0.transpose(1, 2).contiguous() if self.dims == 3 else x0[:, 0].contiguous()
        eps = torch.randn(x0.shape, generator=self.gen, device=self.device)
        t = torch.randint(0, self.num_timesteps, (B,), generator=self.gen, device=self.device)
        return Clip(x0, cond, {"input_values": audio}, eps, t)

    def close(self):
        if self._pool is not None:
            self._pool.shutdown(wait=True)
            self._pool = None
            self._pending = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
