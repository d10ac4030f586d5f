"""Edge inputs of the C-ABI host code (CPU, no GPU call): the audio-window DSP at the ends of
the track and for tiny / multi-channel tracks, the PIL resize plan for up-, down- and
identity scales and a too-small tap cap, and argument checks that must fail with a status
and a message.  Also run against the ASan/UBSan build (csrc/Makefile.asan `check`), where
any out-of-bounds access or undefined behaviour aborts the run."""
import ctypes

import numpy as np
import pytest

from oracle import data as od
from vdiff import _lib
from vdiff import data as vd


def _wave(C, n, seed):
    g = np.random.default_rng(seed)
    return (0.3 * np.sin(np.arange(n) * 0.03)[None] + 0.1 * g.standard_normal((C, n))
            ).astype(np.float32)


@pytest.mark.parametrize("C,n,sr,fps,frames", [
    (1, 16000, 16000, 25.0, (1, 5, 24, 25, 26, 400)),   # past the end: empty / clipped windows
    (2, 3000, 8000, 30.0, (1, 2, 11, 12, 90)),           # stereo, tiny track
    (3, 40, 16000, 30.0, (0, 1, 6)),                     # fewer samples than one frame
    (1, 48000, 48000, 29.97, (7, 300)),                  # 48 kHz, NTSC rate
])
@pytest.mark.parametrize("bug", [True, False])
def test_audio_window_edges(C, n, sr, fps, frames, bug):
    wave = _wave(C, n, C * 7 + n)
    for f in frames:
        got = vd.audio_window(wave, sr, fps, f, bug_compatible=bug)
        assert got.shape == (C, 4000) and np.isfinite(got).all()
        s0 = int(sr * max(0.0, (f - 5) / fps))
        s1 = min(int(sr * f / fps), n)
        if s1 - s0 >= 2:  # a window with a defined std: the oracle's arithmetic
            ref = od.audio_window(wave, sr, fps, f, bug_compatible=bug)
            np.testing.assert_allclose(got, ref, rtol=0, atol=2e-4)


@pytest.mark.parametrize("n_in,n_out", [(1, 1), (1, 128), (3, 128), (128, 1), (1000, 7),
                                        (129, 128), (127, 128), (4096, 128)])
def test_resize_plan_edges(n_in, n_out):
    cap = 2 * -(-n_in // n_out) + 1
    b = np.zeros((n_out, 2), np.int32)
    c = np.zeros((n_out, cap), np.int32)
    _lib.call("vd_resize_plan", n_in, n_out, b.ctypes.data, c.ctypes.data, cap)
    assert (b[:, 0] >= 0).all() and (b[:, 0] + b[:, 1] <= n_in).all() and (b[:, 1] >= 1).all()
    assert (b[:, 1] <= cap).all()
    assert np.abs(c.sum(1) - (1 << 22)).max() <= cap


def test_resize_plan_rejects_small_cap():
    b = np.zeros((16, 2), np.int32)
    c = np.zeros((16, 3), np.int32)
    with pytest.raises(RuntimeError, match="taps"):
        _lib.call("vd_resize_plan", 160, 16, b.ctypes.data, c.ctypes.data, 3)


def test_argument_checks_fail_with_a_message():
    lib = _lib.load()
    out = np.zeros((1, 4000), np.float32)
    rc = lib.vd_audio_window(None, 1, 100, 16000, ctypes.c_double(30.0), 3, 5, 4000, 16000, 1,
                             ctypes.c_void_p(out.ctypes.data))
    assert rc != 0 and b"audio" in lib.vd_last_error()
    rc = lib.vd_resize_plan(0, 16, None, None, 3)
    assert rc != 0 and b"resize" in lib.vd_last_error()
