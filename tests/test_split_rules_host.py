"""Host-side split rules (CPU, no GPU call), through the C-ABI workspace-size functions, which
run the launchers' own shape logic without launching:

- the conv weight gradient (conv.hip wgrad_run): pixel splits of the kw-strip / 1x1 kernels
  under the occupancy-round rule and the per-shape kw-strip tile width (round 4), restated
  here and checked for every 3x3x3 / 1x1 shape of the config-2 train step;
- the hand-scheduled head_dim-256 forward (attention.hip fwd256_lsplit): key splits, <= 4,
  every split non-empty, whole 128-key iterations, the grid filling the chip.

The default environment is assumed (no VDIFF_WGRAD* / VDIFF_ASM256* overrides)."""
import os

import pytest

from vdiff import _lib, ops
import torch

ENV = ("VDIFF_WGRAD1", "VDIFF_WGRAD3", "VDIFF_WGRAD_QRULE", "VDIFF_WGRAD_SPLITS",
       "VDIFF_CONV_WPLANE", "VDIFF_ASM256_FWD",
       "VDIFF_ATTN_CFG", "VDIFF_CONV_DMA", "VDIFF_CONV_LEGACY")
pytestmark = pytest.mark.skipif(any(os.environ.get(e) for e in ENV),
                                reason="non-default kernel-selection environment")

# (Ci, Co, k, H = W, T) of the config-2 step (tools/wgrad3_bench.py SHAPES)
SHAPES = ((256, 256, 3, 32, 16), (64, 64, 3, 128, 16), (128, 128, 3, 64, 16),
          (128, 64, 3, 128, 16), (200, 64, 3, 128, 16), (512, 256, 3, 32, 16),
          (128, 128, 3, 128, 16), (256, 256, 3, 64, 16), (384, 128, 3, 64, 16),
          (192, 64, 3, 128, 16), (256, 128, 3, 64, 16), (192, 128, 3, 64, 16),
          (384, 256, 3, 32, 16), (64, 128, 3, 64, 16), (128, 256, 3, 32, 16),
          (64, 8, 3, 128, 16), (256, 768, 1, 128, 1), (64, 192, 1, 512, 1),
          (128, 384, 1, 256, 1), (64, 64, 1, 512, 1), (256, 256, 1, 128, 1),
          (128, 128, 1, 256, 1))


def cdiv(a, b):
    return -(-a // b)


def real_splits(M, s):
    """splits after rounding the pixels per split up to whole 64-pixel steps"""
    return cdiv(M, cdiv(cdiv(M, s), 64) * 64)


def expected_splits(Ci, Co, k, H, T):
    """conv.hip wgrad_run, LDS-DMA branch, default knobs (VDIFF_WGRAD1 = 4,64;
    VDIFF_WGRAD3 = 2,0,32; occupancy-round rule on)."""
    M = T * H * H
    one = k == 1
    wc = 64 if one else min(H, 64)
    rows = 64 if one else (64 // wc) * (wc + 2)
    rw = 96 if rows <= 96 else 128 if rows <= 128 else 192
    taps_rows = 1 if one else 3 * 3            # kt * kh tile rows of the kw strip
    if one:
        cot, nst = 64, 4
    else:
        nst = 2
        slots128 = 256 * max(1, min(3, 163840 // (nst * (128 + rw) * 128)))
        fill128 = cdiv(Co, 128) * cdiv(Ci, 64) * taps_rows * cdiv(M, 64 * 32) * 10 >= 9 * slots128
        cot = 128 if Co % 128 == 0 and fill128 else 64
    tiles = cdiv(Co, cot) * cdiv(Ci, 64) * taps_rows
    s = cdiv(2048, tiles)
    s = min(s, cdiv(M, 1024 if one else 64 * 32))
    ring = nst * (cot + (64 if one else rw)) * 128
    slots = 256 * max(1, min(3, 163840 // ring))
    pick = fill_pick = 0
    best = -1.0
    for c in range(max(1, s // 3), s + 1):
        r = tiles * real_splits(M, c) / slots
        if r < 0.9:
            continue
        fill = r / -(-r // 1)
        if fill >= 0.93:
            pick = c
            break
        if fill > best + 1e-9:
            best, fill_pick = fill, c
    s0 = real_splits(M, max(1, s))
    s = pick or fill_pick or s
    return real_splits(M, max(1, s)), tiles, slots, s0


@pytest.mark.parametrize("Ci,Co,k,H,T", SHAPES)
def test_wgrad_split_rule(Ci, Co, k, H, T):
    p = k // 2
    d = ops._desc(1, [T, H, H], Ci, [T, H, H], Co, [k] * 3 if k == 3 else [1, 1, 1],
                  [1, 1, 1], [p] * 3, ops._DT[torch.bfloat16])
    ws = _lib.lib().vd_conv3d_bwd_weight_workspace_size(d)
    taps = k ** 3
    per_split = Co * taps * Ci * 4
    assert (ws - 256) % per_split == 0
    got = (ws - 256) // per_split
    want, tiles, slots, before = expected_splits(Ci, Co, k, H, T)
    assert got == want, (got, want)
    # every split non-empty; the last round of resident workgroups no emptier than under the
    # pre-round-4 count (which the rule only ever lowers, by at most 3x)
    M = T * H * H
    assert (got - 1) * cdiv(cdiv(M, got), 64) * 64 < M
    assert before // 3 <= got <= before

    def fill(n):
        r = tiles * n / slots
        return r / -(-r // 1)
    if tiles * got / slots >= 0.9:
        assert fill(got) >= fill(before) - 1e-9


@pytest.mark.parametrize("nseq,N", [(1, 16384), (1, 16401), (2, 3000), (1, 1024), (4, 1024),
                                    (16, 1024), (1, 65536)])
def test_fwd256_key_splits(nseq, N):
    """vd_attention_fwd_workspace_size for the head_dim-256 asm forward: max(the asm split,
    the compiled fallback's split) x rows x (256 + 2) fp32; the asm split count follows the
    dQ rule and leaves every split non-empty."""
    (d, *_), = ops._attn_desc(nseq, N, 256, 1, 256, "joint", None, ops._DT[torch.bfloat16],
                              True)
    ws = _lib.lib().vd_attention_fwd_workspace_size(d)
    wgs = cdiv(N, 128) * nseq
    lsplit = 0
    while lsplit < 2 and (wgs << lsplit) < 256:
        S = 2 << lsplit
        kps = cdiv(cdiv(N, S), 128) * 128
        if (S - 1) * kps >= N:
            break
        lsplit += 1
    S = 1 << lsplit
    kps = cdiv(cdiv(N, S), 128) * 128
    assert (S - 1) * kps < N <= S * kps
    # the compiled 4-wave fallback's KV split (attention.hip kv_splits)
    kv = 1
    if wgs < 256:
        kv = min(4, cdiv(256, wgs))
        while kv > 1 and cdiv(N, 64) // kv < 4:
            kv -= 1
    s = max(S, kv)
    assert ws == (s * nseq * N * (256 + 2) * 4 if s > 1 else 0), (ws, S, kv)
