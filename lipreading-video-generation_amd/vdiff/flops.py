"""Analytic algorithmic work of the denoiser (the denominators of roofline.achieved).

Counts follow torch.utils.flop_counter conventions on the reference modules (2 FLOP
per MAC): conv = 2*B*out_pixels*Co*Ci*taps; attention = 2 bmm per block =
4*B*heads*N^2*ch (joint), per-frame N = H*W (spatial) or per-pixel N = T (temporal).
Linear layers and elementwise work are not counted.
The training step is counted as 3 x forward (no credit for recompute).
"""
from __future__ import annotations

from dataclasses import dataclass, field


@dataclass
class Work:
    conv: float = 0.0
    attn: float = 0.0
    attn_by_dim: dict = field(default_factory=dict)  # head_dim -> (fwd FLOP, launches, N, nseq)

    @property
    def total(self):
        return self.conv + self.attn


def _conv(w: Work, B, pix, co, ci, taps):
    w.conv += 2.0 * B * pix * co * ci * taps


def _attn(w: Work, B, C, heads, T, HW, mode):
    ch = C // heads
    modes = ["spatial", "temporal"] if mode == "spatial_temporal" else [mode]
    for md in modes:
        if md == "joint":
            nseq, n = B * heads, T * HW
        elif md == "spatial":
            nseq, n = B * heads * T, HW
        else:
            nseq, n = B * heads * HW, T
        f = 4.0 * nseq * n * n * ch
        w.attn += f
        prev = w.attn_by_dim.get((ch, n), (0.0, 0, n, nseq))
        w.attn_by_dim[(ch, n)] = (prev[0] + f, prev[1] + 1, n, nseq)
        # qkv / proj 1x1 convs per sub-attention
        _conv(w, B, T * HW, 3 * C, C, 1)
        _conv(w, B, T * HW, C, C, 1)


def unet_forward_work(model, x_shape, audio_tokens=12) -> Work:
    """Walk a vdiff UNetModel for input shape [B, Cin, (T,) H, W] (audio cross-attention
    branches, when present, onto `audio_tokens` wav2vec2 tokens per frame)."""
    from .nn import AttentionBlock, Downsample, ResBlock, Upsample

    B = x_shape[0]
    if len(x_shape) == 5:
        T, H, W = x_shape[2:]
    else:
        T, (H, W) = 1, x_shape[2:]
    w = Work()
    k = 27 if model.dims == 3 else 9
    state = {"H": H, "W": W}

    def block(seq):
        for layer in seq:
            pix = T * state["H"] * state["W"]
            if isinstance(layer, ResBlock):
                _conv(w, B, pix, layer.out_channels, layer.channels, k)
                _conv(w, B, pix, layer.out_channels, layer.out_channels, k)
                if layer.out_channels != layer.channels:
                    _conv(w, B, pix, layer.out_channels, layer.channels, 1)
            elif isinstance(layer, AttentionBlock):
                _attn(w, B, layer.channels, layer.num_heads, T, state["H"] * state["W"],
                      layer.attention_mode)
                if getattr(layer, "audio_attention", False):  # build extension
                    C, HW = layer.channels, state["H"] * state["W"]
                    L = audio_tokens if layer.audio_per_frame else T * audio_tokens
                    nq = HW if layer.audio_per_frame else T * HW
                    w.attn += 4.0 * B * (T * HW // nq) * nq * L * C
                    _conv(w, B, T * HW, C, C, 1)              # audio_q
                    _conv(w, B, T * HW, C, C, 1)              # audio_proj_out
                    _conv(w, B * T, audio_tokens, 2 * C, layer.audio_kv.in_features, 1)
            elif isinstance(layer, Downsample):
                state["H"] = (state["H"] + 1) // 2
                state["W"] = (state["W"] + 1) // 2
                _conv(w, B, T * state["H"] * state["W"], layer.out_channels, layer.channels, k)
            elif isinstance(layer, Upsample):
                state["H"] *= 2
                state["W"] *= 2
                _conv(w, B, T * state["H"] * state["W"], layer.out_channels, layer.channels, k)
            else:  # the input conv
                _conv(w, B, pix, layer.out_channels, layer.in_channels, k)

    for m in model.input_blocks:
        block(m)
    block(model.middle_block)
    for m in model.output_blocks:
        block(m)
    _conv(w, B, T * H * W, model.out_channels, model.out[2].in_channels, k)
    return w


def attention_kernel_flops(kind: str, n: int, ch: int, nseq: int) -> float:
    """EXECUTED FLOP of one launch of a flash-attention kernel (what the MFMAs do):
    fwd = 2 products (QK^T, PV); bwd dQ = 3 (QK^T and dO V^T recomputed, dS K);
    bwd dK/dV = 4 (QK^T, dO V^T, dO^T P, dS^T Q).  Each product = 2*n*n*ch per sequence.
    The backward pair therefore executes 7 products against 4 algorithmic ones.  "bwd" is the
    fused short-sequence backward (attn_short.hip): S and dP once, dQ, dK, dV = 5 products
    over the sequence padded to 16 / 32 tokens."""
    kind = kind.replace("attn_", "")
    products = {"fwd": 2, "bwd_dq": 3, "bwd_dkdv": 4, "bwd": 5}[kind]
    return products * 2.0 * nseq * n * n * ch


def short_attention_bytes(kind: str, n: int, ch: int, nseq: int, elem: int = 2) -> float:
    """ALGORITHMIC HBM bytes of one short-sequence attention launch (attn_short.hip; the bound
    of the temporal attention, 16 tokens per sequence): forward reads q, k, v and writes o
    (4 rows of ch elements per token) plus the fp32 log-sum-exp; the fused backward reads q,
    k, v, dO and lse and writes dq, dk, dv (7 rows per token: since round 5 it takes
    delta = rowsum(P dP) from the scores it holds instead of reading o)."""
    rows = {"fwd": 4, "bwd": 7}[kind.replace("attn_", "")]
    return float(nseq) * n * (rows * ch * elem + 4)


def attention_unit_flops(unit: str, n: int, ch: int, nseq: int) -> float:
    """ALGORITHMIC FLOP of one attention unit (backward = 2x forward, no credit
    for recompute): unit "fwd" = 2 products (QK^T, PV); unit "bwd" = the dQ + dK/dV
    launch pair = 4 products (dO V^T, P^T dO, dS K, dS^T Q) -- the S = QK^T each kernel
    recomputes and the dP = dO V^T the dQ kernel recomputes are not counted."""
    products = {"fwd": 2, "bwd": 4}[unit]
    return products * 2.0 * nseq * n * n * ch
