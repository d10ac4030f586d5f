"""Micro-benchmark of the flash-attention kernels at the UNet3D 128x128x16 shapes
(joint attention, 1 head): level 0 (d 64, N 262144), level 1 (d 128, N 65536),
level 2 (d 256, N 16384).  Times fwd / bwd_dq / bwd_dkdv per launch with HIP
events on the launch stream; prints TFLOP/s and fraction of the 2.5 PF/s bf16 peak.
Also checks a small case against a materialised fp32 softmax reference."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd"))

import torch  # noqa: E402

from vdiff import ops  # noqa: E402
from vdiff.flops import attention_kernel_flops  # noqa: E402


def check():
    torch.manual_seed(0)
    for C, N in ((64, 300), (128, 200), (256, 130)):
        qkv = torch.randn(1, 3 * C, N, device="cuda")
        q, k, v = qkv.reshape(3, C, N)
        ref = torch.softmax((q.T @ k) / C ** 0.5, -1) @ v.T
        out = ops.attention(ops.to_cl(qkv.bfloat16()), 1)
        e = ((out.float()[0].T - ref).norm() / ref.norm()).item()
        print(f"check C={C} N={N}: rel-L2 {e:.2e}", flush=True)
        assert e < 2e-2


def bench(C, N, reps, bwd=True, mode="joint", T=16):
    """mode "temporal": the spatial_temporal mode's per-pixel sequences of T frames over the
    N = T * HW tokens of a clip (the short-sequence kernels, HBM-bound: GB/s reported)."""
    from vdiff.flops import short_attention_bytes
    sp = (T, N // T, 1) if mode != "joint" else None
    qkv = ops.to_cl(torch.randn(1, 3 * C, N, device="cuda", dtype=torch.bfloat16))
    qkv.requires_grad_(True)
    g = ops.to_cl(torch.randn(1, C, N, device="cuda", dtype=torch.bfloat16))
    for _ in range(1):
        out = ops.attention(qkv, 1, mode=mode, spatial=sp)
        if bwd:
            out.backward(g)
    torch.cuda.synchronize()
    timer = ops.KernelTimer()
    ops.set_timer(timer)
    for _ in range(reps):
        out = ops.attention(qkv, 1, mode=mode, spatial=sp)
        if bwd:
            out.backward(g)
    ops.set_timer(None)
    for (kind, hd, n, nseq), (cnt, tot) in sorted(timer.summary().items()):
        f = attention_kernel_flops(kind, n, hd, nseq)
        avg = tot / cnt
        extra = ""
        if n <= 32:
            extra = f"  {short_attention_bytes(kind, n, hd, nseq) / avg / 1e6:7.1f} GB/s"
        print(f"{kind:14s} d={hd:3d} N={n:6d} x{nseq}: {avg:8.3f} ms  {f / avg / 1e9:7.1f} TF/s "
              f"({f / avg / 1e9 / 2500 * 100:5.1f}% of 2.5 PF){extra}", flush=True)


CALIB_ELEMS = 1 << 27   # bf16 elements per operand: 256 MiB each, past the 256 MiB L3


def calib():
    """PMC calibration launch: q_sample over bf16 streams (16 B per lane loads and stores).
    Algorithmic bytes per launch: 2 reads + 1 write of CALIB_ELEMS bf16 (tools/pmc_traffic.py)."""
    x = torch.randn(CALIB_ELEMS, device="cuda", dtype=torch.bfloat16).view(4, -1)
    e = torch.randn_like(x)
    t = torch.tensor([1, 2, 3, 4], device="cuda")
    tab = torch.linspace(0.1, 0.9, 1000, device="cuda")
    for _ in range(3):
        ops.q_sample(x, e, t, tab, tab)
    torch.cuda.synchronize()


if __name__ == "__main__":
    if "--calib" in sys.argv:
        calib()
        sys.argv.remove("--calib")
    only = None
    if "--only" in sys.argv:  # --only 64: just the head_dim 64 level
        i = sys.argv.index("--only")
        only = int(sys.argv[i + 1])
        del sys.argv[i:i + 2]
    if "--nocheck" in sys.argv:  # ablation builds are wrong by design
        sys.argv.remove("--nocheck")
    else:
        check()
    temporal = "--temporal" in sys.argv  # the short-sequence kernels (spatial_temporal mode)
    if temporal:
        sys.argv.remove("--temporal")
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    for C, N in ((64, 262144), (128, 65536), (256, 16384)):
        if only is None or C == only:
            if temporal:
                bench(C, N, reps, mode="temporal")
            else:
                bench(C, N, reps)
