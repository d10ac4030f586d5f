"""Time the single-K-step 1x1 conv forwards of the UNet3D at 128x128x16 (qkv 64->192 and
proj 64->64 over 262144 pixels) with HIP events; VDIFF_CONV_1X1 selects the tile variant."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd"))

import torch  # noqa: E402

from vdiff import ops  # noqa: E402

for Ci, Co, P in ((64, 192, 262144), (64, 64, 262144), (32, 96, 262144)):
    x = ops.to_cl(torch.randn(1, Ci, P, device="cuda", dtype=torch.bfloat16))
    w = torch.randn(Co, Ci, 1, device="cuda") / Ci ** 0.5
    b = torch.randn(Co, device="cuda")
    y = ops.conv(x, w, b)
    ref = (torch.einsum("oc,cp->op", w[:, :, 0], x[0].float()) + b[:, None])
    err = float((y[0].float() - ref).norm() / ref.norm())
    for _ in range(3):
        ops.conv(x, w, b)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.conv(x, w, b)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    gb = (P * Ci + P * Co) * 2 / 1e9
    print(f"variant {os.environ.get('VDIFF_CONV_1X1', '0')} {Ci:4d}->{Co:4d} x {P}: {ms * 1e3:7.1f} us "
          f"(incl. weight pack) {gb / ms * 1e3:6.0f} GB/s  rel-L2 {err:.1e}", flush=True)
