"""Time the UNet3D 1x1 convs (fwd and bwd-data) at the 128x128x16 shapes with HIP events:
level 0 (262144 pixels: qkv 64->192, proj 64->64, skip 128->64) and level 1 (65536 pixels:
qkv 128->384, proj 128->128).  VDIFF_CONV_PW=0 turns the streaming 1x1 kernel off
(igemm tiles); GB/s counts the algorithmic bytes (X in + Y out, bf16)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd"))

import torch  # noqa: E402

from vdiff import _lib, ops  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


tag = "pw" if os.environ.get("VDIFF_CONV_PW", "1") != "0" else "igemm"
for Ci, Co, P in ((64, 192, 262144), (64, 64, 262144), (128, 64, 262144), (128, 384, 65536),
                  (128, 128, 65536), (256, 768, 16384), (256, 256, 16384)):
    x = ops.to_cl(torch.randn(1, Ci, P, device="cuda", dtype=torch.bfloat16))
    w = torch.nn.Parameter(torch.randn(Co, Ci, 1, device="cuda") / Ci ** 0.5, requires_grad=False)
    b = torch.randn(Co, device="cuda")
    dy = ops.to_cl(torch.randn(1, Co, P, device="cuda", dtype=torch.bfloat16))
    xg = x.detach().requires_grad_(True)
    with ops.frozen_weights():  # packed weights cached: time the conv kernels alone
        y = ops.conv(x, w, b)
        ref = (torch.einsum("oc,cp->op", w[:, :, 0], x[0].float()) + b[:, None])
        err = float((y[0].float() - ref).norm() / ref.norm())
        ms_f = timeit(lambda: ops.conv(x, w, b))
        # fwd + bwd-data (x only needs a gradient: no weight / bias gradient kernels)
        ms_b = timeit(lambda: torch.autograd.grad(ops.conv(xg, w, b), xg, dy)) - ms_f
    gb = (P * Ci + P * Co) * 2 / 1e9
    print(f"{tag:6s} {Ci:4d}->{Co:4d} x {P}: fwd {ms_f * 1e3:7.1f} us {gb / ms_f * 1e3:6.0f} GB/s"
          f"  bwd-data {ms_b * 1e3:7.1f} us {gb / ms_b * 1e3:6.0f} GB/s  rel-L2 {err:.1e}",
          flush=True)

# proj_out with the block's residual fused into the store (AttentionBlock, unet.py:317):
# GB/s counts X + residual in + Y out
tag_r = tag
for C, P in ((64, 262144), (128, 65536), (256, 16384)):
    x = ops.to_cl(torch.randn(1, C, P, device="cuda", dtype=torch.bfloat16))
    r = ops.to_cl(torch.randn(1, C, P, device="cuda", dtype=torch.bfloat16))
    w = torch.nn.Parameter(torch.randn(C, C, 1, device="cuda") / C ** 0.5, requires_grad=False)
    b = torch.randn(C, device="cuda")
    with ops.frozen_weights():
        y = ops.conv(x, w, b, residual=r)
        ref = (torch.einsum("oc,cp->op", w[:, :, 0], x[0].float()) + b[:, None] + r[0].float())
        err = float((y[0].float() - ref).norm() / ref.norm())
        ms_f = timeit(lambda: ops.conv(x, w, b, residual=r))
    gb = 3 * P * C * 2 / 1e9
    print(f"{tag_r:6s} proj {C:4d}->{C:4d} x {P} + residual: fwd {ms_f * 1e3:7.1f} us "
          f"{gb / ms_f * 1e3:6.0f} GB/s  rel-L2 {err:.1e}", flush=True)
