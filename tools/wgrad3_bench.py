"""Time the 3x3x3 conv weight gradients of the UNet3D train step (128x128x16, bf16) with HIP
events: vd_conv3d_bwd_weight for every stride-1 3x3x3 shape of the step with its per-step
launch count (profiles/r02_conv_breakdown.txt), checked against torch's fp32 conv3d weight
gradient.  The kernel variant comes from VDIFF_WGRAD3=nst,cot (read once per process).
Prints per-shape microseconds and TFLOP/s and the per-step total."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd"))

import torch  # noqa: E402

from vdiff import _lib, ops  # noqa: E402

# (Ci, Co, H = W, launches per train step); T = 16 frames
SHAPES = ((256, 256, 32, 10), (64, 64, 128, 7), (128, 128, 64, 6), (128, 64, 128, 2),
          (200, 64, 128, 1), (512, 256, 32, 2), (128, 128, 128, 1), (256, 256, 64, 1),
          (384, 128, 64, 1), (192, 64, 128, 1), (256, 128, 64, 1), (192, 128, 64, 1),
          (384, 256, 32, 1), (64, 128, 64, 1), (128, 256, 32, 1))


def main():
    variant = os.environ.get("VDIFF_WGRAD3", "2,64")
    total, worst = 0.0, 0.0
    T = 16
    for Ci, Co, H, per in SHAPES:
        g = torch.Generator(device="cuda").manual_seed(Ci * 7 + Co + H)
        x = torch.randn(1, T, H, H, Ci, generator=g, device="cuda").bfloat16()
        dy = torch.randn(1, T, H, H, Co, generator=g, device="cuda").bfloat16()
        d = ops._desc(1, [T, H, H], Ci, [T, H, H], Co, [3, 3, 3], [1, 1, 1], [1, 1, 1],
                      ops._DT[torch.bfloat16])
        dw = torch.zeros(Co, 27, Ci, dtype=torch.float32, device="cuda")
        st = ops._stream(x)

        def run():
            dw.zero_()
            _lib.call("vd_conv3d_bwd_weight", d, x.data_ptr(), dy.data_ptr(), dw.data_ptr(), st)

        run()
        xr = x.float().permute(0, 4, 1, 2, 3)
        dyr = dy.float().permute(0, 4, 1, 2, 3)
        ref = torch.nn.grad.conv3d_weight(xr, (Co, Ci, 3, 3, 3), dyr, padding=1)
        ref = ref.reshape(Co, Ci, 27).permute(0, 2, 1)
        err = float((dw - ref).norm() / ref.norm())
        worst = max(worst, err)
        for _ in range(3):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        e0.record()
        for _ in range(reps):
            dw.zero_()
        e1.record()
        torch.cuda.synchronize()
        us -= e0.elapsed_time(e1) / reps * 1e3
        tf = 2.0 * T * H * H * Co * 27 * Ci / (us * 1e-6) / 1e12
        total += us * per
        print(f"[{variant}] wgrad 3x3x3 {Ci:4d}->{Co:4d} at {T}x{H}x{H}: {us:7.1f} us "
              f"{tf:7.1f} TF/s  rel-L2 {err:.1e}", flush=True)
    print(f"[{variant}] per train step: {total / 1e3:.3f} ms (worst rel-L2 {worst:.1e})",
          flush=True)
    assert worst < 1e-2


if __name__ == "__main__":
    main()
