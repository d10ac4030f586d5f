"""Time the 1x1 conv weight gradients of the UNet3D train step (128x128x16, bf16) with HIP
events: vd_conv3d_bwd_weight for every 1x1 shape of the step, with the per-step launch
counts of profiles/r02_conv_breakdown.txt, checked against a torch fp32 dY^T X.  The kernel
variant comes from VDIFF_WGRAD1=nst,cot (read once per process: run one process per
variant).  Prints per-shape microseconds, algorithmic GB/s (X + dY read once) and the
per-step total."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd"))

import torch  # noqa: E402

from vdiff import _lib, ops  # noqa: E402

# (Ci, Co, pixels, launches per train step)
SHAPES = ((64, 192, 262144, 5), (128, 384, 65536, 5), (256, 768, 16384, 6),
          (256, 256, 16384, 6), (64, 64, 262144, 5), (128, 128, 65536, 5),
          (128, 64, 262144, 2), (512, 256, 16384, 2), (192, 64, 262144, 1),
          (384, 128, 65536, 1), (256, 128, 65536, 1), (192, 128, 65536, 1),
          (384, 256, 16384, 1), (128, 256, 16384, 1), (64, 128, 65536, 1))


def main():
    variant = os.environ.get("VDIFF_WGRAD1", "2,64")
    total = 0.0
    worst = 0.0
    for Ci, Co, P, per in SHAPES:
        g = torch.Generator(device="cuda").manual_seed(Ci * 7 + Co)
        x = torch.randn(1, P, Ci, generator=g, device="cuda").bfloat16()
        dy = torch.randn(1, P, Co, generator=g, device="cuda").bfloat16()
        d = ops._desc(1, [1, 1, P], Ci, [1, 1, P], Co, [1, 1, 1], [1, 1, 1], [0, 0, 0],
                      ops._DT[torch.bfloat16])
        dw = torch.zeros(Co, 1, Ci, dtype=torch.float32, device="cuda")
        st = ops._stream(x)

        def run():
            dw.zero_()
            _lib.call("vd_conv3d_bwd_weight", d, x.data_ptr(), dy.data_ptr(), dw.data_ptr(), st)

        run()
        ref = dy[0].float().T @ x[0].float()
        err = float((dw[:, 0] - ref).norm() / ref.norm())
        worst = max(worst, err)
        for _ in range(3):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        zero_us = 0.0
        e0.record()
        for _ in range(reps):
            dw.zero_()
        e1.record()
        torch.cuda.synchronize()
        zero_us = e0.elapsed_time(e1) / reps * 1e3
        us -= zero_us
        gbs = P * (Ci + Co) * 2 / (us * 1e-6) / 1e9
        total += us * per
        print(f"[{variant}] wgrad 1x1 {Ci:4d}->{Co:4d} x {P:6d} px: {us:7.1f} us  {gbs:7.1f} GB/s"
              f"  rel-L2 {err:.1e}", flush=True)
    print(f"[{variant}] per train step: {total / 1e3:.3f} ms (worst rel-L2 {worst:.1e})",
          flush=True)
    assert worst < 1e-2


if __name__ == "__main__":
    main()
