"""A/B of the conv weight gradients of the config-2 train step (128x128x16, bf16): every
3x3x3 stride-1 and 1x1 shape of the step with its per-step launch count, through
vd_conv3d_bwd_weight_det (fixed-order split-K, the default) or vd_conv3d_bwd_weight (atomics,
VDIFF_WGRAD_ATOMIC=1), timed with HIP events; the grid layout follows VDIFF_WGRAD_XCD (read
once per process).  Checked against the fp32 parity-mode weight gradient of the same values on
the device (whole tensors).  Prints per-shape microseconds / TFLOP/s and the per-step totals.
    VDIFF_WGRAD_XCD=0|1 [VDIFF_WGRAD_ATOMIC=1] python tools/wgrad_ab.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd"))

import torch  # noqa: E402

from vdiff import _lib, ops  # noqa: E402

# (Ci, Co, k, H = W, T, launches per train step)
SHAPES = ((256, 256, 3, 32, 16, 10), (64, 64, 3, 128, 16, 7), (128, 128, 3, 64, 16, 6),
          (128, 64, 3, 128, 16, 2), (200, 64, 3, 128, 16, 1), (512, 256, 3, 32, 16, 2),
          (128, 128, 3, 128, 16, 1), (256, 256, 3, 64, 16, 1), (384, 128, 3, 64, 16, 1),
          (192, 64, 3, 128, 16, 1), (256, 128, 3, 64, 16, 1), (192, 128, 3, 64, 16, 1),
          (384, 256, 3, 32, 16, 1), (64, 128, 3, 64, 16, 1), (128, 256, 3, 32, 16, 1),
          (64, 8, 3, 128, 16, 1),
          (256, 768, 1, 128, 1, 6), (64, 192, 1, 512, 1, 5), (128, 384, 1, 256, 1, 5),
          (64, 64, 1, 512, 1, 5), (256, 256, 1, 128, 1, 6), (128, 128, 1, 256, 1, 5))


def main():
    atomic = os.environ.get("VDIFF_WGRAD_ATOMIC", "0") == "1"
    tag = f"xcd={os.environ.get('VDIFF_WGRAD_XCD', '1')} {'atomic' if atomic else 'det'}"
    tot3 = tot1 = 0.0
    worst = 0.0
    for Ci, Co, k, H, T, per in SHAPES:
        g = torch.Generator(device="cuda").manual_seed(Ci * 7 + Co + H)
        x = torch.randn(1, T, H, H, Ci, generator=g, device="cuda").bfloat16()
        dy = torch.randn(1, T, H, H, Co, generator=g, device="cuda").bfloat16()
        p = k // 2
        d = ops._desc(1, [T, H, H], Ci, [T, H, H], Co, [k] * 3 if k == 3 else [1, 1, 1],
                      [1, 1, 1], [p] * 3, ops._DT[torch.bfloat16])
        taps = k ** 3
        st = ops._stream(x)
        if atomic:
            dw = torch.zeros(Co, taps, Ci, dtype=torch.float32, device="cuda")

            def run():
                dw.zero_()
                _lib.call("vd_conv3d_bwd_weight", d, x.data_ptr(), dy.data_ptr(),
                          dw.data_ptr(), st)
        else:
            dw = torch.empty(Co, Ci, taps, dtype=torch.float32, device="cuda")
            ws = torch.empty(_lib.lib().vd_conv3d_bwd_weight_workspace_size(d),
                             dtype=torch.uint8, device="cuda")

            def run():
                _lib.call("vd_conv3d_bwd_weight_det", d, x.data_ptr(), dy.data_ptr(),
                          dw.data_ptr(), Co, Ci, ws.data_ptr(), ws.numel(), st)
        run()
        # reference: the fp32 parity-mode weight gradient (conv_wgrad_kernel, exact-fp32 MFMA;
        # torch-checked in tests/test_gpu_conv.py) on the same bf16 values, whole tensors
        xr, dyr = x.float().contiguous(), dy.float().contiguous()
        d32 = ops._desc(1, [T, H, H], Ci, [T, H, H], Co, [k] * 3 if k == 3 else [1, 1, 1],
                        [1, 1, 1], [p] * 3, ops._DT[torch.float32])
        ref = torch.zeros(Co, taps, Ci, dtype=torch.float32, device="cuda")
        _lib.call("vd_conv3d_bwd_weight", d32, xr.data_ptr(), dyr.data_ptr(), ref.data_ptr(), st)
        got = dw.permute(0, 2, 1) if not atomic else dw
        err = float((got - ref).norm() / ref.norm())
        worst = max(worst, err)
        del xr, dyr, ref
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
        tf = 2.0 * T * H * H * Co * taps * Ci / (us * 1e-6) / 1e12
        gbs = T * H * H * (Ci + Co) * 2 / (us * 1e-6) / 1e9
        if k == 3:
            tot3 += us * per
        else:
            tot1 += us * per
        print(f"[{tag}] wgrad k{k} {Ci:4d}->{Co:4d} at {T}x{H}x{H}: {us:7.1f} us {tf:7.1f} TF/s "
              f"{gbs:7.0f} GB/s  rel-L2 {err:.1e}", flush=True)
    print(f"[{tag}] per train step: 3x3x3 {tot3 / 1e3:.3f} ms + 1x1 {tot1 / 1e3:.3f} ms = "
          f"{(tot3 + tot1) / 1e3:.3f} ms (worst rel-L2 {worst:.1e})", flush=True)
    assert worst < 1e-2


if __name__ == "__main__":
    main()
