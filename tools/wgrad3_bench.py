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


# (Ci, Co, pixels, launches per train step) -- the 1x1 weight gradients
SHAPES1 = ((64, 192, 262144, 5), (128, 384, 65536, 5), (256, 768, 16384, 6),
           (256, 256, 16384, 6), (64, 64, 262144, 5), (128, 128, 65536, 5),
           (128, 64, 262144, 2), (512, 256, 16384, 2), (192, 64, 262144, 1),
           (384, 128, 65536, 1), (256, 128, 65536, 1), (192, 128, 65536, 1),
           (384, 256, 16384, 1), (128, 256, 16384, 1), (64, 128, 65536, 1))


def main():
    """--det: the default deterministic path (vd_conv3d_bwd_weight_det: per-split partials +
    the ordered finish, dW in the torch layout), else the atomic one; --only CI,CO,H."""
    variant = os.environ.get("VDIFF_WGRAD3", "2,64")
    det = "--det" in sys.argv
    one = "--1x1" in sys.argv
    shapes = SHAPES1 if one else SHAPES
    if "--only" in sys.argv:
        want = tuple(int(v) for v in sys.argv[sys.argv.index("--only") + 1].split(","))
        shapes = [s for s in SHAPES if s[:3] == want]
    modes = [1]
    if "--modes" in sys.argv:
        modes = [int(v) for v in sys.argv[sys.argv.index("--modes") + 1].split(",")]
    totals = {}
    for mode in modes:
        _lib.lib().vd_conv_set_wgrad(mode)
        totals[mode] = _run_all(shapes, det, variant, mode, one)
    if len(modes) > 1:
        print("totals:", {m: round(t, 3) for m, t in totals.items()})


OUTS = {}


def _run_all(shapes, det, variant, mode, one=False):
    total, worst = 0.0, 0.0
    T = 16
    for Ci, Co, H, per in shapes:
        g = torch.Generator(device="cuda").manual_seed(Ci * 7 + Co + H)
        taps = 1 if one else 27
        if one:  # H = the pixel count
            x = torch.randn(1, 1, 1, H, Ci, generator=g, device="cuda").bfloat16()
            dy = torch.randn(1, 1, 1, H, Co, generator=g, device="cuda").bfloat16()
            d = ops._desc(1, [1, 1, H], Ci, [1, 1, H], Co, [1, 1, 1], [1, 1, 1], [0, 0, 0],
                          ops._DT[torch.bfloat16])
        else:
            x = torch.randn(1, T, H, H, Ci, generator=g, device="cuda").bfloat16()
            dy = torch.randn(1, T, H, H, Co, generator=g, device="cuda").bfloat16()
            d = ops._desc(1, [T, H, H], Ci, [T, H, H], Co, [3, 3, 3], [1, 1, 1], [1, 1, 1],
                          ops._DT[torch.bfloat16])
        dw = torch.zeros(Co, taps, Ci, dtype=torch.float32, device="cuda")
        st = ops._stream(x)
        if det:
            dwt = torch.empty(Co, Ci, taps, dtype=torch.float32, device="cuda")
            ws = torch.empty(_lib.lib().vd_conv3d_bwd_weight_workspace_size(d), dtype=torch.uint8,
                             device="cuda")

        def run():
            if det:
                _lib.call("vd_conv3d_bwd_weight_det", d, x.data_ptr(), dy.data_ptr(),
                          dwt.data_ptr(), Co, Ci, ws.data_ptr(), ws.numel(), st)
                dw.copy_(dwt.permute(0, 2, 1))
                return
            dw.zero_()
            _lib.call("vd_conv3d_bwd_weight", d, x.data_ptr(), dy.data_ptr(), dw.data_ptr(), st)

        run()
        if one:
            ref = (dy.reshape(-1, Co).float().T @ x.reshape(-1, Ci).float()).reshape(Co, 1, Ci)
        else:
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
            if det:  # the kernel pair alone, no layout copy
                _lib.call("vd_conv3d_bwd_weight_det", d, x.data_ptr(), dy.data_ptr(),
                          dwt.data_ptr(), Co, Ci, ws.data_ptr(), ws.numel(), st)
            else:
                run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        if not det:
            e0.record()
            for _ in range(reps):
                dw.zero_()
            e1.record()
            torch.cuda.synchronize()
            us -= e0.elapsed_time(e1) / reps * 1e3
        tf = 2.0 * (H if one else T * H * H) * Co * taps * Ci / (us * 1e-6) / 1e12
        total += us * per
        same = ""
        key = (Ci, Co, H, one)
        if key in OUTS:
            same = " bit-identical to the first mode" if torch.equal(OUTS[key], dw) else \
                " DIFFERS from the first mode"
        else:
            OUTS[key] = dw.clone()
        print(f"[{variant} m{mode}] wgrad {'1x1' if one else '3x3x3'} {Ci:4d}->{Co:4d} at "
              f"{H if one else f'{T}x{H}x{H}'}: {us:7.1f} us "
              f"{tf:7.1f} TF/s  rel-L2 {err:.1e}{same}", flush=True)
    print(f"[{variant} m{mode}] per train step: {total / 1e3:.3f} ms (worst rel-L2 {worst:.1e})",
          flush=True)
    assert worst < 1e-2
    return total / 1e3


if __name__ == "__main__":
    main()
