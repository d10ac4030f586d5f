"""Time the 3x3x3 stride-1 conv forward and bwd-data launches of the UNet3D train step
(128x128x16, bf16) through the C-ABI with HIP events, per shape and per kernel choice.

    python tools/conv3_bench.py [--modes 2,3] [--dir fwd|bwd|both] [--only CI,CO,H] [--reps 20]
                                [--check]

--modes: values for vd_conv_set_halo (0 gathered tiles, 1 halo everywhere, 2 the default
selection, >= 3 experimental kernels), interleaved round by round in ONE process (rule 24).
Prints per shape the median microseconds and TFLOP/s of each mode, the per-step total
(launch counts of the train step's forward), and the max relative difference of each mode's
output against the first mode's.  --check also compares the first mode with torch's fp32
conv3d on a shape subset."""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd"))

import torch  # noqa: E402

from vdiff import _lib, ops  # noqa: E402

# (Ci, Co, H = W, launches per train-step forward); T = 16 frames (tools/wgrad3_bench.py)
SHAPES = ((64, 64, 128, 7), (128, 128, 64, 6), (256, 256, 32, 10), (128, 64, 128, 2),
          (200, 64, 128, 1), (512, 256, 32, 2), (256, 256, 64, 1), (384, 128, 64, 1),
          (192, 64, 128, 1), (256, 128, 64, 1), (192, 128, 64, 1), (384, 256, 32, 1),
          (64, 128, 64, 1), (128, 256, 32, 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="2")
    ap.add_argument("--dir", default="both", choices=["fwd", "bwd", "both"])
    ap.add_argument("--only", default=None)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--T", type=int, default=16)
    ap.add_argument("--cold", action="store_true",
                    help="flush L2 / Infinity Cache (a 1 GiB fill) before every timed launch and "
                         "time launches one by one (the in-model state: inputs not re-read)")
    ap.add_argument("--epilogue", action="store_true",
                    help="forward with bias + per-(b, co) add + residual, as a ResBlock conv")
    a = ap.parse_args()
    modes = [int(m) for m in a.modes.split(",")]
    lib = _lib.lib()
    T = a.T
    shapes = SHAPES
    if a.only:
        want = tuple(int(v) for v in a.only.split(","))
        shapes = [s for s in SHAPES if s[:3] == want] or [want + (1,)]
    dirs = ["fwd", "bwd"] if a.dir == "both" else [a.dir]
    tot = {(d, m): 0.0 for d in dirs for m in modes}
    dt = ops._DT[torch.bfloat16]
    flush = torch.empty(1 << 28, dtype=torch.float32, device="cuda") if a.cold else None
    for Ci, Co, H, per in shapes:
        g = torch.Generator(device="cuda").manual_seed(Ci * 7 + Co + H)
        x = (torch.rand(1, T, H, H, Ci, generator=g, device="cuda") * 2 - 1).bfloat16()
        dy = (torch.rand(1, T, H, H, Co, generator=g, device="cuda") * 2 - 1).bfloat16()
        w = torch.randn(Co, Ci, 3, 3, 3, generator=g, device="cuda") / (27 * Ci) ** 0.5
        wf = ops._pack_weight_now(w, Co, Ci, 27, Ci, Co, False, torch.bfloat16)
        wb = ops._pack_weight_now(w, Co, Ci, 27, Ci, Co, True, torch.bfloat16)
        d = ops._desc(1, [T, H, H], Ci, [T, H, H], Co, [3, 3, 3], [1, 1, 1], [1, 1, 1], dt)
        st = ops._stream(x)
        y = torch.empty(1, T, H, H, Co, dtype=torch.bfloat16, device="cuda")
        dx = torch.empty(1, T, H, H, Ci, dtype=torch.bfloat16, device="cuda")
        flop = 2.0 * T * H * H * Co * 27 * Ci
        bias = torch.randn(Co, generator=g, device="cuda") if a.epilogue else None
        ca = torch.randn(1, Co, generator=g, device="cuda") if a.epilogue else None
        res = torch.randn(1, T, H, H, Co, generator=g, device="cuda").bfloat16() if a.epilogue \
            else None
        ptr = lambda t: None if t is None else t.data_ptr()
        runs = {
            "fwd": lambda: _lib.call("vd_conv3d_fwd", d, x.data_ptr(), wf.data_ptr(), ptr(bias),
                                     ptr(ca), ptr(res), y.data_ptr(), st),
            "bwd": lambda: _lib.call("vd_conv3d_bwd_data", d, dy.data_ptr(), wb.data_ptr(),
                                     dx.data_ptr(), st)}
        outs = {"fwd": y, "bwd": dx}
        for dname in dirs:
            times = {m: [] for m in modes}
            ref = {}
            for r in range(a.rounds):
                for m in modes:
                    lib.vd_conv_set_halo(m)
                    runs[dname]()
                    torch.cuda.synchronize()
                    if r == 0:
                        ref[m] = outs[dname].float().clone()
                    if a.cold:
                        ts = []
                        for _ in range(a.reps):
                            flush.fill_(1.0)
                            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                            ev[0].record()
                            runs[dname]()
                            ev[1].record()
                            torch.cuda.synchronize()
                            ts.append(ev[0].elapsed_time(ev[1]) * 1e3)
                        times[m].append(statistics.median(ts))
                        continue
                    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                    ev[0].record()
                    for _ in range(a.reps):
                        runs[dname]()
                    ev[1].record()
                    torch.cuda.synchronize()
                    times[m].append(ev[0].elapsed_time(ev[1]) / a.reps * 1e3)
            m0 = modes[0]
            cells = []
            for m in modes:
                us = statistics.median(times[m])
                tot[(dname, m)] += us * per
                diff = float((ref[m] - ref[m0]).abs().max() / ref[m0].abs().max())
                cells.append(f"m{m} {us:8.1f} us {flop / us / 1e6:7.1f} TF/s d{diff:.1e}")
            print(f"{dname} {Ci:4d}->{Co:<4d} {H:4d}^2 x{per:<3d} " + " | ".join(cells), flush=True)
            if a.check and dname == "fwd" and Ci * Co * H <= 64 * 64 * 128:
                xr = x.float().permute(0, 4, 1, 2, 3)
                yr = torch.nn.functional.conv3d(xr, w, padding=1).permute(0, 2, 3, 4, 1)
                err = float((ref[m0] - yr).norm() / yr.norm())
                print(f"   check vs torch fp32 conv3d: rel-L2 {err:.2e}", flush=True)
    lib.vd_conv_set_halo(2)
    for (dname, m), v in tot.items():
        print(f"total {dname} mode {m}: {v / 1e3:.3f} ms per train-step forward pass")


if __name__ == "__main__":
    main()
