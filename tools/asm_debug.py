"""Diagnostics of the hand-scheduled attention kernels against the default kernels on one
small shape: per output (dQ, dK, dV) the non-finite count, the error on finite entries, and
where the bad entries sit (row mod 64 / 256, column, first bad rows).
    python tools/asm_debug.py [N] [seed]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd"))

import torch  # noqa: E402

from vdiff import ops  # noqa: E402


def grads(qkv, g, cfg):
    x = qkv.detach().clone().requires_grad_(True)
    with ops.attention_config(cfg):
        y = ops.attention(x, 1)
        y.backward(g)
    torch.cuda.synchronize()
    return x.grad.detach()[0].float().T  # [N, 3C]


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    gen = torch.Generator(device="cuda").manual_seed(seed)
    qkv = ops.to_cl((torch.randn((1, 192, N), generator=gen, device="cuda") * 1.3).bfloat16())
    g = ops.to_cl(torch.randn((1, 64, N), generator=gen, device="cuda").bfloat16())
    ref = grads(qkv, g, "auto")
    got = grads(qkv, g, "asm")
    for name, sl in (("dq", slice(0, 64)), ("dk", slice(64, 128)), ("dv", slice(128, 192))):
        a, b = ref[:, sl], got[:, sl]
        fin = torch.isfinite(b)
        bad = ~fin | ((a - b).abs() > 1e-2 * a.abs().max())
        print(f"{name}: nonfinite {int((~fin).sum())}/{b.numel()}, bad {int(bad.sum())}, "
              f"|ref| max {float(a.abs().max()):.3g}, |got| max(finite) "
              f"{float(b[fin].abs().max()) if fin.any() else float('nan'):.3g}, "
              f"zeros {int((b == 0).sum())}")
        if fin.all():
            print(f"   rel-L2 {float((a - b).norm() / a.norm()):.3e}")
        if bad.any():
            rows = bad.any(1).nonzero().flatten()
            cols = bad.any(0).nonzero().flatten()
            print(f"   bad rows {rows.numel()}: first {rows[:12].tolist()}; mod 64 "
                  f"{sorted(set((rows % 64).tolist()))[:16]}; //64 {sorted(set((rows // 64).tolist()))[:16]}")
            print(f"   bad cols {cols.tolist()[:64]}")
            r0 = int(rows[0])
            print(f"   row {r0} ref {a[r0, :8].tolist()}")
            print(f"   row {r0} got {b[r0, :8].tolist()}")


if __name__ == "__main__":
    main()
