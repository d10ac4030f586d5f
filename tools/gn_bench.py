"""GroupNorm(32)+SiLU forward and backward (vd_groupnorm_silu_fwd/_bwd through
ops.group_norm_silu) at the UNet3D 128x128x16 shapes, bf16, timed with HIP events; GB/s
counts the algorithmic bytes (fwd: x read twice + y written; bwd: x and dy read twice +
dx written)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd"))

import torch  # noqa: E402

from vdiff import ops  # noqa: E402

# (channels, frames, H = W)
SHAPES = ((64, 16, 128), (128, 16, 128), (192, 16, 128), (128, 16, 64), (256, 16, 64),
          (384, 16, 64), (256, 16, 32), (512, 16, 32), (768, 16, 32))


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def capi(C, T, H, reps=50):
    """GPU time of the C-ABI calls alone (back to back, no autograd): fwd, bwd in us."""
    from vdiff import _lib
    B, S, G = 1, T * H * H, 32
    x = torch.randn(B, S, C, device="cuda").bfloat16()
    dy = torch.randn(B, S, C, device="cuda").bfloat16()
    y, dx = torch.empty_like(x), torch.empty_like(x)
    g32 = torch.randn(C, device="cuda")
    b32 = torch.randn(C, device="cuda")
    mean = torch.empty(B * G, device="cuda")
    rstd = torch.empty_like(mean)
    dg, db = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    ws = torch.empty(_lib.lib().vd_groupnorm_workspace_size(B, S, C, G), dtype=torch.uint8,
                     device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    dt = ops._DT[torch.bfloat16]
    p = lambda t: t.data_ptr()  # noqa: E731

    def fwd():
        _lib.call("vd_groupnorm_silu_fwd", p(x), p(g32), p(b32), p(y), p(mean), p(rstd), B, S, C,
                  G, 1e-5, 1, 0.0, 0, dt, p(ws), st)

    def bwd():
        _lib.call("vd_groupnorm_silu_bwd", p(x), p(dy), p(g32), p(b32), p(mean), p(rstd), p(dx),
                  p(dg), p(db), B, S, C, G, 1, 0.0, 0, dt, p(ws), st)
    return timeit(fwd, reps), timeit(bwd, reps)


def main():
    if "--capi" in sys.argv:
        # --unroll 1,4: vd_groupnorm_set_unroll values, interleaved shape by shape in this process
        us = [1]
        if "--unroll" in sys.argv:
            us = [int(v) for v in sys.argv[sys.argv.index("--unroll") + 1].split(",")]
        from vdiff import _lib
        tot = {u: [0.0, 0.0] for u in us}
        for C, T, H in SHAPES:
            size = C * T * H * H * 2
            for u in us:
                _lib.lib().vd_groupnorm_set_unroll(u)
                f, b = capi(C, T, H)
                tot[u][0] += f
                tot[u][1] += b
                print(f"GN+SiLU C-ABI U={u} C={C:4d} {T}x{H}x{H}: fwd {f:7.1f} us "
                      f"({3 * size / f / 1e3:6.0f} GB/s)  bwd {b:7.1f} us "
                      f"({5 * size / b / 1e3:6.0f} GB/s)", flush=True)
        _lib.lib().vd_groupnorm_set_unroll(2)
        for u in us:
            print(f"U={u}: fwd {tot[u][0]:.1f} us, bwd {tot[u][1]:.1f} us over the shapes")
        return
    for C, T, H in SHAPES:
        x = ops.to_cl(torch.randn(1, C, T, H, H, device="cuda").bfloat16()).requires_grad_(True)
        w = torch.randn(C, device="cuda", requires_grad=True)
        b = torch.randn(C, device="cuda", requires_grad=True)
        g = ops.to_cl(torch.randn(1, C, T, H, H, device="cuda").bfloat16())
        size = x.numel() * 2
        fwd = timeit(lambda: ops.group_norm_silu(x.detach(), w.detach(), b.detach()))
        y = ops.group_norm_silu(x, w, b)

        def bwd():
            torch.autograd.grad(y, (x, w, b), g, retain_graph=True)

        full = timeit(bwd)
        print(f"GN+SiLU C={C:4d} {T}x{H}x{H}: fwd {fwd:7.1f} us ({3 * size / fwd / 1e3:6.0f} GB/s)"
              f"  bwd {full:7.1f} us ({5 * size / full / 1e3:6.0f} GB/s)", flush=True)


if __name__ == "__main__":
    main()
