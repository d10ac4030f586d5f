"""Head_dim-256 forward A/B: the hand-scheduled vd_attn_fwd_d256 (config "asm",
csrc/asm/gen_fwd256.py) against the compiled 4-wave forward (config "base", the round-4
default) at the config-2 UNet3D shape (joint attention, N = 16384 = 16 x 32 x 32, one head)
and a shorter one.  Per launch: HIP-event time over `--reps` launches on the launch stream,
TFLOP/s (4 N^2 D algorithmic) and the fraction of the 2.5 PF/s dense bf16 peak; the two
outputs are compared (rel-L2 of O, max |d lse|).
    python tools/fwd256_ab.py [--reps 30] [--n 16384,4096]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "lipreading-video-generation_amd"), ROOT]

import torch  # noqa: E402

C = 256
PEAK = 2.5e15


def run(qkv, cfg, reps):
    from vdiff import _lib, ops
    B, C3, N = qkv.shape
    (d, qo, ko, vo, oo), = ops._attn_desc(B, N, C, 1, C, "joint", None, ops._DT[qkv.dtype], True)
    out = ops.empty_cl([B, C, N], qkv.dtype, qkv.device)
    lse = torch.empty(d.nseq * d.seq_len, dtype=torch.float32, device=qkv.device)
    es, base = qkv.element_size(), qkv.data_ptr()
    with ops.attention_config(cfg):
        nws = _lib.lib().vd_attention_fwd_workspace_size(d)
        ws = torch.empty(max(1, nws), dtype=torch.uint8, device=qkv.device)
        st = torch.cuda.current_stream()

        def call():
            _lib.call("vd_attention_fwd_ws", d, base + qo * es, base + ko * es, base + vo * es,
                      out.data_ptr(), lse.data_ptr(), ws.data_ptr() if nws else None, nws,
                      st.cuda_stream)
        call()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            call()
        e1.record(st)
        torch.cuda.synchronize()
    return out, lse, e0.elapsed_time(e1) / reps, nws


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--n", default="16384,4096")
    ap.add_argument("--amp", type=float, default=1.0)
    a = ap.parse_args()
    from vdiff import ops
    for N in (int(x) for x in a.n.split(",")):
        gen = torch.Generator(device="cuda").manual_seed(N)
        qkv = ops.to_cl((torch.randn((1, 3 * C, N), generator=gen, device="cuda") * a.amp)
                        .bfloat16())
        res = {}
        for cfg in ("base", "asm", "base", "asm"):
            o, l, ms, nws = run(qkv, cfg, a.reps)
            fl = 4.0 * N * N * C
            res[cfg] = (o, l)
            print(f"fwd D=256 N={N} {cfg:5s}: {ms * 1e3:8.1f} us  {fl / ms / 1e9:7.1f} TF/s  "
                  f"frac {fl / ms / 1e-3 / PEAK:.3f}  ws {nws} B", flush=True)
        (o0, l0), (o1, l1) = res["base"], res["asm"]
        err = float((o1.float() - o0.float()).norm() / o0.float().norm())
        print(f"  asm vs base: O rel-L2 {err:.2e}  max|d lse| {float((l1 - l0).abs().max()):.2e}",
              flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
