"""Localise the head_dim-256 hand-scheduled backward failure of batch r04b (rel-L2 ~4 against
the compiled kernels whenever the key / query split was on): the asm dQ and dK/dV at each
split count (VDIFF_ASM256_DQ_L / VDIFF_ASM256_DKDV_L cap the split's log2), against the
compiled kernels ("base" dQ, "role" dK/dV), with the projection <asm, ref> / <ref, ref> and
the norm ratio (a scale error vs garbage).   python tools/asm256_debug.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "lipreading-video-generation_amd"), ROOT]

import torch  # noqa: E402

C = 256


def grads(qkv, g, cfg):
    from vdiff import ops
    x = qkv.detach().clone().requires_grad_(True)
    y = ops.attention(x, 1)
    with ops.attention_config(cfg):
        y.backward(g)
    torch.cuda.synchronize()
    return x.grad.detach().float()


def stats(a, r):
    a, r = a.flatten().double(), r.flatten().double()
    return {"rel": float((a - r).norm() / r.norm()), "proj": float(a @ r / (r @ r)),
            "norm_ratio": float(a.norm() / r.norm()),
            "zero_frac": float((a == 0).double().mean()),
            "rows_bad_frac": None}


def rows_bad(a, r, tol=1e-3):
    # fraction of token rows whose rel error exceeds tol (a, r: [C, N])
    e = (a - r).norm(dim=0) / r.norm(dim=0).clamp_min(1e-30)
    bad = (e > tol)
    idx = bad.nonzero().flatten()
    return float(bad.double().mean()), idx[:8].tolist(), idx[-8:].tolist()


def main():
    from vdiff import ops
    dev = "cuda"
    out = []
    for N, seed in ((4096, 1), (16384, 4), (1024, 0)):
        gen = torch.Generator(device=dev).manual_seed(seed)
        qkv = torch.randn((1, 3 * C, N), generator=gen, device=dev) * 1.3
        gout = torch.randn((1, C, N), generator=gen, device=dev)
        qkv, gout = ops.to_cl(qkv.bfloat16()), ops.to_cl(gout.bfloat16())
        ref_q = grads(qkv, gout, "base")[0]
        ref_kv = grads(qkv, gout, "role")[0]
        for L in (0, 1, 2):
            os.environ["VDIFF_ASM256_DQ_L"] = str(L)
            os.environ["VDIFF_ASM256_DKDV_L"] = "0"
            a = grads(qkv, gout, "asm")[0]
            s = stats(a[:C], ref_q[:C])
            s["rows_bad_frac"] = rows_bad(a[:C], ref_q[:C])
            rec = {"N": N, "what": "dq", "L": L, **s}
            print(json.dumps(rec), flush=True)
            out.append(rec)
        for L in (0, 1, 2, 3):
            os.environ["VDIFF_ASM256_DQ_L"] = "0"
            os.environ["VDIFF_ASM256_DKDV_L"] = str(L)
            a = grads(qkv, gout, "asm")[0]
            for name, sl in (("dk", slice(C, 2 * C)), ("dv", slice(2 * C, 3 * C))):
                s = stats(a[sl], ref_kv[sl])
                s["rows_bad_frac"] = rows_bad(a[sl], ref_kv[sl])
                rec = {"N": N, "what": name, "L": L, **s}
                print(json.dumps(rec), flush=True)
                out.append(rec)
    return 0


if __name__ == "__main__":
    sys.exit(main())
