"""Compare the cfg-sp backward against the default pipelines per gradient slice (dq, dk, dv)
at a few sequence lengths.  GPU box: python tools/sp_debug.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd"))
import torch  # noqa: E402

from vdiff import ops  # noqa: E402


def run(cfg, qkv, g):
    x = qkv.clone().requires_grad_(True)
    with ops.attention_config(cfg):
        out = ops.attention(x, 1)
        out.backward(g)
    torch.cuda.synchronize()
    return out.float(), x.grad.float()


for N in [int(a) for a in (sys.argv[1:] or ["1024", "1157", "4096"])]:
    C = 64
    torch.manual_seed(N)
    qkv = ops.to_cl(torch.randn(1, 3 * C, N, device="cuda").bfloat16())
    g = ops.to_cl(torch.randn(1, C, N, device="cuda").bfloat16())
    o0, g0 = run("p8", qkv, g)
    o1, g1 = run("sp", qkv, g)
    gr0, gr1 = g0[0].T.reshape(N, 3, C), g1[0].T.reshape(N, 3, C)  # logical [1, 3C, N]
    msg = []
    for i, nm in enumerate("qkv"):
        a, b = gr0[:, i], gr1[:, i]
        e = ((a - b).norm() / a.norm()).item()
        bad = ((a - b).abs() > 0.05 * a.abs().max()).any(dim=1).nonzero().flatten()
        msg.append(f"d{nm} {e:.2e} bad rows {bad.numel()} first {bad[:6].tolist()}")
    print(f"N={N}: out {((o0 - o1).norm() / o0.norm()).item():.2e} | " + " | ".join(msg), flush=True)
