"""Dump the fp32 key-split partials of the hand-scheduled head_dim-256 dQ
(vd_attn_bwd_dq_d256, VDIFF_ASM256_DQ_L caps the split) straight from the backward workspace
and compare each split with its fp32 reference, dQ_z = scale * dS[:, keys of z] K[keys of z]
(tools/asm256_debug.py, batch r04d: with the split on, rows r with r % 16 >= 12 come out
wrong).  Per split: rel-L2 over all rows, over the good / bad row classes, and for a few bad
(row, column) pairs the value found next to candidate sources (another row / column of the
reference, zero).   VDIFF_ASM256_DQ_L=1 python tools/asm256_dump.py [N]"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "lipreading-video-generation_amd"), ROOT]

import torch  # noqa: E402

C = 256


def main():
    from vdiff import _lib, ops
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    dev = "cuda"
    gen = torch.Generator(device=dev).manual_seed(3)
    qkv = (torch.randn((N, 3 * C), generator=gen, device=dev) * 1.3).bfloat16()
    dout = torch.randn((N, C), generator=gen, device=dev).bfloat16()
    (d, qo, ko, vo, oo), = ops._attn_desc(1, N, C, 1, C, "joint", None, ops._DT[torch.bfloat16],
                                          True)
    es = 2
    base = qkv.data_ptr()
    o = torch.empty((N, C), dtype=torch.bfloat16, device=dev)
    lse = torch.empty(N, dtype=torch.float32, device=dev)
    nws = _lib.lib().vd_attention_fwd_workspace_size(d)
    fws = torch.empty(max(1, nws), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    _lib.call("vd_attention_fwd_ws", d, base + qo * es, base + ko * es, base + vo * es,
              o.data_ptr(), lse.data_ptr(), fws.data_ptr(), nws, st)
    dqkv = torch.zeros((N, 3 * C), dtype=torch.bfloat16, device=dev)
    with ops.attention_config("asm"):
        nb = _lib.lib().vd_attention_bwd_workspace_size(d)
        ws = torch.zeros(nb, dtype=torch.uint8, device=dev)
        _lib.call("vd_attention_bwd_dq", d, base + qo * es, base + ko * es, base + vo * es,
                  o.data_ptr(), dout.data_ptr(), lse.data_ptr(), dqkv.data_ptr() + qo * es,
                  ws.data_ptr(), st)
    torch.cuda.synchronize()
    L = int(os.environ.get("VDIFF_ASM256_DQ_L", "2"))
    # the host's split rule (attention.hip dq256_lsplit / dq256_kps)
    wgs = -(-N // 128)
    l = 0
    while l < L and (wgs << l) < 256:
        S = 2 << l
        kps = -(-(-(-N // S)) // 128) * 128
        if (S - 1) * kps >= N:
            break
        l += 1
    S = 1 << l
    kps = -(-(-(-N // S)) // 128) * 128
    print(f"N {N} splits {S} kps {kps} ws {nb} B")
    f = ws.view(torch.float32)
    rows = N
    dq_off = 2 * rows + 64
    # fp32 reference
    q, k, v = (qkv[:, i * C:(i + 1) * C].float() for i in range(3))
    do = dout.float()
    scale = 1.0 / math.sqrt(C)
    s = (q @ k.T) * scale
    p = torch.softmax(s, -1)
    delta = (do * o.float()).sum(-1, keepdim=True)
    dp = do @ v.T
    ds = p * (dp - delta)
    dq_full = (ds @ k) * scale
    got = dqkv[:, :C].float()
    print(f"dq (summed) rel-L2 {float((got - dq_full).norm() / dq_full.norm()):.3e}")
    bad_rows = torch.tensor([r for r in range(N) if r % 16 >= 12], device=dev)
    good_rows = torch.tensor([r for r in range(N) if r % 16 < 12], device=dev)
    if S == 1:
        return 0
    parts = f[dq_off:dq_off + S * rows * C].view(S, rows, C)
    for z in range(S):
        ks = slice(z * kps, min(N, (z + 1) * kps))
        ref = (ds[:, ks] @ k[ks]) * scale
        pz = parts[z]
        rel = lambda a, b: float((a - b).norm() / b.norm().clamp_min(1e-30))  # noqa: E731
        print(f"split {z}: rel all {rel(pz, ref):.3e}  good rows {rel(pz[good_rows], ref[good_rows]):.3e}"
              f"  bad rows {rel(pz[bad_rows], ref[bad_rows]):.3e}  |pz| {float(pz.norm()):.3e} |ref| {float(ref.norm()):.3e}")
        # per-column error on bad rows: which dims are wrong?
        ce = (pz[bad_rows] - ref[bad_rows]).norm(dim=0) / ref[bad_rows].norm(dim=0).clamp_min(1e-30)
        badc = (ce > 1e-2).nonzero().flatten().tolist()
        print(f"  bad-row columns wrong: {len(badc)} e.g. {badc[:24]}")
        for r in (12, 13, 15, 28, 44, 60, 76):
            if r >= N:
                continue
            for c in (0, 1, 4, 8, 32, 255):
                val = float(pz[r, c])
                # candidate sources: same column of nearby rows, zero, the full dq
                cands = {f"ref[{rr},{c}]": float(ref[rr, c]) for rr in range(max(0, r - 16), min(N, r + 17))}
                best = min(cands.items(), key=lambda kv: abs(kv[1] - val))
                print(f"  z{z} row {r} col {c}: got {val:+.5e} ref {float(ref[r, c]):+.5e} "
                      f"closest {best[0]}={best[1]:+.5e} full-dq {float(dq_full[r, c]):+.5e}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
