"""A/B timing of generator variants of the hand-scheduled head_dim-256 forward (GPU box):
each variant is generated with the given csrc/asm/gen_fwd256.py knobs, assembled, loaded with
hipModuleLoadData and timed with HIP events on one N = 16384 sequence (the config-2 32x32 level,
joint attention), unsplit (128 workgroups) and with the product's 2-way key split (256
workgroups, fp32 partials; the combine is done in torch for the check, not timed).  Its output
is checked against the library's compiled forward (config "base").
    python tools/asm_ab256.py 'name:KNOB=v,KNOB=v' ...
(knobs: RD_AHEAD, TR_AHEAD, CHAINS, CHECK_NOP -- module globals of gen_fwd256.py)"""
import math
import os
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASM = os.path.join(ROOT, "lipreading-video-generation_amd", "csrc", "asm")
sys.path.insert(0, ASM)
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import gen_d256 as Q  # noqa: E402
import gen_fwd256 as F  # noqa: E402
from asm_ab import check, hip, launch  # noqa: E402
from asmgen import code_object_text  # noqa: E402
import ctypes as C  # noqa: E402


def build(knobs):
    saved = {k: getattr(F, k) for k in knobs}
    for k, v in knobs.items():
        setattr(F, k, v)
    try:
        kfw, _ = F.gen_fwd256()
    finally:
        for k, v in saved.items():
            setattr(F, k, v)
    kdq, ddq, _ = Q.gen_dq256()
    d = tempfile.mkdtemp()
    s, o, co = (os.path.join(d, x) for x in ("f.s", "f.o", "f.hsaco"))
    open(s, "w").write(code_object_text([kdq, kfw], ddq))
    subprocess.run(["/opt/rocm/llvm/bin/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa",
                    "-mcpu=gfx950", "-c", s, "-o", o], check=True)
    subprocess.run(["/opt/rocm/llvm/bin/ld.lld", "-shared", o, "-o", co], check=True)
    blob = open(co, "rb").read()
    mod, fn = C.c_void_p(), C.c_void_p()
    buf = C.create_string_buffer(blob, len(blob))
    check(hip.hipModuleLoadData(C.byref(mod), buf), "load")
    check(hip.hipModuleGetFunction(C.byref(fn), mod, b"vd_attn_fwd_d256"), "function")
    return fn, buf


def main():
    from vdiff import ops
    N, D = 16384, 256
    C3 = 3 * D
    torch.manual_seed(0)
    qkv_t = (torch.randn(N, C3, device="cuda") * 1.3).bfloat16()   # token-major
    qkv = qkv_t.T.unsqueeze(0)                                      # [1, 768, N] channels-last
    with ops.attention_config("base"):
        ref = ops.attention(qkv, 1)
    refo = ref[0].T.float()
    o = torch.empty(N, D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(N, device="cuda", dtype=torch.float32)
    S = 2
    part = torch.empty(S * N * (D + 2), device="cuda", dtype=torch.float32)
    ts_b, ots_b = C3 * 2, D * 2
    flops = 4 * N * N * D

    def args(lsplit):
        kps = -(-(-(-N // (1 << lsplit))) // 128) * 128
        base = struct.pack("<5Q4I4Qf5I", qkv_t.data_ptr(), qkv_t.data_ptr() + 2 * D,
                           qkv_t.data_ptr() + 4 * D, o.data_ptr(), lse.data_ptr(), N, ts_b,
                           ots_b, 1, 0, 0, 0, 0, (1 / math.sqrt(D)) * 1.4426950408889634,
                           ((N - 1) * C3 + D) * 2, ((N - 1) * D + D) * 2, 32 * ts_b, 0, 0)
        tail = struct.pack("<QIIQQI3I", part.data_ptr() if lsplit else 0, kps, lsplit, N * 1024,
                           (1 << lsplit) * N * 1024, N * 8, 0, 0, 0)
        return base + tail

    for spec in sys.argv[1:]:
        name, _, kv = spec.partition(":")
        knobs = {}
        for item in filter(None, kv.split(",")):
            k, v = item.split("=")
            knobs[k] = int(v)
        fn, keep = build(knobs)
        for lsplit in (0, 1):
            a = args(lsplit)
            grid = (N // 128, 1, 1 << lsplit)
            launch(fn, a, grid)
            torch.cuda.synchronize()
            if lsplit:
                po = part[:S * N * D].view(S, N, D)
                ml = part[S * N * D:].view(S, N, 2)
                M = ml[..., 0].max(0).values
                w = torch.exp2(ml[..., 0] - M)
                got = (w[..., None] * po).sum(0) / (w * ml[..., 1]).sum(0)[:, None]
            else:
                got = o.float()
            err = float((got - refo).norm() / refo.norm())
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ts = []
            for _ in range(7):
                ev[0].record()
                for _ in range(5):
                    launch(fn, a, grid)
                ev[1].record()
                torch.cuda.synchronize()
                ts.append(ev[0].elapsed_time(ev[1]) / 5)
            ts.sort()
            print(f"{name:12s} {knobs} split {1 << lsplit}: median {ts[3] * 1e3:.1f} us  "
                  f"min {ts[0] * 1e3:.1f} us  {flops / ts[3] / 1e9:.1f} TF/s  "
                  f"frac {flops / ts[3] / 1e-3 / 2.5e15:.3f}  rel-L2 vs base {err:.2e}",
                  flush=True)
        del keep


if __name__ == "__main__":
    main()
