"""How often the forward's lagged-max rare path runs (GPU box, diagnostic build): one
workgroup of the hand-scheduled forward on an N-token sequence with a probe after the loop
that stores the rare-path counter (s79) and a few row statistics per lane.
    python tools/asm_rare_count.py [N] [scale]"""
import math
import os
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd", "csrc", "asm"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import gen_attn_asm as G  # noqa: E402
import gen_fwd as F  # noqa: E402
from asmgen import code_object_text  # noqa: E402
from asm_ab import hip, check, launch  # noqa: E402
import ctypes as C  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    sc = float(sys.argv[2]) if len(sys.argv) > 2 else 1.3
    V, _ = F.regs()
    regs = ["s79", V.r("m", 0), V.r("m", 1), V.r("l", 0), V.r("ps", 0)]
    kfw, _ = F.gen_fwd(probe=("loop", regs))
    kdq, ddq, _ = G.gen_dq()
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
    check(hip.hipModuleGetFunction(C.byref(fn), mod, b"vd_attn_fwd_d64"), "function")
    C3, D = 192, 64
    torch.manual_seed(0)
    qkv = (torch.randn(N, C3, device="cuda") * sc).bfloat16()
    o_ = torch.empty(N, D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(N, device="cuda", dtype=torch.float32)
    dbg = torch.zeros(256 * len(regs), dtype=torch.int32, device="cuda")
    niter = math.ceil(N / 512)
    ts_b = C3 * 2
    args = struct.pack("<5Q4I4Qf5IQ", qkv.data_ptr(), qkv.data_ptr() + 128, qkv.data_ptr() + 256,
                       o_.data_ptr(), lse.data_ptr(), N, ts_b, D * 2, 1, 0, 0, 0, 0,
                       (1 / math.sqrt(D)) * 1.4426950408889634, ((N - 1) * C3 + 64) * 2,
                       ((N - 1) * D + 64) * 2, 64 * ts_b, niter, N - 512 * (niter - 1),
                       dbg.data_ptr())
    launch(fn, args, (1, 1, 1))
    torch.cuda.synchronize()
    got = dbg.view(256, len(regs)).cpu()
    f = got.view(torch.float32)
    tiles = N // 64
    for w in range(4):
        ln = 64 * w
        print(f"wave {w}: rare-path calls {int(got[ln, 0])} of {tiles} tiles; m[0] lane0 "
              f"{float(f[ln, 1]):.3f} m[1] {float(f[ln, 2]):.3f} l[0] {float(f[ln, 3]):.3e} "
              f"ps[0] {float(f[ln, 4]):.3e}")
    # the true row max (log2 units) of the first queries, for comparison
    q = qkv[:4, :64].float() * (1 / math.sqrt(D)) * 1.4426950408889634
    k = qkv[:, 64:128].float()
    s = q @ k.T
    print("true max (log2) of queries 0..3:", [round(float(x), 3) for x in s.max(1).values])
    print("first-tile max of queries 0..3:", [round(float(x), 3) for x in s[:, :64].max(1).values])


if __name__ == "__main__":
    main()
