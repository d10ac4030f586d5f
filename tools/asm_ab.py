"""A/B timing of generator variants of the hand-scheduled forward (GPU box): each variant is
generated with the given gen_fwd knobs, assembled, loaded with hipModuleLoadData and timed
with HIP events on one N = 262144 head_dim-64 sequence; its output is checked against the
library's default forward.   python tools/asm_ab.py 'name:KNOB=v,KNOB=v' ...
(knobs: PD, BAR2, CHECK_NOP -- module globals of csrc/asm/gen_fwd.py)"""
import ctypes as C
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

import torch  # noqa: E402

import gen_attn_asm as G  # noqa: E402
import gen_fwd as F64  # noqa: E402
import gen_fwd128 as F128  # noqa: E402
from asmgen import code_object_text  # noqa: E402

D128 = "--d128" in sys.argv  # the head_dim-128 forward (gen_fwd128 knobs), N = 65536
if D128:
    sys.argv.remove("--d128")
F = F128 if D128 else F64

hip = C.CDLL("libamdhip64.so.7")


def check(e, what):
    if e != 0:
        raise RuntimeError(f"{what}: hip error {e}")


def build(knobs):
    saved = {k: getattr(F, k) for k in knobs}
    for k, v in knobs.items():
        setattr(F, k, v)
    try:
        if D128:
            kfw, dfw, _ = F.gen_fwd128()
        else:
            kfw, _ = F.gen_fwd()
    finally:
        for k, v in saved.items():
            setattr(F, k, v)
    d = tempfile.mkdtemp()
    s, o, co = (os.path.join(d, x) for x in ("f.s", "f.o", "f.hsaco"))
    if D128:
        open(s, "w").write(code_object_text([kfw], dfw))
    else:
        kdq, ddq, _ = G.gen_dq()
        open(s, "w").write(code_object_text([kdq, kfw], ddq))
    subprocess.run(["/opt/rocm/llvm/bin/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa",
                    "-mcpu=gfx950", "-c", s, "-o", o], check=True)
    subprocess.run(["/opt/rocm/llvm/bin/ld.lld", "-shared", o, "-o", co], check=True)
    blob = open(co, "rb").read()
    mod, fn = C.c_void_p(), C.c_void_p()
    buf = C.create_string_buffer(blob, len(blob))
    check(hip.hipModuleLoadData(C.byref(mod), buf), "load")
    name = b"vd_attn_fwd_d128" if D128 else b"vd_attn_fwd_d64"
    check(hip.hipModuleGetFunction(C.byref(fn), mod, name), "function")
    return fn, buf


def launch(fn, args: bytes, grid):
    a = C.create_string_buffer(args, len(args))
    size = C.c_size_t(len(args))
    extra = (C.c_void_p * 5)(C.c_void_p(1), C.cast(a, C.c_void_p), C.c_void_p(2),
                             C.cast(C.pointer(size), C.c_void_p), C.c_void_p(3))
    check(hip.hipModuleLaunchKernel(fn, grid[0], grid[1], grid[2], 256, 1, 1, 0, None, None,
                                    extra), "launch")


def main():
    from vdiff import ops
    N, C3, D = (65536, 384, 128) if D128 else (262144, 192, 64)
    TR = 32 if D128 else 64  # keys per tile; 8 tiles per iteration
    torch.manual_seed(0)
    qkv_t = (torch.randn(N, C3, device="cuda") * 1.3).bfloat16()   # token-major
    qkv = qkv_t.T.unsqueeze(0)                                      # [1, 192, N] channels-last view
    ref = ops.attention(qkv, 1)                                     # [1, 64, N], default kernel
    refo = ref[0].T.float()
    o = torch.empty(N, D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(N, device="cuda", dtype=torch.float32)
    niter = math.ceil(N / (8 * TR))
    ts_b, ots_b = C3 * 2, D * 2
    args = struct.pack("<5Q4I4Qf5I", qkv_t.data_ptr(), qkv_t.data_ptr() + 2 * D,
                       qkv_t.data_ptr() + 4 * D, o.data_ptr(), lse.data_ptr(), N, ts_b, ots_b, 1,
                       0, 0, 0, 0, (1 / math.sqrt(D)) * 1.4426950408889634,
                       ((N - 1) * C3 + D) * 2, ((N - 1) * D + D) * 2, TR * ts_b, niter,
                       N - 8 * TR * (niter - 1))
    flops = 4 * N * N * D
    for spec in sys.argv[1:]:
        name, _, kv = spec.partition(":")
        knobs = {}
        for item in filter(None, kv.split(",")):
            k, v = item.split("=")
            knobs[k] = int(v)
        fn, keep = build(knobs)
        stamp = knobs.get("STAMP", 0)
        dbg = torch.zeros(N // 256 * 8, dtype=torch.int32, device="cuda")
        largs = args + (struct.pack("<Q", dbg.data_ptr()) if stamp else b"")
        args_v = largs
        launch(fn, args_v, (N // 256, 1, 1))
        torch.cuda.synchronize()
        err = float((o.float() - refo).norm() / refo.norm())
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ts = []
        for _ in range(5):
            ev[0].record()
            launch(fn, args_v, (N // 256, 1, 1))
            ev[1].record()
            torch.cuda.synchronize()
            ts.append(ev[0].elapsed_time(ev[1]))
        ts.sort()
        extra = ""
        if stamp:
            st = dbg.view(-1, 2).cpu().double()
            cyc, rt = st[:, 0], st[:, 1]
            extra = (f"  cycles/body {float(cyc.mean()) / (N // 64):.0f} (min wave "
                     f"{float(cyc.min()) / (N // 64):.0f}, max {float(cyc.max()) / (N // 64):.0f})"
                     f"  clock {float((cyc / (rt / 100e6)).mean()) / 1e9:.2f} GHz")
        print(f"{name:12s} {knobs}  median {ts[2]:.3f} ms  min {ts[0]:.3f} ms  "
              f"{flops / ts[2] / 1e9:.1f} TF/s  rel-L2 vs default {err:.2e}{extra}", flush=True)
        del keep


if __name__ == "__main__":
    main()
