"""A/B timing of generator variants of the hand-scheduled head_dim-128 backward kernels
(csrc/asm/gen_d128.py: vd_attn_bwd_dq_d128, vd_attn_bwd_dkdv_d128) on the GPU box.  Each
variant is generated with the given module knobs, assembled, loaded with hipModuleLoadData
and timed with HIP events on one N = 65536 sequence; dQ / dK / dV are checked against the
library's default backward of the same inputs.
    python tools/asm_ab_bwd128.py 'name:KNOB=v,KNOB=v' ...
(knobs: START, DK_TR0, DK_ROW1, DK_TR1, DK_DMA0, DQ_START, DQ_KV0, DQ_TR0, DQ_KV1, DQ_TR1)"""
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

import gen_d128 as G  # noqa: E402
from asmgen import code_object_text  # noqa: E402

hip = C.CDLL("libamdhip64.so.7")


def check(e, what):
    if e != 0:
        raise RuntimeError(f"{what}: hip error {e}")


def build(knobs):
    saved = {k: getattr(G, k) for k in knobs}
    for k, v in knobs.items():
        setattr(G, k, v)
    try:
        kdk, ddk, _ = G.gen_dkdv128()
        kdq, _ = G.gen_dq128()
    finally:
        for k, v in saved.items():
            setattr(G, k, v)
    d = tempfile.mkdtemp()
    s, o, co = (os.path.join(d, x) for x in ("b.s", "b.o", "b.hsaco"))
    open(s, "w").write(code_object_text([kdk, kdq], ddk))
    subprocess.run(["/opt/rocm/llvm/bin/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa",
                    "-mcpu=gfx950", "-c", s, "-o", o], check=True)
    subprocess.run(["/opt/rocm/llvm/bin/ld.lld", "-shared", o, "-o", co], check=True)
    blob = open(co, "rb").read()
    mod = C.c_void_p()
    buf = C.create_string_buffer(blob, len(blob))
    check(hip.hipModuleLoadData(C.byref(mod), buf), "load")
    fns = []
    for name in (b"vd_attn_bwd_dq_d128", b"vd_attn_bwd_dkdv_d128"):
        fn = C.c_void_p()
        check(hip.hipModuleGetFunction(C.byref(fn), mod, name), "function")
        fns.append(fn)
    return fns, buf


def launch(fn, args: bytes, grid):
    a = C.create_string_buffer(args, len(args))
    size = C.c_size_t(len(args))
    extra = (C.c_void_p * 5)(C.c_void_p(1), C.cast(a, C.c_void_p), C.c_void_p(2),
                             C.cast(C.pointer(size), C.c_void_p), C.c_void_p(3))
    check(hip.hipModuleLaunchKernel(fn, grid[0], grid[1], grid[2], 256, 1, 1, 0, None, None,
                                    extra), "launch")


def main():
    from vdiff import ops
    N, D = 65536, 128
    C3 = 3 * D
    torch.manual_seed(0)
    qkv_t = (torch.randn(N, C3, device="cuda") * 1.3).bfloat16()
    dout_t = torch.randn(N, D, device="cuda").bfloat16()
    x = qkv_t.T.unsqueeze(0).detach().requires_grad_(True)           # [1, 384, N] channels-last
    y = ops.attention(x, 1)                                           # default kernels
    lse = y.grad_fn.saved_tensors[2].detach().reshape(N).float()
    y.backward(dout_t.T.unsqueeze(0))
    ref = x.grad[0].T.float()                                         # [N, 384]: dq | dk | dv
    o = y.detach()[0].T.contiguous()                                   # [N, 128]
    nlse2 = (-lse * 1.4426950408889634).contiguous()
    ndelta = (-(dout_t.float() * o.float()).sum(-1)).contiguous()
    grad = torch.zeros(N, C3, device="cuda", dtype=torch.bfloat16)   # dq | dk | dv, token-major
    ts_b, ots_b = C3 * 2, D * 2
    scale = 1 / math.sqrt(D)
    niter = math.ceil(math.ceil(N / 64) / 4)
    kv_bytes, o_bytes = ((N - 1) * C3 + D) * 2, ((N - 1) * D + D) * 2
    q0 = qkv_t.data_ptr()
    dq_args = struct.pack("<7Q4I4Q2f4I", q0, q0 + 2 * D, q0 + 4 * D, dout_t.data_ptr(),
                          nlse2.data_ptr(), ndelta.data_ptr(), grad.data_ptr(), N, ts_b, ots_b, 1,
                          0, 0, 0, 0, scale, scale * 1.4426950408889634, kv_bytes, o_bytes,
                          64 * ts_b, niter)
    dk_args = struct.pack("<8Q4I4Q2f6I", q0, q0 + 2 * D, q0 + 4 * D, dout_t.data_ptr(),
                          nlse2.data_ptr(), ndelta.data_ptr(), grad.data_ptr() + 2 * D,
                          grad.data_ptr() + 4 * D, N, ts_b, ots_b, 1, 0, 0, 0, 0, scale,
                          scale * 1.4426950408889634, kv_bytes, o_bytes, 64 * ts_b, 64 * ots_b,
                          niter, 0)
    assert len(dq_args) == 128 and len(dk_args) == 144
    fl_dq, fl_dk = 6 * N * N * D, 8 * N * N * D
    for spec in sys.argv[1:]:
        name, _, kv = spec.partition(":")
        knobs = {}
        for item in filter(None, kv.split(",")):
            k, v = item.split("=")
            knobs[k] = int(v)
        (fdq, fdk), keep = build(knobs)
        grad.zero_()
        launch(fdq, dq_args, (N // 128, 1, 1))
        launch(fdk, dk_args, (N // 128, 1, 1))
        torch.cuda.synchronize()
        g = grad.float()
        errs = [float((g[:, a:a + D] - ref[:, a:a + D]).norm() / ref[:, a:a + D].norm())
                for a in (0, D, 2 * D)]
        res = []
        for fn, args in ((fdq, dq_args), (fdk, dk_args)):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ts = []
            for _ in range(7):
                ev[0].record()
                launch(fn, args, (N // 128, 1, 1))
                ev[1].record()
                torch.cuda.synchronize()
                ts.append(ev[0].elapsed_time(ev[1]))
            ts.sort()
            res.append(ts[3])
        print(f"{name:10s} {knobs}  dQ {res[0]:.3f} ms ({fl_dq / res[0] / 1e9:.0f} TF/s)  "
              f"dK/dV {res[1]:.3f} ms ({fl_dk / res[1] / 1e9:.0f} TF/s)  unit {res[0] + res[1]:.3f} ms"
              f"  rel-L2 vs default dq/dk/dv {errs[0]:.1e} {errs[1]:.1e} {errs[2]:.1e}", flush=True)
        del keep


if __name__ == "__main__":
    main()
