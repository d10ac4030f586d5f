"""Register probes of the hand-scheduled dQ kernel (diagnostic builds, GPU box):
generate csrc/asm/gen_attn_asm.py with a probe point, assemble it, load it with
hipModuleLoadData and launch ONE workgroup on a small sequence; the probe stores the chosen
registers of every lane and ends the wave.  The values are compared with what the kernel
should hold at that point (lane tables, scaled Q fragments, row constants, dQ partials).
    python tools/asm_probe.py prologue|loop [N]"""
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

hip = C.CDLL("libamdhip64.so.7")  # the runtime torch loaded (same soname)


def check(e, what):
    if e != 0:
        raise RuntimeError(f"{what}: hip error {e}")


def build(probe):
    kdq, ddq, _ = G.gen_dq(probe)
    from asmgen import code_object_text
    d = tempfile.mkdtemp()
    s, o, co = (os.path.join(d, x) for x in ("p.s", "p.o", "p.hsaco"))
    open(s, "w").write(code_object_text([kdq], ddq))
    subprocess.run(["/opt/rocm/llvm/bin/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa",
                    "-mcpu=gfx950", "-c", s, "-o", o], check=True)
    subprocess.run(["/opt/rocm/llvm/bin/ld.lld", "-shared", o, "-o", co], check=True)
    return open(co, "rb").read()


def run(blob, args: bytes, grid):
    mod, fn = C.c_void_p(), C.c_void_p()
    buf = C.create_string_buffer(blob, len(blob))
    check(hip.hipModuleLoadData(C.byref(mod), buf), "load")
    check(hip.hipModuleGetFunction(C.byref(fn), mod, b"vd_attn_bwd_dq_d64"), "function")
    a = C.create_string_buffer(args, len(args))
    size = C.c_size_t(len(args))
    extra = (C.c_void_p * 5)(C.c_void_p(1), C.cast(a, C.c_void_p), C.c_void_p(2),
                             C.cast(C.pointer(size), C.c_void_p), C.c_void_p(3))
    check(hip.hipModuleLaunchKernel(fn, grid[0], grid[1], grid[2], 256, 1, 1, 0, None, None,
                                    extra), "launch")
    check(hip.hipDeviceSynchronize(), "sync")


def main():
    point = sys.argv[1] if len(sys.argv) > 1 else "prologue"
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    dev = "cuda"
    torch.manual_seed(0)
    C3, D = 192, 64
    qkv = (torch.randn(N, C3, device=dev) * 1.3).bfloat16()   # token-major: ts = 192
    dout = torch.randn(N, D, device=dev).bfloat16()
    q, k, v = qkv[:, :64].float(), qkv[:, 64:128].float(), qkv[:, 128:].float()
    scale = 1.0 / math.sqrt(D)
    s = (q @ k.T) * scale
    lse = torch.logsumexp(s, 1)
    o = torch.softmax(s, 1) @ v
    nlse2 = (-lse * 1.4426950408889634).contiguous()
    ndelta = (-(dout.float() * o.bfloat16().float()).sum(1)).contiguous()
    dq = torch.zeros(N, D, device=dev, dtype=torch.bfloat16)
    V, A = G.regs_dq()
    if point == "prologue":
        regs = ([f"v{V['rowoff'] + i}" for i in range(4)] + [f"v{V['troff'] + i}" for i in range(4)]
                + [f"v{V['dma'] + i}" for i in range(2)] + [f"v{V['stq'] + i}" for i in range(2)]
                + [f"a{A['qf'] + i}" for i in range(32)] + [f"a{A['of'] + i}" for i in range(4)]
                + [f"v{V['il']}", f"v{V['il'] + 16}", f"v{V['id']}", f"v{V['id'] + 16}"]
                + ["v0", "v1", "s2", "s3", "s4", "s84", "s85", "s86", "s30", "s31"])
    else:
        regs = [f"a{A['acc'] + i}" for i in range(64)]
    dbg = torch.zeros(256 * len(regs), dtype=torch.int32, device=dev)
    ts_b, ots_b = C3 * 2, D * 2
    kvb = ((N - 1) * C3 + 64) * 2
    ob = ((N - 1) * D + 64) * 2
    args = struct.pack("<7Q4I4Q2f4IQ", qkv.data_ptr(), qkv.data_ptr() + 128,
                       qkv.data_ptr() + 256, dout.data_ptr(), nlse2.data_ptr(), ndelta.data_ptr(),
                       dq.data_ptr(), N, ts_b, ots_b, 1, 0, 0, 0, 0, scale,
                       scale * 1.4426950408889634, kvb, ob, 64 * ts_b,
                       (N + 255) // 256, dbg.data_ptr())
    torch.cuda.synchronize()
    run(build((point, regs)), args, (1, 1, 1))
    got = dbg.view(256, len(regs)).cpu()
    tab = torch.tensor(G.lane_table(), dtype=torch.int64)  # [256][16]
    bad = 0

    def cmp(name, col, exp):
        nonlocal bad
        g = got[:, col].to(torch.int64) & 0xffffffff
        e = exp.to(torch.int64) & 0xffffffff
        nb = int((g != e).sum())
        bad += nb
        print(f"{name:10s} mismatches {nb:4d}/256" + (f"  e.g. lane {int((g != e).nonzero()[0])}: "
              f"got {int(g[(g != e).nonzero()[0]])} exp {int(e[(g != e).nonzero()[0]])}" if nb else ""))

    if point == "prologue":
        for i in range(4):
            cmp(f"rowoff{i}", i, tab[:, i])
            cmp(f"troff{i}", 4 + i, tab[:, 4 + i])
        for i in range(2):
            cmp(f"dma{i}", 8 + i, tab[:, 8 + i] * ts_b + tab[:, 10 + i] + 2 * 64 * ts_b)
        tid = torch.arange(256)
        lane, wave = tid % 64, tid // 64
        hh = lane // 32
        for j in range(2):
            qrow = wave * 64 + 32 * j + lane % 32
            cmp(f"stq{j}", 10 + j, qrow * ts_b + 8 * hh)
        # Q' fragments: bf16(Q * scale * log2 e), pairs per dword
        qs = (qkv[:, :64].float() * torch.tensor(scale * 1.4426950408889634,
                                                 dtype=torch.float32)).bfloat16()
        qbits = qs.view(torch.int16).to(torch.int64) & 0xffff
        for j in range(2):
            for s in range(4):
                for w in range(4):
                    qrow = (wave * 64 + 32 * j + lane % 32).clamp(max=N - 1)
                    e0 = 16 * s + 8 * hh + 2 * w
                    exp = qbits[qrow.cuda(), e0.cuda()].cpu() | (qbits[qrow.cuda(), (e0 + 1).cuda()].cpu() << 16)
                    cmp(f"qf{j}{s}{w}", 12 + 16 * j + 4 * s + w, exp)
        ob_bits = dout.view(torch.int16).to(torch.int64) & 0xffff
        for w in range(4):
            qrow = (wave * 64 + lane % 32).clamp(max=N - 1)
            e0 = 8 * hh + 2 * w
            exp = ob_bits[qrow.cuda(), e0.cuda()].cpu() | (ob_bits[qrow.cuda(), (e0 + 1).cuda()].cpu() << 16)
            cmp(f"of0{w}", 44 + w, exp)
        for j in range(2):
            qrow = (wave * 64 + 32 * j + lane % 32)
            cmp(f"il{j}", 48 + j, nlse2.cpu()[qrow].view(torch.int32))
            cmp(f"id{j}", 50 + j, ndelta.cpu()[qrow].view(torch.int32))
        for k, nm in enumerate(["v0", "v1", "s2", "s3", "s4", "s84", "s85", "s86", "s30", "s31"]):
            col = got[:, 52 + k]
            print(f"{nm:5s} lanes 0,64,128,192: {[int(col[x]) for x in (0, 64, 128, 192)]}")
    else:
        # dQ^T partial of workgroup 0 after all tiles: acc[i][j][r] = dQ[q][d] / scale with
        # q = 64 wave + 32 j + lane % 32, d = 32 i + acc_row(r, hh)
        ds = torch.softmax(s, 1) * ((dout.float() @ v.T) + ndelta[:, None])
        dqf = (ds.bfloat16().float() @ k.bfloat16().float()).cpu()
        f = got.view(torch.float32)
        print(f"non-finite partials: {int((~torch.isfinite(f)).sum())}/{f.numel()}, zeros "
              f"{int((f == 0).sum())}")
        tid = torch.arange(256)
        lane, wave = tid % 64, tid // 64
        hh = lane // 32
        err = 0.0
        for i in range(2):
            for j in range(2):
                for r in range(16):
                    qrow = wave * 64 + 32 * j + lane % 32
                    d = 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hh
                    e = dqf[qrow, d]
                    gv = f[:, 16 * (2 * i + j) + r]
                    d_ = float(((gv - e).abs() / (e.abs().max() + 1e-6)).max())
                    err = d_ if d_ != d_ else max(err, d_)  # NaN propagates
        print(f"dQ partial max rel err vs fp32 (bf16 dS): {err:.3e}")
        bad = int(err > 5e-2)
    print("PROBE", point, "OK" if bad == 0 else f"BAD ({bad})")


if __name__ == "__main__":
    main()
