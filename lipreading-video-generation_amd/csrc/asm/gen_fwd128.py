"""vd_attn_fwd_d128: hand-scheduled gfx950 forward of the head_dim-128 joint attention
(reference QKVAttentionLegacy.forward, unet.py:349-366, at C = 128: softmax(Q K^T / sqrt(D))
V), the head_dim-64 kernel's algorithm (gen_fwd.py) with 32-key tiles: 4 waves x 64 queries
(2 query blocks j) per workgroup, ONE wave per SIMD, the whole 512-entry register file.

Per 32-key tile t a wave runs 32 v_mfma_f32_32x32x16_bf16 in body t:
    G(t-1) [16: O^T += V^T P^T over 4 output-dim blocks x 2 key k-steps x 2 j] |
    S(t+1) [16: S^T = K Q'^T - m over 8 dim k-steps x 2 j, one tile ahead]
and the softmax of tile t (32 v_exp_f32, 30 row-sum adds into 4 accumulators per query
block, 16 v_cvt_pk_bf16_f32) spread over the same 32 gaps by cost.  At D = 128 the MFMA
work per score doubles while the softmax does not, so the body is MFMA-bound where the
head_dim-64 body is issue-bound.  Registers: Q' (64) and the O^T accumulators (128) of the
wave's queries, the K row fragments of tile t+1 (32) and the V^T fragments of tile t (32) in
AGPRs; two S sets (one per tile parity), P^T, the -m splats and the softmax in VGPRs.

Lagged max and the rare path (a subroutine, s_swappc) as in gen_fwd.py.  Ring: 8 stages x
(K tile 8 KiB | V tile 8 KiB) = 128 KiB of LDS by LDS-DMA, tile t+4 issued in body t (2 + 2
pieces per wave), one barrier per body; stages 4..7 are addressed from +64 KiB copies of
the per-lane offsets.  An iteration is 8 bodies (256 keys); keys past the end are masked to
-inf only in the last iteration, its own copy of the 8 bodies.
"""
from __future__ import annotations

from asmgen import Regs, Stream, kernel_text

MFMA = "v_mfma_f32_32x32x16_bf16"
NW = 4
D = 128
TK = 32                # keys per tile
NST = 8                # ring stages
PD = 4                 # prefetch distance (tiles)
STAGE = 16384          # K tile | V tile (32 x 128 bf16 each)
VOFF = 8192
KARG = 112             # AsmFwdArgs (vd_asm.h); tile_bytes = 32 rows here
HI = 65536
NINF, PINF = "0xff800000", "0x7f800000"
CHECK_NOP = 3
CHAINS = 4
DMAS = 0               # LDS-DMA slots of a body (A/B): 0 {4,12,20,28} 1 {1,9,17,25} 2 {6,14,22,30}
KSLOT = 0              # first gap of the K(t+1) row reads (one per gap)

S_KARG = "s[0:1]"
S_WGX, S_WGY, S_WGZ = "s2", "s3", "s4"
RQ, RK, RV, RO, RL = "s[44:47]", "s[48:51]", "s[52:55]", "s[56:59]", "s[60:63]"
S_WAVE, S_Q0, S_M0, S_ITER, S_TAB = "s64", "s65", "s66", "s67", "s[68:69]"
S_ST, S_ST1, S_KB, S_RET, S_TGT = "s76", "s77", "s78", "s[80:81]", 82


def swz(r):
    """attention.hip swz_row<128>."""
    return ((r & 3) << 2) | ((r >> 2) & 3)


def toff_bytes(r, c):
    return 2 * (r * D + (((c >> 3) ^ swz(r)) << 3) + (c & 7))


def lane_table():
    """tab[wave][lane][32] u32: 0-7 K row-fragment offsets (k-step s), 8-15 V^T
    transposed-fragment offsets (2 i + hi), 16-17 DMA rows of the wave's 2 pieces of a
    32-row tile, 18-19 their source chunk * 16."""
    out = []
    for w in range(NW):
        for lane in range(64):
            r, hh = lane & 31, lane >> 5
            row = [toff_bytes(r, 16 * s + 8 * hh) for s in range(8)]
            g, fr = lane >> 4, lane & 15
            q4, p4 = fr >> 2, fr & 3
            tr = []
            for i in range(4):
                col = 32 * i + 16 * (g & 1) + 4 * p4
                kr = 4 * (g >> 1) + q4
                tr += [toff_bytes(kr, col), toff_bytes(kr + 8, col)]
            drow, dch = [], []
            for i in range(2):
                gi = w * 2 + i
                rr = gi * 4 + lane // 16
                drow.append(rr)
                dch.append(((lane % 16) ^ swz(rr)) * 16)
            out.append(row + tr + drow + dch + [0] * 12)
    return out


def regs():
    V, A = Regs("v"), Regs("a")
    for name, n in (("tid", 1), ("lane", 1), ("rowoff", 8), ("troff", 8), ("rowhi", 8),
                    ("trhi", 8), ("dma", 2), ("dmac", 2), ("tmp", 4), ("sto", 2), ("klim", 1),
                    ("ps", 2), ("l", 2), ("m", 2), ("ninf", 1), ("tc", 2), ("c", 8)):
        V.alloc(name, n)
    V.alloc("s0", 32, 16)    # S' of the even tiles, per query block j
    V.alloc("s1", 32)        # ... of the odd tiles
    V.alloc("p", 16)         # P^T as bf16 B operands [j][s2]
    V.alloc("negm", 32)      # -m splats per query block (srcC of the first S MFMA)
    A.alloc("qf", 64)        # Q' fragments [j][s]
    A.alloc("acc", 128)      # O^T accumulators [i][j]
    A.alloc("kf", 32)        # K row fragments [s] of tile t+1
    A.alloc("trf", 32)       # V^T fragments [i][s2] (lo 2 + hi 2) of tile t
    assert V.next <= 256 and A.next <= 256, (V.next, A.next)
    return V, A


def sblk(V, par, j):
    return V.r(f"s{par}", 16 * j, 16)


def lds(V, name, k, off):
    if off >= HI:
        return V.r({"rowoff": "rowhi", "troff": "trhi"}[name], k), off - HI
    return V.r(name, k), off


def k_reads(V, A, stage):
    out = []
    for s in range(8):
        b, off = lds(V, "rowoff", s, stage * STAGE)
        out.append((f"ds_read_b128 {A.r('kf', 4 * s, 4)}, {b} offset:{off}", ("K", s)))
    return out


def tr_reads(V, A, stage):
    out = []
    for i in range(4):
        for s2 in range(2):
            for hi in range(2):
                b, off = lds(V, "troff", 2 * i + hi, stage * STAGE + VOFF + s2 * 4096)
                out.append((f"ds_read_b64_tr_b16 {A.r('trf', 8 * i + 4 * s2 + 2 * hi, 2)}, "
                            f"{b} offset:{off}", ("T", i, s2, hi)))
    return out


def g_mfmas(V, A):
    out = []
    for i in range(4):
        for s2 in range(2):
            tr = A.r("trf", 8 * i + 4 * s2, 4)
            for j in range(2):
                acc = A.r("acc", 16 * (2 * i + j), 16)
                out.append((f"{MFMA} {acc}, {tr}, {V.r('p', 8 * j + 4 * s2, 4)}, {acc}", ()))
    return out


def s_mfmas(V, A, par, zero_c=False):
    out = []
    for s in range(8):
        for j in range(2):
            d = sblk(V, par, j)
            c = ("0" if zero_c else V.r("negm", 16 * j, 16)) if s == 0 else d
            out.append((f"{MFMA} {d}, {A.r('kf', 4 * s, 4)}, {A.r('qf', 32 * j + 4 * s, 4)}, "
                        f"{c}", (("K", s),)))
    return out


# ------------------------------------------------------------------ softmax stream
COST = {"exp": 8.0, "add": 4.0, "cvt": 4.5, "cmp": 4.0, "cnd": 4.0}


def softmax_list(V, par, masked, u):
    """[(text, cost, earliest gap)] of tile t's softmax: per score v_exp_f32, an add into one
    of CHAINS row-sum accumulators of its query block 4 scores behind, half a cvt; the cvt
    writing P^T[j][s2] waits for gap 16 + 2 s2 + j (G(t-1)'s last read of it is at gap
    12 + 2 s2 + j)."""
    out = []
    seq = [(j, r) for j in range(2) for r in range(16)]
    lag = 4
    for i in range(len(seq) + lag):
        if i < len(seq):
            j, r = seq[i]
            S = V[f"s{par}"] + 16 * j
            if r == 0 and masked:
                out += mask_list(V, S, u)
            out.append((f"v_exp_f32 v{S + r}, v{S + r}", COST["exp"], 0))
        if i >= lag:
            j, r = seq[i - lag]
            S = V[f"s{par}"] + 16 * j
            c = V.r("c", 4 * j + r % CHAINS)
            if r < CHAINS:
                out.append((f"v_mov_b32 {c}, v{S + r}", COST["add"], 0))
            else:
                out.append((f"v_add_f32 {c}, {c}, v{S + r}", COST["add"], 0))
            if r % 2:
                k = r // 2
                out.append((f"v_cvt_pk_bf16_f32 {V.r('p', 8 * j + k)}, v{S + r - 1}, v{S + r}",
                            COST["cvt"], 16 + 2 * (k // 4) + j))
    out += combine_list(V)
    return out


def combine_list(V):
    """The CHAINS row-sum accumulators of each query block into ps (a pairwise tree)."""
    out = []
    if CHAINS == 1:
        return [(f"v_mov_b32 {V.r('ps', j)}, {V.r('c', 4 * j)}", COST["add"], 0)
                for j in range(2)]
    step = 1
    while step < CHAINS:
        last = 2 * step >= CHAINS
        for a in range(0, CHAINS, 2 * step):
            for j in range(2):
                dst = V.r("ps", j) if last else V.r("c", 4 * j + a)
                out.append((f"v_add_f32 {dst}, {V.r('c', 4 * j + a)}, "
                            f"{V.r('c', 4 * j + a + step)}", COST["add"], 0))
        step *= 2
    return out


def mask_list(V, S, u):
    """Keys >= n to -inf in query block j's score block S (klim = keys left - 4 hh)."""
    out = []
    for r in range(16):
        c = TK * u + (r & 3) + 8 * (r >> 2)
        out.append((f"v_cmp_lt_i32 vcc, {c}, {V.r('klim')}", COST["cmp"], 0))
        out.append((f"v_cndmask_b32 v{S + r}, {V.r('ninf')}, v{S + r}, vcc", COST["cnd"], 0))
    return out


def place(items, ngaps):
    """Greedy list schedule by cost (gen_fwd.place)."""
    total = sum(c for _, c, _ in items)
    per = total / ngaps
    slots = [[] for _ in range(ngaps)]
    done = [False] * len(items)
    budget = 0.0
    for g in range(ngaps):
        budget += per
        last = g == ngaps - 1
        for k, (text, cost, early) in enumerate(items):
            if done[k] or early > g:
                continue
            if not last and cost > budget + 1e-9:
                break
            slots[g].append(text)
            budget -= cost
            done[k] = True
    assert all(done)
    return slots


# ------------------------------------------------------------------ prologue
def prologue(st: Stream, V, A):
    e, r = st.emit, st.raw
    r(f"s_load_dwordx16 s[16:31], {S_KARG}, 0x0")
    r(f"s_load_dwordx8 s[32:39], {S_KARG}, 0x40")
    r(f"s_load_dwordx4 s[40:43], {S_KARG}, 0x60")
    e(f"v_and_b32 {V.r('lane')}, 63, {V.r('tid')}")
    r(f"v_readfirstlane_b32 {S_WAVE}, {V.r('tid')}")
    r("s_nop 1")
    r(f"s_lshr_b32 {S_WAVE}, {S_WAVE}, 6")
    r("s_getpc_b64 s[68:69]")
    r("s_add_u32 s68, s68, vd_attn_fwd128_lanes@rel32@lo+4")
    r("s_addc_u32 s69, s69, vd_attn_fwd128_lanes@rel32@hi+12")
    r(f"s_getpc_b64 s[{S_TGT}:{S_TGT + 1}]")
    st.label(".Lfwd128_pc")
    for v in (3, 2, 1, 0):
        r(f"s_add_u32 s{S_TGT + 2 * v}, s{S_TGT}, .Lfwd128_rare{v}-.Lfwd128_pc")
        r(f"s_addc_u32 s{S_TGT + 2 * v + 1}, s{S_TGT + 1}, 0")
    r("s_waitcnt lgkmcnt(0)")
    r(f"s_mul_i32 s70, {S_WGZ}, s29")
    r(f"s_add_u32 s70, s70, {S_WGY}")

    def mad64(dlo, dhi, a, blo, bhi, t):
        r(f"s_mul_i32 {dlo}, {a}, {blo}")
        r(f"s_mul_hi_u32 {dhi}, {a}, {blo}")
        r(f"s_mul_i32 {t}, {a}, {bhi}")
        r(f"s_add_u32 {dhi}, {dhi}, {t}")

    mad64("s72", "s73", S_WGZ, "s30", "s31", "s71")
    mad64("s76", "s77", S_WGY, "s32", "s33", "s71")
    r("s_add_u32 s72, s72, s76")
    r("s_addc_u32 s73, s73, s77")
    mad64("s74", "s75", S_WGZ, "s34", "s35", "s71")
    mad64("s76", "s77", S_WGY, "s36", "s37", "s71")
    r("s_add_u32 s74, s74, s76")
    r("s_addc_u32 s75, s75, s77")

    def rsrc(dst, plo, phi, blo, bhi, nrec):
        d0 = int(dst[2:].split(":")[0])
        r(f"s_add_u32 s{d0}, {plo}, {blo}")
        r(f"s_addc_u32 s{d0 + 1}, {phi}, {bhi}")
        r(f"s_and_b32 s{d0 + 1}, s{d0 + 1}, 0xffff")
        r(f"s_mov_b32 s{d0 + 2}, {nrec}")
        r(f"s_mov_b32 s{d0 + 3}, 0x20000")

    rsrc(RQ, "s16", "s17", "s72", "s73", "s39")
    rsrc(RK, "s18", "s19", "s72", "s73", "s39")
    rsrc(RV, "s20", "s21", "s72", "s73", "s39")
    rsrc(RO, "s22", "s23", "s74", "s75", "s40")
    r("s_mul_i32 s76, s70, s26")
    r("s_mul_hi_u32 s77, s70, s26")
    r("s_lshl_b64 s[76:77], s[76:77], 2")
    r("s_lshl_b32 s71, s26, 2")
    rsrc(RL, "s24", "s25", "s76", "s77", "s71")
    # q0 = wgx * 256 + wave * 64 ; M0 base of this wave's DMA pieces = wave * 2048
    r(f"s_lshl_b32 {S_Q0}, {S_WGX}, 8")
    r(f"s_lshl_b32 s71, {S_WAVE}, 6")
    r(f"s_add_u32 {S_Q0}, {S_Q0}, s71")
    r(f"s_lshl_b32 {S_M0}, {S_WAVE}, 11")
    r(f"s_sub_u32 {S_ITER}, s42, 1")
    r("s_mov_b32 s79, 0")
    t0, t1 = V.r("tmp", 0), V.r("tmp", 1)
    e(f"v_lshlrev_b32 {t0}, 7, {V.r('tid')}")
    r(f"global_load_dwordx4 {V.r('rowoff', 0, 4)}, {t0}, {S_TAB}")
    r(f"global_load_dwordx4 {V.r('rowoff', 4, 4)}, {t0}, {S_TAB} offset:16")
    r(f"global_load_dwordx4 {V.r('troff', 0, 4)}, {t0}, {S_TAB} offset:32")
    r(f"global_load_dwordx4 {V.r('troff', 4, 4)}, {t0}, {S_TAB} offset:48")
    r(f"global_load_dwordx4 v[{V['dma']}:{V['dma'] + 3}], {t0}, {S_TAB} offset:64")
    # staging in the -m splat registers (Q is staged in s0 | s1)
    qrow = [V.r("negm", 0), V.r("negm", 1)]
    hh16, h8 = V.r("negm", 2), V.r("negm", 3)
    e(f"v_and_b32 {qrow[0]}, 31, {V.r('lane')}")
    e(f"v_add_u32 {qrow[0]}, {S_Q0}, {qrow[0]}")
    e(f"v_add_u32 {qrow[1]}, 32, {qrow[0]}")
    e(f"v_lshrrev_b32 {hh16}, 5, {V.r('lane')}")
    e(f"v_lshlrev_b32 {hh16}, 4, {hh16}")
    e(f"v_lshrrev_b32 {h8}, 1, {hh16}")
    qv = V["s0"]  # Q fragments staged in v[s0 .. s0 + 63] (s0 and s1 are adjacent)
    assert V["s1"] == qv + 32
    for j in range(2):
        vq = V.r("negm", 4 + j)
        e(f"v_mul_lo_u32 {vq}, {qrow[j]}, s27")
        e(f"v_add_u32 {vq}, {vq}, {hh16}")
        for s in range(8):
            w0 = qv + 32 * j + 4 * s
            r(f"buffer_load_dwordx4 v[{w0}:{w0 + 3}], {vq}, {RQ}, 0 offen offset:{32 * s}")
        e(f"v_mul_lo_u32 {V.r('sto', j)}, {qrow[j]}, s28")
        e(f"v_add_u32 {V.r('sto', j)}, {V.r('sto', j)}, {h8}")
    e(f"v_lshrrev_b32 {t1}, 2, {hh16}")
    e(f"v_sub_u32 {V.r('klim')}, s43, {t1}")
    r("s_waitcnt vmcnt(0)")
    for w in range(64):
        x = f"v{qv + w}"
        e(f"v_lshlrev_b32 {t0}, 16, {x}")
        e(f"v_and_b32 {t1}, 0xffff0000, {x}")
        e(f"v_mul_f32 {t0}, s38, {t0}")
        e(f"v_mul_f32 {t1}, s38, {t1}")
        e(f"v_cvt_pk_bf16_f32 {x}, {t0}, {t1}")
        e(f"v_accvgpr_write_b32 {A.r('qf', w)}, {x}")
    for k in range(8):
        e(f"v_add_u32 {V.r('rowhi', k)}, {HI:#x}, {V.r('rowoff', k)}")
        e(f"v_add_u32 {V.r('trhi', k)}, {HI:#x}, {V.r('troff', k)}")
    d0 = V["dma"]
    for i in range(2):
        e(f"v_mul_lo_u32 v{d0 + i}, v{d0 + i}, s27")
        e(f"v_add_u32 v{d0 + i}, v{d0 + i}, v{d0 + 2 + i}")
    # O = 0, l = 0, m = -inf (-m splat +inf), S'(0) = +inf (the first check fails),
    # G(-1) adds 0 (zero V^T fragments and P^T)
    for k in range(128):
        e(f"v_accvgpr_write_b32 {A.r('acc', k)}, 0")
    for k in range(32):
        e(f"v_accvgpr_write_b32 {A.r('trf', k)}, 0")
        e(f"v_mov_b32 {V.r('negm', k)}, {PINF}")
        e(f"v_mov_b32 {V.r('s0', k)}, {PINF}")
    for k in range(16):
        e(f"v_mov_b32 {V.r('p', k)}, 0")
    for j in range(2):
        e(f"v_mov_b32 {V.r('m', j)}, {NINF}")
        e(f"v_mov_b32 {V.r('l', j)}, 0")
        e(f"v_mov_b32 {V.r('ps', j)}, 0")
    e(f"v_mov_b32 {V.r('ninf')}, {NINF}")
    for t in range(PD):
        ops, adv = dma_ops(V, t)
        for m0, ld in ops:
            r(m0)
            r("s_nop 0")
            e(ld)
        for a in adv:
            e(a)


def dma_ops(V, stage):
    d0 = V["dma"]
    ops = []
    for x, rs in ((0, RK), (VOFF, RV)):
        for i in range(2):
            ops.append((f"s_add_u32 m0, {S_M0}, {stage * STAGE + x + i * 1024}",
                        f"buffer_load_dwordx4 v{d0 + i}, {rs}, 0 offen lds"))
    adv = [f"v_add_u32 v{d0 + i}, s41, v{d0 + i}" for i in range(2)]
    return ops, adv


# ------------------------------------------------------------------ one body
def emit_body(st: Stream, V, A, u, masked, tag):
    par = u % 2
    st.comment(f"---- body, stage {u}{' (masked)' if masked else ''}")
    st.raw(f"s_waitcnt vmcnt({(PD - 2) * 4}) lgkmcnt(0)")  # tile t+1 landed
    st.raw("s_barrier")
    st.flush_lds()
    mf = g_mfmas(V, A) + s_mfmas(V, A, 1 - par)
    nm = len(mf)
    reads = {}

    def put(slot0, lst, per):
        for k, item in enumerate(lst):
            reads.setdefault(slot0 + k // per, []).append(item)

    kst = (u + 1) % NST
    put(KSLOT, k_reads(V, A, kst), 1)  # K(t+1) rows: gaps 0..7, read by S(t+1) from gap 16
    put(16, tr_reads(V, A, u), 2)     # V(t)^T for G(t) in the next body: gaps 16..23
    ops, adv = dma_ops(V, (u + PD) % NST)
    dma_at = {g: i for i, g in enumerate(((4, 12, 20, 28), (1, 9, 17, 25), (6, 14, 22, 30))[DMAS])}
    valu = place(softmax_list(V, par, masked, u), nm)
    for g in range(nm):
        if g in dma_at:
            m0, ld = ops[dma_at[g]]
            st.raw(m0)
            st.raw("s_nop 0")
            st.emit(ld)
            if dma_at[g] == 3:
                for a in adv:
                    st.emit(a)
        for text, rid in reads.get(g, []):
            st.emit(text, lds_id=rid)
        for text in valu[g]:
            st.emit(text)
        text, deps = mf[g]
        st.emit(text, wait_lds=deps)
    tc = V.r("tc", 0)
    st.emit(f"v_max_f32 {tc}, {V.r('ps', 0)}, {V.r('ps', 1)}")
    st.emit(f"v_cmp_ngt_f32 vcc, 0x47800000, {tc}")
    st.raw(f"s_nop {CHECK_NOP}")
    st.raw(f"s_cbranch_vccz .Lfwd128_ok{tag}")
    st.raw(f"s_mov_b32 {S_ST}, {u * STAGE}")
    st.raw(f"s_mov_b32 {S_ST1}, {kst * STAGE}")
    st.raw(f"s_mov_b32 {S_KB}, {TK * u}")
    v = 2 * int(masked) + par
    st.raw(f"s_swappc_b64 {S_RET}, s[{S_TGT + 2 * v}:{S_TGT + 2 * v + 1}]")
    st.label(f".Lfwd128_ok{tag}")
    for j in range(2):
        st.emit(f"v_add_f32 {V.r('l', j)}, {V.r('l', j)}, {V.r('ps', j)}")


def emit_tail(st: Stream, V, A):
    st.comment("---- tail: G of the last tile")
    st.raw("s_waitcnt lgkmcnt(0)")
    st.flush_lds()
    for text, _ in g_mfmas(V, A):
        st.emit(text)


def epilogue(st: Stream, V, A):
    e = st.emit
    st.raw("s_waitcnt vmcnt(0)")
    t = [V["s0"] + k for k in range(8)]
    ad, lx, inv = V["s0"] + 8, V["s0"] + 10, V["s0"] + 12
    e(f"v_xor_b32 v{ad}, 32, {V.r('lane')}")
    e(f"v_lshlrev_b32 v{ad}, 2, v{ad}")
    for j in range(2):
        e(f"ds_bpermute_b32 v{lx + j}, v{ad}, {V.r('l', j)}")
    st.raw("s_waitcnt lgkmcnt(0)")
    for j in range(2):
        e(f"v_add_f32 {V.r('l', j)}, {V.r('l', j)}, v{lx + j}")
        e(f"v_rcp_f32 v{inv + j}, {V.r('l', j)}")
    for j in range(2):
        for i in range(4):
            for g in range(4):
                base = 16 * (2 * i + j) + 4 * g
                for k in range(4):
                    e(f"v_accvgpr_read_b32 v{t[k]}, {A.r('acc', base + k)}")
                for k in range(4):
                    e(f"v_mul_f32 v{t[k]}, v{inv + j}, v{t[k]}")
                e(f"v_cvt_pk_bf16_f32 v{t[4]}, v{t[0]}, v{t[1]}")
                e(f"v_cvt_pk_bf16_f32 v{t[5]}, v{t[2]}, v{t[3]}")
                e(f"buffer_store_dwordx2 v[{t[4]}:{t[5]}], {V.r('sto', j)}, {RO}, 0 offen "
                  f"offset:{64 * i + 16 * g}")
    for j in range(2):
        q, lg = V["s1"] + 2 * j, V["s1"] + 2 * j + 1
        e(f"v_and_b32 v{q}, 31, {V.r('lane')}")
        e(f"v_add_u32 v{q}, {S_Q0}, v{q}")
        if j:
            e(f"v_add_u32 v{q}, 32, v{q}")
        e(f"v_lshlrev_b32 v{q}, 2, v{q}")
        e(f"v_log_f32 v{lg}, {V.r('l', j)}")
        e(f"v_add_f32 v{lg}, {V.r('m', j)}, v{lg}")
        e(f"v_mul_f32 v{lg}, 0x3f317218, v{lg}")
        e(f"buffer_store_dword v{lg}, v{q}, {RL}, 0 offen")


# ------------------------------------------------------------------ the rare path
def rare_path(V, A, par, masked):
    """Subroutine .Lfwd128_rare{2 masked + par}: S_ST / S_ST1 = ring offsets of tiles t / t+1,
    S_KB = tile t's first key within the masked iteration; returns through S_RET."""
    st = Stream()
    e, r = st.emit, st.raw
    st.label(f".Lfwd128_rare{2 * int(masked) + par}")
    r("s_add_u32 s79, s79, 1")  # rare-path count (diagnostic probes only)
    r("s_nop 15")
    r("s_nop 15")
    r("s_waitcnt lgkmcnt(0)")

    def reads_from(sreg, ta):
        for s in range(8):
            e(f"v_add_u32 {ta[s]}, {sreg}, {V.r('rowoff', s)}")
        for s in range(8):
            e(f"ds_read_b128 {A.r('kf', 4 * s, 4)}, {ta[s]}", lds_id=("K", s))

    # P^T is rewritten below and the row-sum chains are idle here: address scratch
    reads_from(S_ST, [V.r("p", k) for k in range(8)])
    for text, deps in s_mfmas(V, A, par, zero_c=True):
        e(text, wait_lds=deps)
    st.flush_lds()
    r("s_nop 15")
    r("s_nop 15")
    if masked:
        vl = V.r("p", 0)
        e(f"v_subrev_u32 {vl}, {S_KB}, {V.r('klim')}")
        for rr in range(16):
            c = (rr & 3) + 8 * (rr >> 2)
            e(f"v_cmp_lt_i32 vcc, {c}, {vl}")
            for j in range(2):
                x = V[f"s{par}"] + 16 * j + rr
                e(f"v_cndmask_b32 v{x}, {V.r('ninf')}, v{x}, vcc")
    mx, oth, ad, alpha = V["p"] + 8, V["p"] + 10, V["p"] + 12, V["p"] + 14
    for j in range(2):
        R = [V[f"s{par}"] + 16 * j + k for k in range(16)]
        e(f"v_max3_f32 v{mx + j}, v{R[0]}, v{R[1]}, v{R[2]}")
        for k in range(3, 15, 2):
            e(f"v_max3_f32 v{mx + j}, v{mx + j}, v{R[k]}, v{R[k + 1]}")
        e(f"v_max_f32 v{mx + j}, v{mx + j}, v{R[15]}")
    e(f"v_xor_b32 v{ad}, 32, {V.r('lane')}")
    e(f"v_lshlrev_b32 v{ad}, 2, v{ad}")
    for j in range(2):
        e(f"ds_bpermute_b32 v{oth + j}, v{ad}, v{mx + j}")
    r("s_waitcnt lgkmcnt(0)")
    for j in range(2):
        m, l = V.r("m", j), V.r("l", j)
        e(f"v_max_f32 v{mx + j}, v{mx + j}, v{oth + j}")
        e(f"v_max_f32 v{mx + j}, {m}, v{mx + j}")                 # m_new
        e(f"v_sub_f32 v{alpha + j}, {m}, v{mx + j}")
        e(f"v_exp_f32 v{alpha + j}, v{alpha + j}")               # exp2(m - m_new)
        e(f"v_cmp_eq_f32 vcc, {m}, v{mx + j}")
        e(f"v_cndmask_b32 v{alpha + j}, v{alpha + j}, 1.0, vcc")
        e(f"v_mov_b32 {m}, v{mx + j}")
        e(f"v_mul_f32 {l}, v{alpha + j}, {l}")
        e(f"v_xor_b32 v{oth + j}, 0x80000000, v{mx + j}")
        for k in range(16):
            e(f"v_mov_b32 {V.r('negm', 16 * j + k)}, v{oth + j}")
        tmp = [V.r("tmp", k) for k in range(4)]
        for i in range(4):
            for g in range(4):
                base = 16 * (2 * i + j) + 4 * g
                for k in range(4):
                    e(f"v_accvgpr_read_b32 {tmp[k]}, {A.r('acc', base + k)}")
                for k in range(4):
                    e(f"v_mul_f32 {tmp[k]}, v{alpha + j}, {tmp[k]}")
                for k in range(4):
                    e(f"v_accvgpr_write_b32 {A.r('acc', base + k)}, {tmp[k]}")
    # tile t's softmax against m_new (m_new lives in p[8..9]: every subtraction first)
    for j in range(2):
        S = V[f"s{par}"] + 16 * j
        for k in range(16):
            e(f"v_sub_f32 v{S + k}, v{S + k}, v{mx + j}")
    for j in range(2):
        S = V[f"s{par}"] + 16 * j
        ps = V.r("ps", j)
        for k in range(8):
            a, b = S + 2 * k, S + 2 * k + 1
            e(f"v_exp_f32 v{a}, v{a}")
            e(f"v_exp_f32 v{b}, v{b}")
            if k == 0:
                e(f"v_add_f32 {ps}, v{a}, v{b}")
            else:
                e(f"v_add_f32 {ps}, {ps}, v{a}")
                e(f"v_add_f32 {ps}, {ps}, v{b}")
            e(f"v_cvt_pk_bf16_f32 {V.r('p', 8 * j + k)}, v{a}, v{b}")
    # S(t+1) against m_new
    reads_from(S_ST1, [V.r("c", k) for k in range(8)])
    for text, deps in s_mfmas(V, A, 1 - par):
        e(text, wait_lds=deps)
    st.flush_lds()
    r("s_nop 15")
    r("s_nop 15")
    r(f"s_setpc_b64 {S_RET}")
    return st


def gen_fwd128():
    V, A = regs()
    st = Stream()
    prologue(st, V, A)
    st.label(".Lfwd128_loop")
    for u in range(NST):
        emit_body(st, V, A, u, False, f"{u}")
    st.raw(f"s_sub_u32 {S_ITER}, {S_ITER}, 1")
    st.raw(f"s_cmp_lg_u32 {S_ITER}, 0")
    st.raw("s_cbranch_scc1 .Lfwd128_loop")
    for u in range(NST):
        emit_body(st, V, A, u, True, f"m{u}")
    emit_tail(st, V, A)
    epilogue(st, V, A)
    body = st.text() + "\ts_endpgm\n"
    for masked in (False, True):
        for par in range(2):
            body += rare_path(V, A, par, masked).text()
    k = kernel_text("vd_attn_fwd_d128", body, vgprs=V.next, agprs=A.next, sgprs=96,
                    lds_bytes=NST * STAGE, kernarg_bytes=KARG, wg_size=64 * NW)
    data = "\n.rodata\n.p2align 8\nvd_attn_fwd128_lanes:\n"
    for row in lane_table():
        data += "\t.long " + ", ".join(str(x) for x in row) + "\n"
    return k, data, st
