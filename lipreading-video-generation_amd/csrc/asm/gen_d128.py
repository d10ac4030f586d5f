"""Hand-scheduled gfx950 head_dim-128 attention backward (reference QKVAttentionLegacy,
unet.py:349-366, at C = 128: the 64x64 level of the config-2 UNet3D).

vd_attn_bwd_dkdv_d128 -- dK / dV of one key block: the arithmetic of the head_dim-64 kernel
(gen_attn_asm.py; attention.hip attn_bwd_dkdv_pipe_kernel: S' = Q K'^T - lse', dP = dO V^T -
delta with the query on the accumulator rows and the key on the lane, dV^T += dO^T P,
dK^T += Q^T dS, K' = K * scale * log2 e in bf16) at ONE wave per SIMD with 32 keys per wave
(4 waves, 128 keys per workgroup): the K' / V fragments of the wave's keys (64 registers)
and its full-width dK^T / dV^T accumulators (128) stay in AGPRs with the current query
block's row fragments; the VGPRs hold the score blocks, the transposed G operands and the
softmax.  Per 64-query tile (2 query blocks qb) a wave runs 64 v_mfma_f32_32x32x16_bf16 in
the order
    S/dP(t, qb0) [16] | G(t-1, qb1) [16] | S/dP(t, qb1) [16] | barrier | G(t, qb0) [16]
(G = 8 dV + 8 dK products: 4 output-dim blocks x 2 query k-steps), 96 VALU instructions (32
v_exp_f32, 32 v_mul_f32, 32 v_cvt_pk_bf16_f32) placed at a constant rate from gap START, 112
LDS fragment reads (48 ds_read_b128, 64 ds_read_b64_tr_b16) and 9 LDS-DMA pieces.

LDS: the row constants (-lse', -delta: 4 x 768 B, as the D = 64 kernel) then a 4-stage ring
of (Q tile 16 KiB | dO tile 16 KiB) = 131 KiB, tile t + 3 issued after the barrier of tile
t.  ds_read immediates are 16 bits, so stages 2 and 3 are addressed from +64 KiB copies of
the per-lane offsets.  The 128-element rows use attention.hip's swz_row<128> chunk XOR.
"""
from __future__ import annotations

from asmgen import Regs, Stream, kernel_text

MFMA = "v_mfma_f32_32x32x16_bf16"
NW = 4
D = 128
KPW = 32                # keys per wave
STAGE = 32768           # Q tile | dO tile (64 x 128 bf16 each)
OOFF = 16384
RC = 768                # per stage: lse' (256 B) | delta (256 B) | junk (256 B)
RC_BYTES = 4 * RC
NST = 4
KARG = 144              # AsmDkdvArgs (vd_asm.h)
START = 17
HI = 65536
# read / DMA placement knobs (A/B, tools/asm_ab_bwd128.py): first gap of each read group
DK_TR0, DK_ROW1, DK_TR1 = 1, 18, 32
DK_DMA0 = 49

# SGPRs (kernel arguments in s[16:51], see gen_attn_asm.py dK/dV map)
S_KARG = "s[0:1]"
S_WGX, S_WGY, S_WGZ = "s2", "s3", "s4"
RQ, RK, RV, RO, RL, RD, RDK, RDV = ("s[60:63]", "s[64:67]", "s[68:71]", "s[72:75]",
                                    "s[76:79]", "s[80:83]", "s[84:87]", "s[88:91]")
S_WAVE, S_K0, S_M0, S_ITER, S_RCM0 = "s92", "s93", "s94", "s95", "s98"
RRC = "s[56:59]"


def swz(r):
    """attention.hip swz_row<128>."""
    return ((r & 3) << 2) | ((r >> 2) & 3)


def toff_bytes(r, c):
    """attention.hip toff<bf16, 128>(r, c) in bytes."""
    return 2 * (r * D + (((c >> 3) ^ swz(r)) << 3) + (c & 7))


def lane_table():
    """tab[wave][lane][32] u32: 0-7 row-fragment offsets (k-step s, block row 0), 8-15 the
    transposed-fragment offsets (2 i + hi: output-dim block i, rows +8 hi), 16-19 the DMA
    rows of the wave's 4 pieces of a tile, 20-23 their source chunk * 16, 24 the
    row-constant read base (16 hh)."""
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
            for i in range(4):
                gi = w * 4 + i
                rr = gi * 4 + lane // 16
                drow.append(rr)
                dch.append(((lane % 16) ^ swz(rr)) * 16)
            out.append(row + tr + drow + dch + [16 * hh] + [0] * 7)
    return out


def regs():
    V, A = Regs("v"), Regs("a")
    for name, n in (("tid", 1), ("lane", 1), ("rowoff", 8), ("troff", 8), ("rowhi", 8),
                    ("trhi", 8), ("dmaq", 4), ("dmao", 4), ("rcv", 1), ("rcoff", 1),
                    ("tmp", 4), ("stk", 1), ("tmp2", 2)):
        V.alloc(name, n)
    V.alloc("s", 32, 16)     # S' blocks [qb]
    V.alloc("dp", 32)        # dP blocks [qb]
    V.alloc("pp", 16)        # P as bf16 B operands [qb] x 8
    V.alloc("ds", 16)        # dS as bf16 B operands
    V.alloc("il", 16)        # -lse' of the current query block's rows (srcC of S)
    V.alloc("id", 16)        # -delta (srcC of dP)
    V.alloc("otr", 32)       # dO^T fragments of the G block [i][s2] (lo 2 + hi 2)
    V.alloc("qtr", 32)       # Q^T fragments
    A.alloc("kf", 32)        # K' fragments [s]
    A.alloc("vf", 32)        # V fragments [s]
    A.alloc("adk", 64)       # dK^T accumulators [i]
    A.alloc("adv", 64)       # dV^T accumulators [i]
    A.alloc("qrow", 32)      # Q row fragments of the current query block [s]
    A.alloc("orow", 32)      # dO row fragments [s]
    assert V.next <= 256 and A.next <= 256, (V.next, A.next)
    return V, A


def lds(V, name, k, off):
    """(base register, immediate) of LDS byte offset `off` from per-lane table entry k."""
    if off >= HI:
        return V.r({"rowoff": "rowhi", "troff": "trhi"}[name], k), off - HI
    return V.r(name, k), off


def row_reads(V, A, stage, qb):
    """Fragment reads of query block qb of the tile in `stage`: -lse' / -delta of the
    block's rows first (the first S / dP products need them), then the Q and dO rows."""
    out = []
    for g in range(4):
        rc = stage * RC + qb * 128 + 32 * g
        out.append((f"ds_read_b128 {V.r('il', 4 * g, 4)}, {V.r('rcoff')} offset:{rc}", ("L", g)))
        out.append((f"ds_read_b128 {V.r('id', 4 * g, 4)}, {V.r('rcoff')} offset:{rc + 256}",
                    ("D", g)))
    tq = RC_BYTES + stage * STAGE + qb * 8192
    for s in range(8):
        b, off = lds(V, "rowoff", s, tq)
        out.append((f"ds_read_b128 {A.r('qrow', 4 * s, 4)}, {b} offset:{off}", ("Q", s)))
        b, off = lds(V, "rowoff", s, tq + OOFF)
        out.append((f"ds_read_b128 {A.r('orow', 4 * s, 4)}, {b} offset:{off}", ("O", s)))
    return out


def tr_reads(V, A, stage, qb):
    out = []
    tq = RC_BYTES + stage * STAGE + qb * 8192
    for i in range(4):
        for s2 in range(2):
            for hi in range(2):
                for x, name in ((OOFF, "otr"), (0, "qtr")):
                    b, off = lds(V, "troff", 2 * i + hi, tq + x + s2 * 4096)
                    out.append((f"ds_read_b64_tr_b16 {V.r(name, 8 * i + 4 * s2 + 2 * hi, 2)}, "
                                f"{b} offset:{off}", (name, i, s2, hi)))
    return out


def sdp(V, A, qb):
    out = []
    sv, dv = V.r("s", 16 * qb, 16), V.r("dp", 16 * qb, 16)
    for s in range(8):
        cs = V.r("il", 0, 16) if s == 0 else sv
        cd = V.r("id", 0, 16) if s == 0 else dv
        out.append((f"{MFMA} {sv}, {A.r('qrow', 4 * s, 4)}, {A.r('kf', 4 * s, 4)}, {cs}",
                    (("Q", s),) + (tuple(("L", g) for g in range(4)) if s == 0 else ())))
        out.append((f"{MFMA} {dv}, {A.r('orow', 4 * s, 4)}, {A.r('vf', 4 * s, 4)}, {cd}",
                    (("O", s),) + (tuple(("D", g) for g in range(4)) if s == 0 else ())))
    return out


def gmm(V, A, qb):
    out = []
    for i in range(4):
        acc = A.r("adv", 16 * i, 16)
        for s2 in range(2):
            out.append((f"{MFMA} {acc}, {V.r('otr', 8 * i + 4 * s2, 4)}, "
                        f"{V.r('pp', 8 * qb + 4 * s2, 4)}, {acc}",
                        tuple(("otr", i, s2, h) for h in range(2))))
        acc = A.r("adk", 16 * i, 16)
        for s2 in range(2):
            out.append((f"{MFMA} {acc}, {V.r('qtr', 8 * i + 4 * s2, 4)}, "
                        f"{V.r('ds', 8 * qb + 4 * s2, 4)}, {acc}",
                        tuple(("qtr", i, s2, h) for h in range(2))))
    return out


def valu(V):
    out = []
    for qb in range(2):
        S, Dp = V["s"] + 16 * qb, V["dp"] + 16 * qb
        P, G = V["pp"] + 8 * qb, V["ds"] + 8 * qb
        for k in range(8):
            a, c = 2 * k, 2 * k + 1
            out += [f"v_exp_f32 v{S + a}, v{S + a}", f"v_exp_f32 v{S + c}, v{S + c}",
                    f"v_mul_f32 v{Dp + a}, v{Dp + a}, v{S + a}",
                    f"v_mul_f32 v{Dp + c}, v{Dp + c}, v{S + c}",
                    f"v_cvt_pk_bf16_f32 v{P + k}, v{S + a}, v{S + c}",
                    f"v_cvt_pk_bf16_f32 v{G + k}, v{Dp + a}, v{Dp + c}"]
    return out


def dma_ops(V, stage):
    """The wave's 9 DMA ops of one tile into `stage` (4 Q pieces, 4 dO pieces, its
    row-constant piece) and the source-offset advances."""
    ops = []
    for x, (rs, nm) in enumerate(((RQ, "dmaq"), (RO, "dmao"))):
        for i in range(4):
            ops.append((f"s_add_u32 m0, {S_M0}, {stage * STAGE + x * OOFF + i * 1024}",
                        f"buffer_load_dwordx4 {V.r(nm, i)}, {rs}, 0 offen lds"))
    ops.append((f"s_add_u32 m0, {S_RCM0}, {stage * RC}",
                f"buffer_load_dword {V.r('rcv')}, {RRC}, 0 offen lds"))
    adv = ([f"v_add_u32 {V.r('dmaq', i)}, s48, {V.r('dmaq', i)}" for i in range(4)]
           + [f"v_add_u32 {V.r('dmao', i)}, s49, {V.r('dmao', i)}" for i in range(4)]
           + [f"v_add_u32 {V.r('rcv')}, 0x100, {V.r('rcv')}"])
    return ops, adv


def prologue(st: Stream, V, A):
    e, r = st.emit, st.raw
    r(f"s_load_dwordx16 s[16:31], {S_KARG}, 0x0")
    r(f"s_load_dwordx16 s[32:47], {S_KARG}, 0x40")
    r(f"s_load_dwordx4 s[48:51], {S_KARG}, 0x80")
    e(f"v_and_b32 {V.r('lane')}, 63, {V.r('tid')}")
    r(f"v_readfirstlane_b32 {S_WAVE}, {V.r('tid')}")  # first lane's id = 64 * wave
    r("s_nop 1")
    r(f"s_lshr_b32 {S_WAVE}, {S_WAVE}, 6")
    r("s_getpc_b64 s[96:97]")
    r("s_add_u32 s96, s96, vd_attn_dkdv128_lanes@rel32@lo+4")
    r("s_addc_u32 s97, s97, vd_attn_dkdv128_lanes@rel32@hi+12")
    r("s_waitcnt lgkmcnt(0)")
    r(f"s_mul_i32 s52, {S_WGZ}, s35")
    r(f"s_add_u32 s52, s52, {S_WGY}")

    def mad64(dlo, dhi, a, blo, bhi, t):
        r(f"s_mul_i32 {dlo}, {a}, {blo}")
        r(f"s_mul_hi_u32 {dhi}, {a}, {blo}")
        r(f"s_mul_i32 {t}, {a}, {bhi}")
        r(f"s_add_u32 {dhi}, {dhi}, {t}")

    mad64("s54", "s55", S_WGZ, "s36", "s37", "s58")
    mad64("s58", "s59", S_WGY, "s38", "s39", "s99")
    r("s_add_u32 s54, s54, s58")
    r("s_addc_u32 s55, s55, s59")
    mad64("s56", "s57", S_WGZ, "s40", "s41", "s58")
    mad64("s58", "s59", S_WGY, "s42", "s43", "s99")
    r("s_add_u32 s56, s56, s58")
    r("s_addc_u32 s57, s57, s59")

    def rsrc(dst, plo, phi, blo, bhi, nrec):
        d0 = int(dst[2:].split(":")[0])
        r(f"s_add_u32 s{d0}, {plo}, {blo}")
        r(f"s_addc_u32 s{d0 + 1}, {phi}, {bhi}")
        r(f"s_and_b32 s{d0 + 1}, s{d0 + 1}, 0xffff")
        r(f"s_mov_b32 s{d0 + 2}, {nrec}")
        r(f"s_mov_b32 s{d0 + 3}, 0x20000")

    rsrc(RQ, "s16", "s17", "s54", "s55", "s46")
    rsrc(RK, "s18", "s19", "s54", "s55", "s46")
    rsrc(RV, "s20", "s21", "s54", "s55", "s46")
    rsrc(RO, "s22", "s23", "s56", "s57", "s47")
    rsrc(RDK, "s28", "s29", "s54", "s55", "s46")
    rsrc(RDV, "s30", "s31", "s54", "s55", "s46")
    r("s_mul_i32 s58, s52, s32")
    r("s_mul_hi_u32 s59, s52, s32")
    r("s_lshl_b64 s[58:59], s[58:59], 2")
    r("s_lshl_b32 s99, s32, 2")
    rsrc(RL, "s24", "s25", "s58", "s59", "s99")
    rsrc(RD, "s26", "s27", "s58", "s59", "s99")
    # wave 1 stages delta, the others lse' (waves 2, 3 into the junk slot)
    r(f"s_cmp_eq_u32 {S_WAVE}, 1")
    r("s_cselect_b64 s[56:57], s[80:81], s[76:77]")
    r("s_cselect_b64 s[58:59], s[82:83], s[78:79]")
    r(f"s_min_u32 s99, {S_WAVE}, 2")
    r(f"s_lshl_b32 {S_RCM0}, s99, 8")
    # k0 = wgx * 128 + wave * 32 ; DMA M0 base = wave * 4096 (+ the tile region)
    r(f"s_lshl_b32 {S_K0}, {S_WGX}, 7")
    r(f"s_lshl_b32 s99, {S_WAVE}, 5")
    r(f"s_add_u32 {S_K0}, {S_K0}, s99")
    r(f"s_lshl_b32 {S_M0}, {S_WAVE}, 12")
    r(f"s_add_u32 {S_M0}, {S_M0}, {RC_BYTES}")
    r(f"s_mov_b32 {S_ITER}, s50")
    t0, t1 = V.r("tmp", 0), V.r("tmp", 1)
    e(f"v_lshlrev_b32 {t0}, 7, {V.r('tid')}")
    r(f"global_load_dwordx4 {V.r('rowoff', 0, 4)}, {t0}, s[96:97]")
    r(f"global_load_dwordx4 {V.r('rowoff', 4, 4)}, {t0}, s[96:97] offset:16")
    r(f"global_load_dwordx4 {V.r('troff', 0, 4)}, {t0}, s[96:97] offset:32")
    r(f"global_load_dwordx4 {V.r('troff', 4, 4)}, {t0}, s[96:97] offset:48")
    r(f"global_load_dwordx4 {V.r('dmaq', 0, 4)}, {t0}, s[96:97] offset:64")
    r(f"global_load_dwordx4 {V.r('dmao', 0, 4)}, {t0}, s[96:97] offset:80")
    r(f"global_load_dword {V.r('rcoff')}, {t0}, s[96:97] offset:96")
    # key row of the lane: krow = k0 + (lane & 31)   (staging registers in dp)
    krow, hh16, vk, h8 = (V.r("dp", k) for k in (28, 29, 30, 31))
    e(f"v_and_b32 {krow}, 31, {V.r('lane')}")
    e(f"v_add_u32 {krow}, {S_K0}, {krow}")
    e(f"v_lshrrev_b32 {hh16}, 5, {V.r('lane')}")
    e(f"v_lshlrev_b32 {hh16}, 4, {hh16}")
    kv = V["s"]  # K fragments staged in v[s .. s+31] for scaling
    e(f"v_mul_lo_u32 {vk}, {krow}, s33")
    e(f"v_add_u32 {vk}, {vk}, {hh16}")
    for s in range(8):
        r(f"buffer_load_dwordx4 v[{kv + 4 * s}:{kv + 4 * s + 3}], {vk}, {RK}, 0 offen "
          f"offset:{32 * s}")
        r(f"buffer_load_dwordx4 {A.r('vf', 4 * s, 4)}, {vk}, {RV}, 0 offen offset:{32 * s}")
    e(f"v_lshrrev_b32 {h8}, 1, {hh16}")
    e(f"v_mul_lo_u32 {V.r('stk')}, {krow}, s33")
    e(f"v_add_u32 {V.r('stk')}, {V.r('stk')}, {h8}")
    r("s_waitcnt vmcnt(0)")
    for w in range(32):
        x = f"v{kv + w}"
        e(f"v_lshlrev_b32 {t0}, 16, {x}")
        e(f"v_and_b32 {t1}, 0xffff0000, {x}")
        e(f"v_mul_f32 {t0}, s45, {t0}")
        e(f"v_mul_f32 {t1}, s45, {t1}")
        e(f"v_cvt_pk_bf16_f32 {x}, {t0}, {t1}")
        e(f"v_accvgpr_write_b32 {A.r('kf', w)}, {x}")
    # DMA source offsets: row * stride + chunk * 16 (the chunks were loaded into dmao)
    for i in range(4):
        e(f"v_mov_b32 {V.r('tmp', i)}, {V.r('dmao', i)}")
    for i in range(4):
        e(f"v_mul_lo_u32 {V.r('dmao', i)}, {V.r('dmaq', i)}, s34")
        e(f"v_add_u32 {V.r('dmao', i)}, {V.r('dmao', i)}, {V.r('tmp', i)}")
        e(f"v_mul_lo_u32 {V.r('dmaq', i)}, {V.r('dmaq', i)}, s33")
        e(f"v_add_u32 {V.r('dmaq', i)}, {V.r('dmaq', i)}, {V.r('tmp', i)}")
    e(f"v_lshlrev_b32 {V.r('rcv')}, 2, {V.r('lane')}")
    for k in range(8):
        e(f"v_add_u32 {V.r('rowhi', k)}, {HI:#x}, {V.r('rowoff', k)}")
        e(f"v_add_u32 {V.r('trhi', k)}, {HI:#x}, {V.r('troff', k)}")
    for k in range(128):
        e(f"v_accvgpr_write_b32 a{A['adk'] + k}, 0")
    for name in ("pp", "ds"):
        for k in range(16):
            e(f"v_mov_b32 {V.r(name, k)}, 0")
    for k in range(32):
        e(f"v_mov_b32 {V.r('s', k)}, 0")
        e(f"v_mov_b32 {V.r('dp', k)}, 0")
    for k in range(4):
        e(f"v_mov_b32 {V.r('tmp', k)}, 0")
    # zero ring stage 3 (tile -1: the A operands of the first G group, times P = dS = 0)
    e(f"v_lshlrev_b32 {V.r('tmp2', 0)}, 7, {V.r('tid')}")
    e(f"v_add_u32 {V.r('tmp2', 0)}, {RC_BYTES + 3 * STAGE:#x}, {V.r('tmp2', 0)}")
    for k in range(8):
        e(f"ds_write_b128 {V.r('tmp2', 0)}, {V.r('tmp', 0, 4)} offset:{16 * k}")
    r("s_waitcnt lgkmcnt(0)")
    for t in range(3):
        ops, adv = dma_ops(V, t)
        for m0, ld in ops:
            r(m0)
            r("s_nop 0")
            e(ld)
        for a in adv:
            e(a)
    r("s_waitcnt vmcnt(18)")
    r("s_barrier")
    st.flush_lds()
    for text, rid in row_reads(V, A, 0, 0):
        e(text, lds_id=rid)


def emit_iter(st: Stream, V, A, stage, vlist):
    """Iteration t (tile t in `stage`): S/dP(t, qb0), G(t-1, qb1), S/dP(t, qb1), barrier for
    tile t+1, G(t, qb0); the reads of (t+1, qb0) and tile t+3's DMA after the barrier."""
    prev, nxt = (stage + 3) % 4, (stage + 1) % 4
    st.comment(f"---- query tile, ring stage {stage}")
    mf = sdp(V, A, 0) + gmm(V, A, 1) + sdp(V, A, 1) + gmm(V, A, 0)
    nm = len(mf)
    slots = {}
    for i, text in enumerate(vlist):
        slots.setdefault((START + (i * nm) // len(vlist)) % nm, []).append((text, None))

    def put(slot0, lst, per=2):
        for k, (text, rid) in enumerate(lst):
            slots.setdefault(slot0 + k // per, []).insert(0 if per == 1 else k % per, (text, rid))

    put(DK_TR0, tr_reads(V, A, prev, 1))     # G(t-1, qb1) operands, tile t-1: slots 1..16
    put(DK_ROW1, row_reads(V, A, stage, 1))  # (t, qb1) fragments: 18..29
    put(DK_TR1, tr_reads(V, A, stage, 0))    # G(t, qb0) operands: 32..47
    ops, adv = dma_ops(V, prev)
    dma_at = list(range(DK_DMA0, DK_DMA0 + 9))
    for g in range(nm):
        if g == 48:
            st.raw("s_waitcnt vmcnt(9) lgkmcnt(0)")
            st.raw("s_barrier")
            st.flush_lds()
            for k, (text, rid) in enumerate(row_reads(V, A, nxt, 0)):
                slots.setdefault(48 + k // 2, []).insert(k % 2, (text, rid))
        if g in dma_at:
            m0, ld = ops[dma_at.index(g)]
            st.raw(m0)
            st.raw("s_nop 0")
            st.emit(ld)
            if g == dma_at[-1]:
                for a in adv:
                    st.emit(a)
        for text, rid in slots.get(g, []):
            st.emit(text, lds_id=rid)
        text, deps = mf[g]
        st.emit(text, wait_lds=deps)


def emit_tail(st: Stream, V, A, vlist):
    nm = 64
    st.comment("---- tail: the last tile's second G group")
    st.raw("s_waitcnt lgkmcnt(0)")
    st.flush_lds()
    rest = [t for i, t in enumerate(vlist) if START + (i * nm) // len(vlist) >= nm]
    for text, rid in tr_reads(V, A, 3, 1):
        st.emit(text, lds_id=rid)
    for t in rest:
        st.emit(t)
    for text, deps in gmm(V, A, 1):
        st.emit(text, wait_lds=deps)


def epilogue(st: Stream, V, A):
    st.raw("s_waitcnt vmcnt(0)")
    t = [V["s"] + k for k in range(8)]
    for name, rs, scale in (("adk", RDK, "s44"), ("adv", RDV, None)):
        for i in range(4):
            for g in range(4):
                base = 16 * i + 4 * g
                for k in range(4):
                    st.emit(f"v_accvgpr_read_b32 v{t[k]}, {A.r(name, base + k)}")
                if scale:
                    for k in range(4):
                        st.emit(f"v_mul_f32 v{t[k]}, {scale}, v{t[k]}")
                st.emit(f"v_cvt_pk_bf16_f32 v{t[4]}, v{t[0]}, v{t[1]}")
                st.emit(f"v_cvt_pk_bf16_f32 v{t[5]}, v{t[2]}, v{t[3]}")
                st.emit(f"buffer_store_dwordx2 v[{t[4]}:{t[5]}], {V.r('stk')}, {rs}, 0 offen "
                        f"offset:{64 * i + 16 * g}")


def gen_dkdv128():
    V, A = regs()
    st = Stream()
    prologue(st, V, A)
    vlist = valu(V)
    st.label(".Ldk128_loop")
    for stage in range(NST):
        emit_iter(st, V, A, stage, vlist)
    st.raw(f"s_sub_u32 {S_ITER}, {S_ITER}, 1")
    st.raw(f"s_cmp_lg_u32 {S_ITER}, 0")
    st.raw("s_cbranch_scc1 .Ldk128_loop")
    emit_tail(st, V, A, vlist)
    epilogue(st, V, A)
    k = kernel_text("vd_attn_bwd_dkdv_d128", st.text(), vgprs=V.next, agprs=A.next, sgprs=100,
                    lds_bytes=RC_BYTES + NST * STAGE, kernarg_bytes=KARG, wg_size=64 * NW)
    data = "\n.rodata\n.p2align 8\nvd_attn_dkdv128_lanes:\n"
    for row in lane_table():
        data += "\t.long " + ", ".join(str(x) for x in row) + "\n"
    return k, data, st


# ================================================================== dQ
# vd_attn_bwd_dq_d128: the arithmetic of the head_dim-64 dQ kernel (gen_attn_asm.py;
# attention.hip attn_bwd_dq_pipe_kernel: S'^T = K Q'^T - lse', dP^T = V dO^T - delta,
# dS^T = exp2(S'^T) * dP^T, dQ^T += K^T dS^T, Q' = Q * scale * log2 e in bf16) at one wave
# per SIMD with 32 queries per wave (128 per workgroup): Q', dO and the dQ^T accumulators
# (128 registers) of the wave's queries and the K / V row fragments of a 64-key tile (2 key
# blocks kb) in AGPRs; the score blocks, the K^T fragments (read one tile ahead) and the
# softmax in VGPRs.  Per 64-key tile a wave runs 48 MFMAs in the order
#     G(t-1, kb0) [8] | S/dP(t, kb0) [16] | G(t-1, kb1) [8] | S/dP(t, kb1) [16]
# (G = dQ^T += K^T dS^T over 4 output-dim blocks x 2 key k-steps) and 80 VALU instructions
# (the softmax of kb0 in the gaps after its S/dP, that of kb1 in the first gaps of the next
# tile).  Ring: 4 stages x (K tile 16 KiB | V tile 16 KiB), tile t + 2 issued in tile t (8
# LDS-DMA pieces per wave), one barrier per tile behind s_waitcnt vmcnt(8).
DQ_KARG = 128
DQ_START = 26
DQ_KV0, DQ_TR0, DQ_KV1, DQ_TR1 = 0, 8, 16, 32   # read placement knobs (A/B)
DQ_DMA = (2, 5, 8, 11, 14, 17, 20, 23)
RQ3, RK3, RV3, RO3, RL3, RD3, RDQ3 = ("s[56:59]", "s[60:63]", "s[64:67]", "s[68:71]",
                                      "s[72:75]", "s[76:79]", "s[80:83]")
S3_WAVE, S3_Q0, S3_M0, S3_ITER = "s84", "s85", "s86", "s87"


def dq_regs():
    V, A = Regs("v"), Regs("a")
    for name, n in (("tid", 1), ("lane", 1), ("rowoff", 8), ("troff", 8), ("rowhi", 8),
                    ("trhi", 8), ("dma", 4), ("tmp", 4), ("stq", 1), ("tmp2", 2)):
        V.alloc(name, n)
    V.alloc("sacc", 32, 16)  # S'^T blocks [kb]
    V.alloc("dpacc", 32)     # dP^T blocks [kb]
    V.alloc("ds", 16)        # dS^T as bf16 B operands [kb] x 8
    V.alloc("il", 16)        # -lse' splat (srcC of the first S MFMA)
    V.alloc("id", 16)        # -delta splat
    V.alloc("trf", 64)       # K^T fragments [kb][i][s2] (lo 2 + hi 2)
    A.alloc("qf", 32)        # Q' fragments [s]
    A.alloc("of", 32)        # dO fragments [s]
    A.alloc("acc", 64)       # dQ^T accumulators [i]
    A.alloc("kf", 64)        # K row fragments [kb][s]
    A.alloc("vf", 64)        # V row fragments [kb][s]
    assert V.next <= 256 and A.next <= 256, (V.next, A.next)
    return V, A


def dq_kv_reads(V, A, stage, kb):
    out = []
    base = stage * STAGE + kb * 8192
    for s in range(8):
        for x, name, off in (("K", "kf", 0), ("V", "vf", OOFF)):
            b, o = lds(V, "rowoff", s, base + off)
            out.append((f"ds_read_b128 {A.r(name, 32 * kb + 4 * s, 4)}, {b} offset:{o}",
                        (x, kb, s)))
    return out


def dq_tr_reads(V, stage, kb):
    out = []
    for i in range(4):
        for s2 in range(2):
            for hi in range(2):
                b, o = lds(V, "troff", 2 * i + hi, stage * STAGE + kb * 8192 + s2 * 4096)
                out.append((f"ds_read_b64_tr_b16 {V.r('trf', 32 * kb + 8 * i + 4 * s2 + 2 * hi, 2)}"
                            f", {b} offset:{o}", ("T", kb, i, s2, hi)))
    return out


def dq_g(V, A, kb, deps=True):
    out = []
    for i in range(4):
        acc = A.r("acc", 16 * i, 16)
        for s2 in range(2):
            d = tuple(("T", kb, i, s2, h) for h in range(2)) if deps else ()
            out.append((f"{MFMA} {acc}, {V.r('trf', 32 * kb + 8 * i + 4 * s2, 4)}, "
                        f"{V.r('ds', 8 * kb + 4 * s2, 4)}, {acc}", d))
    return out


def dq_pair(V, A, kb):
    out = []
    sv, dv = V.r("sacc", 16 * kb, 16), V.r("dpacc", 16 * kb, 16)
    for s in range(8):
        cs = V.r("il", 0, 16) if s == 0 else sv
        cd = V.r("id", 0, 16) if s == 0 else dv
        out.append((f"{MFMA} {sv}, {A.r('kf', 32 * kb + 4 * s, 4)}, {A.r('qf', 4 * s, 4)}, {cs}",
                    (("K", kb, s),)))
        out.append((f"{MFMA} {dv}, {A.r('vf', 32 * kb + 4 * s, 4)}, {A.r('of', 4 * s, 4)}, {cd}",
                    (("V", kb, s),)))
    return out


def dq_valu(V):
    out = []
    for kb in range(2):
        S, Dp, G = V["sacc"] + 16 * kb, V["dpacc"] + 16 * kb, V["ds"] + 8 * kb
        for k in range(8):
            a, b = 2 * k, 2 * k + 1
            out += [f"v_exp_f32 v{S + a}, v{S + a}", f"v_exp_f32 v{S + b}, v{S + b}",
                    f"v_mul_f32 v{Dp + a}, v{S + a}, v{Dp + a}",
                    f"v_mul_f32 v{Dp + b}, v{S + b}, v{Dp + b}",
                    f"v_cvt_pk_bf16_f32 v{G + k}, v{Dp + a}, v{Dp + b}"]
    return out


def dq_dma_ops(V, stage):
    ops = []
    for x, rs in ((0, RK3), (OOFF, RV3)):
        for i in range(4):
            ops.append((f"s_add_u32 m0, {S3_M0}, {stage * STAGE + x + i * 1024}",
                        f"buffer_load_dwordx4 {V.r('dma', i)}, {rs}, 0 offen lds"))
    adv = [f"v_add_u32 {V.r('dma', i)}, s46, {V.r('dma', i)}" for i in range(4)]
    return ops, adv


def dq_prologue(st: Stream, V, A):
    e, r = st.emit, st.raw
    r(f"s_load_dwordx16 s[16:31], {S_KARG}, 0x0")
    r(f"s_load_dwordx16 s[32:47], {S_KARG}, 0x40")
    e(f"v_and_b32 {V.r('lane')}, 63, {V.r('tid')}")
    r(f"v_readfirstlane_b32 {S3_WAVE}, {V.r('tid')}")
    r("s_nop 1")
    r(f"s_lshr_b32 {S3_WAVE}, {S3_WAVE}, 6")
    r("s_getpc_b64 s[88:89]")
    r("s_add_u32 s88, s88, vd_attn_dkdv128_lanes@rel32@lo+4")  # the dK/dV kernel's table
    r("s_addc_u32 s89, s89, vd_attn_dkdv128_lanes@rel32@hi+12")
    r("s_waitcnt lgkmcnt(0)")
    r(f"s_mul_i32 s48, {S_WGZ}, s33")
    r(f"s_add_u32 s48, s48, {S_WGY}")

    def mad64(dlo, dhi, a, blo, bhi, t):
        r(f"s_mul_i32 {dlo}, {a}, {blo}")
        r(f"s_mul_hi_u32 {dhi}, {a}, {blo}")
        r(f"s_mul_i32 {t}, {a}, {bhi}")
        r(f"s_add_u32 {dhi}, {dhi}, {t}")

    mad64("s50", "s51", S_WGZ, "s34", "s35", "s90")
    mad64("s92", "s93", S_WGY, "s36", "s37", "s90")
    r("s_add_u32 s50, s50, s92")
    r("s_addc_u32 s51, s51, s93")
    mad64("s52", "s53", S_WGZ, "s38", "s39", "s90")
    mad64("s92", "s93", S_WGY, "s40", "s41", "s90")
    r("s_add_u32 s52, s52, s92")
    r("s_addc_u32 s53, s53, s93")

    def rsrc(dst, plo, phi, blo, bhi, nrec):
        d0 = int(dst[2:].split(":")[0])
        r(f"s_add_u32 s{d0}, {plo}, {blo}")
        r(f"s_addc_u32 s{d0 + 1}, {phi}, {bhi}")
        r(f"s_and_b32 s{d0 + 1}, s{d0 + 1}, 0xffff")
        r(f"s_mov_b32 s{d0 + 2}, {nrec}")
        r(f"s_mov_b32 s{d0 + 3}, 0x20000")

    rsrc(RQ3, "s16", "s17", "s50", "s51", "s44")
    rsrc(RK3, "s18", "s19", "s50", "s51", "s44")
    rsrc(RV3, "s20", "s21", "s50", "s51", "s44")
    rsrc(RO3, "s22", "s23", "s52", "s53", "s45")
    rsrc(RDQ3, "s28", "s29", "s50", "s51", "s44")
    r("s_mul_i32 s92, s48, s30")
    r("s_mul_hi_u32 s93, s48, s30")
    r("s_lshl_b64 s[92:93], s[92:93], 2")
    r("s_lshl_b32 s94, s30, 2")
    rsrc(RL3, "s24", "s25", "s92", "s93", "s94")
    rsrc(RD3, "s26", "s27", "s92", "s93", "s94")
    # q0 = wgx * 128 + wave * 32 ; M0 base of this wave's DMA pieces = wave * 4096
    r(f"s_lshl_b32 {S3_Q0}, {S_WGX}, 7")
    r(f"s_lshl_b32 s90, {S3_WAVE}, 5")
    r(f"s_add_u32 {S3_Q0}, {S3_Q0}, s90")
    r(f"s_lshl_b32 {S3_M0}, {S3_WAVE}, 12")
    r(f"s_mov_b32 {S3_ITER}, s47")
    t0, t1 = V.r("tmp", 0), V.r("tmp", 1)
    e(f"v_lshlrev_b32 {t0}, 7, {V.r('tid')}")
    r(f"global_load_dwordx4 {V.r('rowoff', 0, 4)}, {t0}, s[88:89]")
    r(f"global_load_dwordx4 {V.r('rowoff', 4, 4)}, {t0}, s[88:89] offset:16")
    r(f"global_load_dwordx4 {V.r('troff', 0, 4)}, {t0}, s[88:89] offset:32")
    r(f"global_load_dwordx4 {V.r('troff', 4, 4)}, {t0}, s[88:89] offset:48")
    r(f"global_load_dwordx4 {V.r('dma', 0, 4)}, {t0}, s[88:89] offset:64")
    r(f"global_load_dwordx4 {V.r('rowhi', 0, 4)}, {t0}, s[88:89] offset:80")  # chunks
    # the lane's query row: qrow = q0 + (lane & 31)   (staging registers in dpacc)
    qrow, hh16, vq, vo, vl, h8 = (V.r("dpacc", k) for k in range(26, 32))
    e(f"v_and_b32 {qrow}, 31, {V.r('lane')}")
    e(f"v_add_u32 {qrow}, {S3_Q0}, {qrow}")
    e(f"v_lshrrev_b32 {hh16}, 5, {V.r('lane')}")
    e(f"v_lshlrev_b32 {hh16}, 4, {hh16}")
    qv = V["sacc"]  # Q fragments staged in v[sacc .. +31] for scaling
    e(f"v_mul_lo_u32 {vq}, {qrow}, s31")
    e(f"v_add_u32 {vq}, {vq}, {hh16}")
    for s in range(8):
        r(f"buffer_load_dwordx4 v[{qv + 4 * s}:{qv + 4 * s + 3}], {vq}, {RQ3}, 0 offen "
          f"offset:{32 * s}")
    e(f"v_mul_lo_u32 {vo}, {qrow}, s32")
    e(f"v_add_u32 {vo}, {vo}, {hh16}")
    for s in range(8):
        r(f"buffer_load_dwordx4 {A.r('of', 4 * s, 4)}, {vo}, {RO3}, 0 offen offset:{32 * s}")
    e(f"v_lshlrev_b32 {vl}, 2, {qrow}")
    r(f"buffer_load_dword {V.r('tmp2', 0)}, {vl}, {RL3}, 0 offen")
    r(f"buffer_load_dword {V.r('tmp2', 1)}, {vl}, {RD3}, 0 offen")
    e(f"v_lshrrev_b32 {h8}, 1, {hh16}")
    e(f"v_mul_lo_u32 {V.r('stq')}, {qrow}, s31")
    e(f"v_add_u32 {V.r('stq')}, {V.r('stq')}, {h8}")
    r("s_waitcnt vmcnt(0)")
    for w in range(32):
        x = f"v{qv + w}"
        e(f"v_lshlrev_b32 {t0}, 16, {x}")
        e(f"v_and_b32 {t1}, 0xffff0000, {x}")
        e(f"v_mul_f32 {t0}, s43, {t0}")
        e(f"v_mul_f32 {t1}, s43, {t1}")
        e(f"v_cvt_pk_bf16_f32 {x}, {t0}, {t1}")
        e(f"v_accvgpr_write_b32 {A.r('qf', w)}, {x}")
    for k in range(16):
        e(f"v_mov_b32 {V.r('il', k)}, {V.r('tmp2', 0)}")
        e(f"v_mov_b32 {V.r('id', k)}, {V.r('tmp2', 1)}")
    # DMA source offsets of tile 0: row * ts_bytes + chunk * 16
    for i in range(4):
        e(f"v_mul_lo_u32 {V.r('dma', i)}, {V.r('dma', i)}, s31")
        e(f"v_add_u32 {V.r('dma', i)}, {V.r('dma', i)}, {V.r('rowhi', i)}")
    for k in range(8):
        e(f"v_add_u32 {V.r('rowhi', k)}, {HI:#x}, {V.r('rowoff', k)}")
        e(f"v_add_u32 {V.r('trhi', k)}, {HI:#x}, {V.r('troff', k)}")
    # zero: accumulators, K^T fragments and dS of "tile -1" (the first tile's G products),
    # and the score blocks (the first tile's kb1 stream of "tile -1" then yields dS = 0)
    for k in range(64):
        e(f"v_accvgpr_write_b32 {A.r('acc', k)}, 0")
        e(f"v_mov_b32 {V.r('trf', k)}, 0")
    for k in range(16):
        e(f"v_mov_b32 {V.r('ds', k)}, 0")
    for k in range(32):
        e(f"v_mov_b32 {V.r('sacc', k)}, 0")
        e(f"v_mov_b32 {V.r('dpacc', k)}, 0")
    for t in range(2):
        ops, adv = dq_dma_ops(V, t)
        for m0, ld in ops:
            r(m0)
            r("s_nop 0")
            e(ld)
        for a in adv:
            e(a)


def dq_emit_tile(st: Stream, V, A, stage, vlist):
    st.comment(f"---- key tile, ring stage {stage}")
    st.raw("s_waitcnt vmcnt(8) lgkmcnt(0)")
    st.raw("s_barrier")
    st.flush_lds()
    mf = dq_g(V, A, 0) + dq_pair(V, A, 0) + dq_g(V, A, 1) + dq_pair(V, A, 1)
    nm = len(mf)
    slots = {}
    for i, text in enumerate(vlist):
        slots.setdefault((DQ_START + (i * nm) // len(vlist)) % nm, []).append((text, None))

    def put(slot0, lst, per=2):
        for k, (text, rid) in enumerate(lst):
            slots.setdefault(slot0 + k // per, []).insert(k % per, (text, rid))

    put(DQ_KV0, dq_kv_reads(V, A, stage, 0))  # kb0 rows: slots 0..7 (consumed 8..23)
    put(DQ_TR0, dq_tr_reads(V, stage, 0))     # K^T kb0 of this tile, for the next G: 8..15
    put(DQ_KV1, dq_kv_reads(V, A, stage, 1))  # kb1 rows: 16..23 (consumed 32..47)
    put(DQ_TR1, dq_tr_reads(V, stage, 1))     # K^T kb1: 32..39
    ops, adv = dq_dma_ops(V, (stage + 2) % NST)
    dma_at = list(DQ_DMA)
    # the G products read the K^T fragments of the previous tile (no LDS wait of their own)
    mf = [(t, ()) if k < 8 or 24 <= k < 32 else (t, d) for k, (t, d) in enumerate(mf)]
    for g in range(nm):
        if g in dma_at:
            m0, ld = ops[dma_at.index(g)]
            st.raw(m0)
            st.raw("s_nop 0")
            st.emit(ld)
            if g == dma_at[-1]:
                for a in adv:
                    st.emit(a)
        for text, rid in slots.get(g, []):
            st.emit(text, lds_id=rid)
        text, deps = mf[g]
        st.emit(text, wait_lds=deps)


def dq_emit_tail(st: Stream, V, A, vlist):
    nm = 48
    st.comment("---- tail: the last tile's dQ products")
    st.raw("s_waitcnt lgkmcnt(0)")
    st.flush_lds()
    rest = [t for i, t in enumerate(vlist) if DQ_START + (i * nm) // len(vlist) >= nm]
    g0, g1 = dq_g(V, A, 0, False), dq_g(V, A, 1, False)
    per = -(-len(rest) // 8)
    for k, (text, _) in enumerate(g0):
        for t in rest[k * per:(k + 1) * per]:
            st.emit(t)
        st.emit(text)
    for text, _ in g1:
        st.emit(text)


def dq_epilogue(st: Stream, V, A):
    st.raw("s_waitcnt vmcnt(0)")
    t = [V["sacc"] + k for k in range(8)]
    for i in range(4):
        for g in range(4):
            base = 16 * i + 4 * g
            for k in range(4):
                st.emit(f"v_accvgpr_read_b32 v{t[k]}, {A.r('acc', base + k)}")
            for k in range(4):
                st.emit(f"v_mul_f32 v{t[k]}, s42, v{t[k]}")
            st.emit(f"v_cvt_pk_bf16_f32 v{t[4]}, v{t[0]}, v{t[1]}")
            st.emit(f"v_cvt_pk_bf16_f32 v{t[5]}, v{t[2]}, v{t[3]}")
            st.emit(f"buffer_store_dwordx2 v[{t[4]}:{t[5]}], {V.r('stq')}, {RDQ3}, 0 offen "
                    f"offset:{64 * i + 16 * g}")


def gen_dq128():
    V, A = dq_regs()
    st = Stream()
    dq_prologue(st, V, A)
    vlist = dq_valu(V)
    st.label(".Ldq128_loop")
    for stage in range(NST):
        dq_emit_tile(st, V, A, stage, vlist)
    st.raw(f"s_sub_u32 {S3_ITER}, {S3_ITER}, 1")
    st.raw(f"s_cmp_lg_u32 {S3_ITER}, 0")
    st.raw("s_cbranch_scc1 .Ldq128_loop")
    dq_emit_tail(st, V, A, vlist)
    dq_epilogue(st, V, A)
    k = kernel_text("vd_attn_bwd_dq_d128", st.text(), vgprs=V.next, agprs=A.next, sgprs=96,
                    lds_bytes=NST * STAGE, kernarg_bytes=DQ_KARG, wg_size=64 * NW)
    return k, st
