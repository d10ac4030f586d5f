"""Hand-scheduled gfx950 head_dim-256 attention backward, dQ (reference QKVAttentionLegacy,
unet.py:349-366, at C = 256: the 32x32 level of the config-2 UNet3D, N = 16 x 32 x 32).

vd_attn_bwd_dq_d256 -- the arithmetic of the head_dim-128 dQ kernel (gen_d128.py; attention.hip
attn_bwd_dq_kernel: S'^T = K Q'^T - lse', dP^T = V dO^T - delta, dS^T = exp2(S'^T) * dP^T,
dQ^T += K^T dS^T, Q' = Q * scale * log2 e in bf16) at ONE wave per SIMD with 32 queries per
wave (128 per workgroup).  At head_dim 256 the wave's Q' and dO fragments (64 registers each)
and its full-width dQ^T accumulators (128) fill the 256 AGPRs, so the K and V row fragments of
the current key tile are STREAMED from LDS through two 4-slot VGPR rings just ahead of their
MFMAs, and a tile is 32 keys (one 32-key block):
    S/dP(t, s 0-7) [16] | G(t-1) [16] | S/dP(t, s 8-15) [16]
(S/dP: the S'^T and dP^T products of the 16 head-dim k-steps s, interleaved; G = dQ^T += K^T
dS^T over 8 output-dim blocks x 2 key k-steps).  The softmax of tile t-1 (16 v_exp_f32, 16
v_mul_f32, 8 v_cvt_pk_bf16_f32) runs in the gaps of the first group; S'^T / dP^T alternate
between two accumulator sets by tile parity so it reads the previous tile's while the
current one is computed.  The K^T fragments of tile t (the A operands of G(t), 32
ds_read_b64_tr_b16) are read in the last group of body t, from the tile's own ring stage.

Ring: 4 stages x (K tile 16 KiB | V tile 16 KiB) = 128 KiB of LDS by LDS-DMA, tile t + 2
issued in body t (8 pieces per wave), one barrier per body behind s_waitcnt vmcnt(8).  The
loop is unrolled by the 4 stages; tiles past the key range are zero rows (the buffer range
check), whose K^T products add nothing.

Key split (grid.z = sequences x 2^lsplit): split z takes keys [z kps, (z + 1) kps) (its K / V
buffer ranges end there) and, with part != 0, writes dQ (times scale) as fp32 partials
part[z][seq][n][256] that attention.hip's attn_dq_sum_kernel adds -- at N = 16384 the query
grid alone is 128 workgroups, half the chip.
"""
from __future__ import annotations

from asmgen import Regs, Stream, kernel_text

MFMA = "v_mfma_f32_32x32x16_bf16"
NW = 4
D = 256
KT = 32                 # keys per tile
KTILE = 16384           # one 32 x 256 bf16 tile; K tiles of the 4 stages in [0, 64 KiB),
VBASE = 65536           # V tiles in [64 KiB, 128 KiB): every K / K^T read stays within the
NST = 4                 # 16-bit ds_read immediate
HI = 65536
KARG = 160              # AsmDq256Args (vd_asm.h)
RING = 8                # K / V row-fragment ring slots (4 VGPRs each)
TRING = 8               # K^T fragment ring slots (4 VGPRs each: lo 2 + hi 2)
TR_AHEAD = 5            # K^T fragments read this many G products ahead

# kernel arguments (AsmDq256Args), s[16:55]:
#  0 q 8 k 16 v 24 dout 32 nlse2 40 ndelta 48 dq               (u64)  s16..s29
#  56 n 60 ts_bytes 64 ots_bytes 68 groups                      (u32)  s30..s33
#  72 bs_bytes 80 gs_bytes 88 obs_bytes 96 ogs_bytes            (u64)  s34..s41
#  104 scale 108 qscale 112 kv_bytes 116 o_bytes 120 tile_bytes 124 niter   s42..s47
#  128 part (u64) s48:49   136 kps (keys per split) s50   140 lsplit s51
#  144 split_bytes (u64: bytes of one split's partials) s52:53   152 n_bytes_part s54  156 pad
S_KARG = "s[0:1]"
S_WGX, S_WGY, S_WGZ = "s2", "s3", "s4"
RQ, RK, RV, RO, RL, RD, RDQ, RP = ("s[56:59]", "s[60:63]", "s[64:67]", "s[68:71]", "s[72:75]",
                                    "s[76:79]", "s[80:83]", "s[84:87]")
S_WAVE, S_Q0, S_M0, S_ITER, S_SEQ, S_SPLIT, S_ZS, S_X = ("s88", "s89", "s90", "s91", "s92",
                                                          "s93", "s94", "s95")
S_T0, S_T1, S_T2, S_T3 = "s96", "s97", "s98", "s99"   # two aligned pairs
S_TAB = "s[100:101]"
DMA_AT = tuple(range(17, 32, 2))   # the 8 LDS-DMA pieces: odd gaps of the G group


def swz(r):
    """attention.hip swz_row<256> (= <128>): 4-bit chunk XOR of row r."""
    return ((r & 3) << 2) | ((r >> 2) & 3)


def toff_bytes(r, c):
    """attention.hip toff<bf16, 256>(r, c) in bytes."""
    return 2 * (r * D + (((c >> 3) ^ swz(r)) << 3) + (c & 7))


def lane_table():
    """tab[wave][lane][32] u32: 0-7 row-fragment offsets of k-steps s = 0..7 (s + 8: +256 B),
    8-15 transposed-fragment offsets (2 i + hi, output-dim blocks i = 0..3; i + 4: +256 B;
    the second key k-step: +16 rows = +8192 B), 16-19 DMA rows of the wave's 4 pieces of a
    tile, 20-23 their source chunk * 16."""
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
                rr = gi * 2 + lane // 32
                drow.append(rr)
                dch.append(((lane % 32) ^ swz(rr)) * 16)
            out.append(row + tr + drow + dch + [0] * 8)
    # checks of the +256 B / +8192 B immediates the kernel relies on
    for r in range(32):
        for c in range(0, 128, 8):
            assert toff_bytes(r, c + 128) == toff_bytes(r, c) + 256
    for r in range(16):
        assert toff_bytes(r + 16, 0) == toff_bytes(r, 0) + 8192
    return out


def regs():
    V, A = Regs("v"), Regs("a")
    for name, n in (("tid", 1), ("lane", 1), ("rowoff", 8), ("troff", 8), ("rowhi", 8),
                    ("dma", 4), ("stq", 1)):
        V.alloc(name, n)
    V.alloc("sacc", 32, 16)  # S'^T [parity] x 16
    V.alloc("dpacc", 32)     # dP^T [parity] x 16
    V.alloc("ds", 8)         # dS^T as bf16 B operands [s2] x 4
    V.alloc("il", 16)        # -lse' splat (srcC of the first S MFMA)
    V.alloc("id", 16)        # -delta splat
    V.alloc("tr", 4 * TRING)  # K^T fragment ring [slot] (lo 2 + hi 2)
    V.alloc("kr", 4 * RING)  # K row-fragment ring
    V.alloc("vr", 4 * RING)  # V row-fragment ring (contiguous with kr: the Q staging)
    V.names["tmp"] = (V["tr"], 4)    # prologue scratch, aliased into the rings
    V.names["tmp2"] = (V["tr"] + 4, 2)
    A.alloc("qf", 64)        # Q' fragments [s]
    A.alloc("of", 64)        # dO fragments [s]
    A.alloc("acc", 128)      # dQ^T accumulators [i]
    assert V.next <= 256 and A.next <= 256, (V.next, A.next)
    return V, A


def row_read(V, stage, s, which):
    """ds_read_b128 of the K (which 0) / V (1) row fragment of k-step s into ring slot s % 8
    (V through the +64 KiB copies of the offsets)."""
    off = stage * KTILE + (256 if s >= 8 else 0)
    assert off + 15870 < HI
    b = V.r("rowoff" if which == 0 else "rowhi", s % 8)
    dst = V.r("kr" if which == 0 else "vr", 4 * (s % RING), 4)
    return (f"ds_read_b128 {dst}, {b} offset:{off}", ("KV"[which], s))


def tr_read_pair(V, stage, j):
    """The lo / hi transposed reads of G product j = 2 i + s2 (output-dim block i, key k-step
    s2) of the K tile in `stage` into ring slot j % 8."""
    i, s2 = j // 2, j % 2
    out = []
    for hi in range(2):
        off = stage * KTILE + (256 if i >= 4 else 0) + 8192 * s2
        assert off + 7934 < HI
        out.append((f"ds_read_b64_tr_b16 {V.r('tr', 4 * (j % TRING) + 2 * hi, 2)}, "
                    f"{V.r('troff', 2 * (i % 4) + hi)} offset:{off}", ("T", j, hi)))
    return out


def sdp_mfmas(V, A, par, s):
    """The S'^T and dP^T products of head-dim k-step s into accumulator set `par`."""
    sv, dv = V.r("sacc", 16 * par, 16), V.r("dpacc", 16 * par, 16)
    cs = V.r("il", 0, 16) if s == 0 else sv
    cd = V.r("id", 0, 16) if s == 0 else dv
    k = V.r("kr", 4 * (s % RING), 4)
    v = V.r("vr", 4 * (s % RING), 4)
    return [(f"{MFMA} {sv}, {k}, {A.r('qf', 4 * s, 4)}, {cs}", (("K", s),)),
            (f"{MFMA} {dv}, {v}, {A.r('of', 4 * s, 4)}, {cd}", (("V", s),))]


def g_mfmas(V, A, deps=True):
    out = []
    for j in range(16):
        i, s2 = j // 2, j % 2
        acc = A.r("acc", 16 * i, 16)
        out.append((f"{MFMA} {acc}, {V.r('tr', 4 * (j % TRING), 4)}, "
                    f"{V.r('ds', 4 * s2, 4)}, {acc}", (("T", j, 0), ("T", j, 1)) if deps else ()))
    return out


def valu(V, par):
    """Softmax of the tile in accumulator set `par`: dS^T = exp2(S'^T) * dP^T as bf16."""
    out = []
    S, Dp, G = V["sacc"] + 16 * par, V["dpacc"] + 16 * par, V["ds"]
    for k in range(8):
        a, b = 2 * k, 2 * k + 1
        out += [f"v_exp_f32 v{S + a}, v{S + a}", f"v_exp_f32 v{S + b}, v{S + b}",
                f"v_mul_f32 v{Dp + a}, v{S + a}, v{Dp + a}",
                f"v_mul_f32 v{Dp + b}, v{S + b}, v{Dp + b}",
                f"v_cvt_pk_bf16_f32 v{G + k}, v{Dp + a}, v{Dp + b}"]
    return out


def dma_ops(V, stage):
    ops = []
    for x, rs in ((0, RK), (VBASE, RV)):
        for i in range(4):
            ops.append((f"s_add_u32 m0, {S_M0}, {x + stage * KTILE + i * 1024}",
                        f"buffer_load_dwordx4 {V.r('dma', i)}, {rs}, 0 offen lds"))
    adv = [f"v_add_u32 {V.r('dma', i)}, s46, {V.r('dma', i)}" for i in range(4)]
    return ops, adv


def prologue(st: Stream, V, A):
    e, r = st.emit, st.raw
    r(f"s_load_dwordx16 s[16:31], {S_KARG}, 0x0")
    r(f"s_load_dwordx16 s[32:47], {S_KARG}, 0x40")
    r(f"s_load_dwordx8 s[48:55], {S_KARG}, 0x80")
    e(f"v_and_b32 {V.r('lane')}, 63, {V.r('tid')}")
    r(f"v_readfirstlane_b32 {S_WAVE}, {V.r('tid')}")
    r("s_nop 1")
    r(f"s_lshr_b32 {S_WAVE}, {S_WAVE}, 6")
    r(f"s_getpc_b64 {S_TAB}")
    r("s_add_u32 s100, s100, vd_attn_d256_lanes@rel32@lo+4")
    r("s_addc_u32 s101, s101, vd_attn_d256_lanes@rel32@hi+12")
    r("s_waitcnt lgkmcnt(0)")
    # grid.z = (sequence group z') << lsplit | split
    r(f"s_lshl_b32 {S_X}, 1, s51")
    r(f"s_sub_u32 {S_X}, {S_X}, 1")
    r(f"s_and_b32 {S_SPLIT}, {S_WGZ}, {S_X}")
    r(f"s_lshr_b32 {S_ZS}, {S_WGZ}, s51")
    r(f"s_mul_i32 {S_SEQ}, {S_ZS}, s33")
    r(f"s_add_u32 {S_SEQ}, {S_SEQ}, {S_WGY}")

    def mad64(dlo, dhi, a, blo, bhi):
        r(f"s_mul_i32 {dlo}, {a}, {blo}")
        r(f"s_mul_hi_u32 {dhi}, {a}, {blo}")
        r(f"s_mul_i32 {S_X}, {a}, {bhi}")
        r(f"s_add_u32 {dhi}, {dhi}, {S_X}")

    def add64():  # T0:T1 += T2:T3
        r(f"s_add_u32 {S_T0}, {S_T0}, {S_T2}")
        r(f"s_addc_u32 {S_T1}, {S_T1}, {S_T3}")

    def rsrc(dst, plo, phi, nrec):
        d0 = int(dst[2:].split(":")[0])
        r(f"s_add_u32 s{d0}, {plo}, {S_T0}")
        r(f"s_addc_u32 s{d0 + 1}, {phi}, {S_T1}")
        r(f"s_and_b32 s{d0 + 1}, s{d0 + 1}, 0xffff")
        r(f"s_mov_b32 s{d0 + 2}, {nrec}")
        r(f"s_mov_b32 s{d0 + 3}, 0x20000")

    # q / dq sequence base
    mad64(S_T0, S_T1, S_ZS, "s34", "s35")
    mad64(S_T2, S_T3, S_WGY, "s36", "s37")
    add64()
    rsrc(RQ, "s16", "s17", "s44")
    rsrc(RDQ, "s28", "s29", "s44")
    # K / V: this split's keys [split * kps, min(n, (split + 1) * kps)): base += split * kps
    # * ts_bytes, range (keys - 1) * ts_bytes + 512 (the host keeps every split non-empty)
    r(f"s_mul_i32 {S_T2}, {S_SPLIT}, s50")       # first key of the split
    r(f"s_sub_u32 {S_T3}, s30, {S_T2}")          # keys left in the sequence
    r(f"s_min_u32 {S_T3}, {S_T3}, s50")          # keys of this split
    r(f"s_sub_u32 {S_T3}, {S_T3}, 1")
    r(f"s_mul_i32 {S_T3}, {S_T3}, s31")
    r(f"s_add_u32 {S_X}, {S_T3}, 512")           # K / V range
    r(f"s_mul_i32 {S_T2}, {S_T2}, s31")          # split offset in bytes (< 2 GiB: asm_dq_ok)
    r(f"s_add_u32 {S_T0}, {S_T0}, {S_T2}")
    r(f"s_addc_u32 {S_T1}, {S_T1}, 0")
    r(f"s_mov_b32 {S_T3}, {S_X}")
    rsrc(RK, "s18", "s19", S_T3)
    rsrc(RV, "s20", "s21", S_T3)
    # dout base
    mad64(S_T0, S_T1, S_ZS, "s38", "s39")
    mad64(S_T2, S_T3, S_WGY, "s40", "s41")
    add64()
    rsrc(RO, "s22", "s23", "s45")
    # lse' / delta rows of the sequence: seq * n * 4, range n * 4
    r(f"s_mul_i32 {S_T0}, {S_SEQ}, s30")
    r(f"s_mul_hi_u32 {S_T1}, {S_SEQ}, s30")
    r(f"s_lshl_b64 s[96:97], s[96:97], 2")
    r(f"s_lshl_b32 {S_T2}, s30, 2")
    rsrc(RL, "s24", "s25", S_T2)
    rsrc(RD, "s26", "s27", S_T2)
    # fp32 partials: part + split * split_bytes + seq * n * 1024, range n * 1024
    mad64(S_T0, S_T1, S_SPLIT, "s52", "s53")
    r(f"s_mul_i32 {S_T2}, {S_SEQ}, s30")
    r(f"s_mul_hi_u32 {S_T3}, {S_SEQ}, s30")
    r(f"s_lshl_b64 s[98:99], s[98:99], 10")
    add64()
    rsrc(RP, "s48", "s49", "s54")
    # q0 = wgx * 128 + wave * 32 ; M0 base of this wave's DMA pieces = wave * 4096
    r(f"s_lshl_b32 {S_Q0}, {S_WGX}, 7")
    r(f"s_lshl_b32 {S_X}, {S_WAVE}, 5")
    r(f"s_add_u32 {S_Q0}, {S_Q0}, {S_X}")
    r(f"s_lshl_b32 {S_M0}, {S_WAVE}, 12")
    r(f"s_mov_b32 {S_ITER}, s47")
    t0, t1 = V.r("tmp", 0), V.r("tmp", 1)
    e(f"v_lshlrev_b32 {t0}, 7, {V.r('tid')}")
    r(f"global_load_dwordx4 {V.r('rowoff', 0, 4)}, {t0}, {S_TAB}")
    r(f"global_load_dwordx4 {V.r('rowoff', 4, 4)}, {t0}, {S_TAB} offset:16")
    r(f"global_load_dwordx4 {V.r('troff', 0, 4)}, {t0}, {S_TAB} offset:32")
    r(f"global_load_dwordx4 {V.r('troff', 4, 4)}, {t0}, {S_TAB} offset:48")
    r(f"global_load_dwordx4 {V.r('dma', 0, 4)}, {t0}, {S_TAB} offset:64")
    r(f"global_load_dwordx4 {V.r('rowhi', 0, 4)}, {t0}, {S_TAB} offset:80")  # chunks
    # the lane's query row: qrow = q0 + (lane & 31)   (staging registers in dpacc)
    qrow, hh16, vq, vo, vl, h8 = (V.r("dpacc", k) for k in range(26, 32))
    e(f"v_and_b32 {qrow}, 31, {V.r('lane')}")
    e(f"v_add_u32 {qrow}, {S_Q0}, {qrow}")
    e(f"v_lshrrev_b32 {hh16}, 5, {V.r('lane')}")
    e(f"v_lshlrev_b32 {hh16}, 4, {hh16}")
    e(f"v_mul_lo_u32 {vq}, {qrow}, s31")
    e(f"v_add_u32 {vq}, {vq}, {hh16}")
    e(f"v_mul_lo_u32 {vo}, {qrow}, s32")
    e(f"v_add_u32 {vo}, {vo}, {hh16}")
    # Q fragments staged in the K / V rings (64 contiguous VGPRs) for scaling, dO straight into
    # the AGPRs
    qv = V["kr"]
    for s in range(16):
        r(f"buffer_load_dwordx4 v[{qv + 4 * s}:{qv + 4 * s + 3}], {vq}, {RQ}, 0 offen "
          f"offset:{32 * s}")
    for s in range(16):
        r(f"buffer_load_dwordx4 {A.r('of', 4 * s, 4)}, {vo}, {RO}, 0 offen offset:{32 * s}")
    e(f"v_lshlrev_b32 {vl}, 2, {qrow}")
    r(f"buffer_load_dword {V.r('tmp2', 0)}, {vl}, {RL}, 0 offen")
    r(f"buffer_load_dword {V.r('tmp2', 1)}, {vl}, {RD}, 0 offen")
    e(f"v_lshrrev_b32 {h8}, 1, {hh16}")
    # store offsets: bf16 dq row (qrow * ts + 8 hh) or fp32 partial row (qrow * 1024 + 16 hh)
    r(f"s_cmp_eq_u64 s[48:49], 0")
    r(f"s_cbranch_scc1 .Ldq256_bf16_st")
    e(f"v_lshlrev_b32 {V.r('stq')}, 10, {qrow}")
    e(f"v_add_u32 {V.r('stq')}, {V.r('stq')}, {hh16}")
    r(f"s_branch .Ldq256_st_done")
    st.label(".Ldq256_bf16_st")
    e(f"v_mul_lo_u32 {V.r('stq')}, {qrow}, s31")
    e(f"v_add_u32 {V.r('stq')}, {V.r('stq')}, {h8}")
    st.label(".Ldq256_st_done")
    r("s_waitcnt vmcnt(0)")
    for w in range(64):
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
    # zero: accumulators, dS of "tile -1" (the first body's G reads stage 3's K^T -- zeroed in
    # LDS below, so no NaN bit pattern meets the zero dS), and both score sets (the first
    # body's softmax of "tile -1" then yields dS = 0)
    for k in range(128):
        e(f"v_accvgpr_write_b32 {A.r('acc', k)}, 0")
    for k in range(4):
        e(f"v_mov_b32 {V.r('tmp', k)}, 0")
    e(f"v_lshlrev_b32 {V.r('tmp2', 0)}, 6, {V.r('tid')}")
    for k in range(4):   # stage 3's K tile: 256 lanes x 64 B
        e(f"ds_write_b128 {V.r('tmp2', 0)}, {V.r('tmp', 0, 4)} offset:{3 * KTILE + 16 * k}")
    for k in range(8):
        e(f"v_mov_b32 {V.r('ds', k)}, 0")
    for k in range(32):
        e(f"v_mov_b32 {V.r('sacc', k)}, 0")
        e(f"v_mov_b32 {V.r('dpacc', k)}, 0")
    for t in range(2):
        ops, adv = dma_ops(V, t)
        for m0, ld in ops:
            r(m0)
            r("s_nop 0")
            e(ld)
        for a in adv:
            e(a)


def emit_body(st: Stream, V, A, stage):
    """Body t (tile t in `stage`, accumulator set par = stage & 1): S/dP(t, s 0-7), G(t-1),
    S/dP(t, s 8-15); softmax(t-1) in the first group's gaps; the K / V row fragments two
    MFMAs ahead through the 8-slot rings; the K^T fragments of tile t-1 (still resident in its
    stage) TR_AHEAD products ahead of G; tile t+2's DMA in the G group."""
    par, prev = stage & 1, (stage + 3) % NST
    st.comment(f"---- key tile, ring stage {stage}")
    st.raw("s_waitcnt vmcnt(8) lgkmcnt(0)")
    st.raw("s_barrier")
    st.flush_lds()
    if stage == 0:  # loop back edge: the previous stage-3 body's last S/dP MFMAs wrote the
        st.raw("s_nop 12", ws=13)  # scores this body's softmax reads (not in the stream history)
    mf = []
    for s in range(8):
        mf += sdp_mfmas(V, A, par, s)
    mf += g_mfmas(V, A)
    for s in range(8, 16):
        mf += sdp_mfmas(V, A, par, s)
    nm = len(mf)                       # 48
    slots = {}

    def at(g, item):
        slots.setdefault(g, []).append(item)

    # row fragments: k-steps 0..7 two MFMAs (one pair) ahead from the barrier on; 8..15 in the
    # G group (their ring slots were last read by k-steps 0..7, in gaps <= 15)
    for s in range(8):
        g = max(0, 2 * s - 2)
        at(g, row_read(V, stage, s, 0))
        at(g, row_read(V, stage, s, 1))
    for s in range(8, 16):
        g = 18 + 2 * (s - 8) if s < 14 else 30
        at(g, row_read(V, stage, s, 0))
        at(g, row_read(V, stage, s, 1))
    # softmax of the previous tile (other accumulator set) over gaps 1..15
    vl = valu(V, 1 - par)
    for i, text in enumerate(vl):
        at(1 + (i * 14) // len(vl), (text, None))
    # K^T fragments of tile t-1 for G(t-1) (gaps 16..31)
    for j in range(16):
        for item in tr_read_pair(V, prev, j):
            at(16 + j - TR_AHEAD, item)
    ops, adv = dma_ops(V, (stage + 2) % NST)
    for g in range(nm):
        if g in DMA_AT:
            m0, ld = ops[DMA_AT.index(g)]
            st.raw(m0)
            st.raw("s_nop 0")
            st.emit(ld)
            if g == DMA_AT[-1]:
                for a in adv:
                    st.emit(a)
        for text, rid in slots.get(g, []):
            st.emit(text, lds_id=rid)
        text, deps = mf[g]
        st.emit(text, wait_lds=deps)


def emit_tail(st: Stream, V, A):
    """After the last tile T-1 (stage 3, set 1): its softmax, then G(T-1) over the K^T
    fragments of stage 3."""
    st.comment("---- tail: softmax and dQ products of the last tile")
    st.raw("s_waitcnt lgkmcnt(0)")
    st.flush_lds()
    for text in valu(V, 1):
        st.emit(text)
    g = g_mfmas(V, A)
    for j in range(16):
        for text, rid in tr_read_pair(V, 3, j):
            st.emit(text, lds_id=rid)
        text, deps = g[j]
        st.emit(text, wait_lds=deps)


def epilogue(st: Stream, V, A):
    st.raw("s_waitcnt vmcnt(0)")
    t = [V["sacc"] + k for k in range(8)]
    st.raw("s_cmp_eq_u64 s[48:49], 0")
    st.raw("s_cbranch_scc1 .Ldq256_ep_bf16")
    # fp32 partials (times scale): row qrow of this split, d = 32 i + 8 g + 4 hh + 0..3
    for i in range(8):
        for g in range(4):
            base = 16 * i + 4 * g
            for k in range(4):
                st.emit(f"v_accvgpr_read_b32 v{t[k]}, {A.r('acc', base + k)}")
            for k in range(4):
                st.emit(f"v_mul_f32 v{t[k]}, s42, v{t[k]}")
            st.emit(f"buffer_store_dwordx4 v[{t[0]}:{t[3]}], {V.r('stq')}, {RP}, 0 offen "
                    f"offset:{128 * i + 32 * g}")
    st.raw("s_branch .Ldq256_ep_done")
    st.label(".Ldq256_ep_bf16")
    for i in range(8):
        for g in range(4):
            base = 16 * i + 4 * g
            for k in range(4):
                st.emit(f"v_accvgpr_read_b32 v{t[k]}, {A.r('acc', base + k)}")
            for k in range(4):
                st.emit(f"v_mul_f32 v{t[k]}, s42, v{t[k]}")
            st.emit(f"v_cvt_pk_bf16_f32 v{t[4]}, v{t[0]}, v{t[1]}")
            st.emit(f"v_cvt_pk_bf16_f32 v{t[5]}, v{t[2]}, v{t[3]}")
            st.emit(f"buffer_store_dwordx2 v[{t[4]}:{t[5]}], {V.r('stq')}, {RDQ}, 0 offen "
                    f"offset:{64 * i + 16 * g}")
    st.label(".Ldq256_ep_done")


def gen_dq256():
    V, A = regs()
    st = Stream()
    prologue(st, V, A)
    st.label(".Ldq256_loop")
    for stage in range(NST):
        emit_body(st, V, A, stage)
    st.raw(f"s_sub_u32 {S_ITER}, {S_ITER}, 1")
    st.raw(f"s_cmp_lg_u32 {S_ITER}, 0")
    st.raw("s_cbranch_scc1 .Ldq256_loop")
    emit_tail(st, V, A)
    epilogue(st, V, A)
    k = kernel_text("vd_attn_bwd_dq_d256", st.text(), vgprs=V.next, agprs=A.next, sgprs=102,
                    lds_bytes=VBASE + NST * KTILE, kernarg_bytes=KARG, wg_size=64 * NW)
    data = "\n.rodata\n.p2align 8\nvd_attn_d256_lanes:\n"
    for row in lane_table():
        data += "\t.long " + ", ".join(str(x) for x in row) + "\n"
    return k, data, st
