"""Hand-scheduled gfx950 head_dim-256 attention backward, dK / dV (reference
QKVAttentionLegacy, unet.py:349-366, at C = 256: the 32x32 level of the config-2 UNet3D).

vd_attn_bwd_dkdv_d256 -- the role-split arithmetic of attention.hip's
attn_bwd_dkdv_role_kernel<256, 4> (S' = Q K'^T - lse' and dP = dO V^T - delta with the query
on the accumulator rows and the key on the lane, P = exp2(S'), dS = P * dP, dV^T += dO^T P,
dK^T += Q^T dS, K' = K * scale * log2 e in bf16), hand-placed.  At head_dim 256 one wave
cannot hold K', V and BOTH full-width accumulator sets of its 32 keys (64 + 64 + 128 + 128
registers), so the keys of a workgroup are owned by wave PAIRS: role A (waves 0, 1) keeps
K' and dV^T, role B (waves 2, 3) keeps V and dK^T of the same 32 keys (pair p = wave & 1:
keys wgx * 64 + 32 p + lane).  Per 32-query tile t (one 32-row block) each wave runs 32
v_mfma_f32_32x32x16_bf16:
    A: S(t) [16] | dV(t-1) [16]     -- exp2(S(t)) and its bf16 pack in the dV gaps, then
                                       P(t) (fp32) to the pair's LDS exchange slot
    B: dP(t) [16] | dK(t-1) [16]    -- dS(t-1) = P(t-1) * dP(t-1) in the dP gaps (P(t-1)
                                       read from the slot A wrote before this tile's barrier)
The query rows of S / dP are streamed from the tile's ring stage through 8-slot AGPR rings
(16 ds_read_b128 each), the transposed dO / Q fragments of the G products from the previous
tile's stage through 8-slot rings (32 ds_read_b64_tr_b16 each).

LDS: 4 ring stages x (Q tile 16 KiB | dO tile 16 KiB) = 128 KiB by LDS-DMA (tile t + 2
issued in tile t: 8 pieces per wave -- A waves the Q rows, B waves the dO rows -- and one
row-constant piece: lse' (A pair 0), delta (B pair 0), or a junk slot), the row constants
(4 x 768 B) and the P exchange (2 parities x 2 pairs x 4 KiB): 147 KiB.  One barrier per tile
behind s_waitcnt vmcnt(9); the loop is unrolled by the 4 stages; query rows past the range
are zero rows (the buffer range check) whose products add nothing to dK / dV.

Query split (grid.z = sequences x 2^lsplit): split z takes queries [z qps, (z + 1) qps) and,
with part != 0, writes fp32 partials part[z][seq][nkv][dK 256 | dV 256] that attention.hip's
attn_dkdv_sum_kernel adds.
"""
from __future__ import annotations

from asmgen import Regs, Stream, kernel_text
from gen_d256 import swz, toff_bytes

MFMA = "v_mfma_f32_32x32x16_bf16"
NW = 4
D = 256
STAGE = 32768           # Q tile | dO tile (32 x 256 bf16 each)
OOFF = 16384
NST = 4
HI = 65536
RC_BASE = NST * STAGE   # 131072: per stage lse' (256 B) | delta (256 B) | junk (256 B)
RC = 768
PX_BASE = RC_BASE + NST * RC   # P exchange [parity][pair] x 4 KiB
PX = 4096
LDS_BYTES = PX_BASE + 4 * PX
KARG = 176              # AsmDkdv256Args (vd_asm.h)
RING = 8                # row-fragment ring slots (4 registers each)
TRING = 8               # transposed-fragment ring slots (4 registers each: lo 2 + hi 2)
RD_AHEAD = 4            # row fragments this many MFMAs ahead
TR_AHEAD = 4            # transposed fragments this many MFMAs ahead
DMA_AT = (1, 4, 7, 10, 13, 19, 22, 25, 28)   # the 9 DMA ops of a tile

# kernel arguments (AsmDkdv256Args), s[16:59]:
#  0 q 8 k 16 v 24 dout 32 nlse2 40 ndelta 48 dk 56 dv          (u64)  s16..s31
#  64 n 68 ts_bytes 72 ots_bytes 76 groups                         s32..s35
#  80 bs 88 gs 96 obs 104 ogs (bytes, u64)                         s36..s43
#  112 scale 116 kscale 120 kv_bytes 124 o_bytes 128 tile_bytes 132 otile_bytes 136 niter
#  140 pad                                                         s44..s51
#  144 part (u64) s52:53  152 qps s54  156 lsplit s55  160 split_bytes (u64) s56:57
#  168 part_bytes s58  172 pad s59
S_KARG = "s[0:1]"
S_WGX, S_WGY, S_WGZ = "s2", "s3", "s4"
R_DMA, R_RC, R_OUT, R_KV = "s[60:63]", "s[64:67]", "s[68:71]", "s[72:75]"
S_WAVE, S_K0, S_M0, S_ITER, S_RCM0, S_SEQ, S_ZS, S_SPLIT, S_X, S_PAIR = (
    "s76", "s77", "s78", "s79", "s80", "s81", "s82", "s83", "s84", "s85")
S_T0, S_T1, S_T2, S_T3 = "s86", "s87", "s88", "s89"   # two aligned pairs
S_TAB = "s[90:91]"


def lane_table():
    """tab[wave][lane][32] u32: 0-7 row-fragment offsets (k-steps 0..7; +8: +256 B), 8-15
    transposed-fragment offsets (2 i + hi, i = 0..3; i + 4: +256 B; k-step s2: +8192 B),
    16-23 the DMA rows of the wave's 8 pieces of a tile (pair p: pieces 8 p .. 8 p + 7 of the
    wave's tile half), 24-31 their source chunk * 16."""
    out = []
    for w in range(NW):
        pair = w & 1
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
            for i in range(8):
                gi = pair * 8 + i
                rr = gi * 2 + lane // 32
                drow.append(rr)
                dch.append(((lane % 32) ^ swz(rr)) * 16)
            out.append(row + tr + drow + dch)
    return out


def common_regs():
    V, A = Regs("v"), Regs("a")
    for name, n in (("tid", 1), ("lane", 1), ("rowoff", 8), ("troff", 8), ("rowhi", 8),
                    ("trhi", 8), ("dma", 8), ("rcv", 1), ("rcoff", 1), ("pxoff", 1),
                    ("stk", 1), ("tmp", 4)):
        V.alloc(name, n)
    return V, A


def regs_a():
    V, A = common_regs()
    V.alloc("sacc", 16, 16)  # S' of the current tile
    V.alloc("pbf", 16)       # P as bf16 B operands [parity][s2] x 4
    V.alloc("il", 16)        # -lse' of the tile's query rows (srcC of S)
    V.alloc("kst", 64)       # prologue: K fragments staged for the scaling
    A.alloc("kf", 64)        # K' fragments [s]
    A.alloc("adv", 128)      # dV^T accumulators [i]
    A.alloc("rr", 4 * RING)  # Q row-fragment ring
    A.alloc("tr", 4 * TRING)  # dO^T fragment ring
    assert V.next <= 256 and A.next <= 256, (V.next, A.next)
    return V, A


def regs_b():
    V, A = common_regs()
    V.alloc("dpacc", 32, 16)  # dP [parity] x 16
    V.alloc("pf", 16)        # P (fp32) of the previous tile, from the exchange slot
    V.alloc("dsb", 8)        # dS as bf16 B operands [s2] x 4
    V.alloc("id", 16)        # -delta of the tile's query rows (srcC of dP)
    A.alloc("vf", 64)        # V fragments [s]
    A.alloc("adk", 128)      # dK^T accumulators [i]
    A.alloc("rr", 4 * RING)  # dO row-fragment ring
    A.alloc("tr", 4 * TRING)  # Q^T fragment ring
    assert V.next <= 256 and A.next <= 256, (V.next, A.next)
    return V, A


def lds(V, base, k, off):
    if off >= HI:
        return V.r({"rowoff": "rowhi", "troff": "trhi"}[base], k), off - HI
    return V.r(base, k), off


def row_read(V, A, stage, s, half):
    """Row fragment of k-step s of the Q (half 0) / dO (half 1) tile into ring slot s % 8."""
    off = stage * STAGE + half * OOFF + (256 if s >= 8 else 0)
    b, o = lds(V, "rowoff", s % 8, off)
    return (f"ds_read_b128 {A.r('rr', 4 * (s % RING), 4)}, {b} offset:{o}", ("R", s))


def tr_read_pair(V, A, stage, j, half):
    """The two transposed reads (lo / hi rows) of G product j = 2 i + s2 (output-dim block
    i, query k-step s2) of the Q (0) / dO (1) tile into ring slot j % 8."""
    i, s2 = j // 2, j % 2
    out = []
    for hi in range(2):
        off = stage * STAGE + half * OOFF + (256 if i >= 4 else 0) + 8192 * s2
        b, o = lds(V, "troff", 2 * (i % 4) + hi, off)
        out.append((f"ds_read_b64_tr_b16 {A.r('tr', 4 * (j % TRING) + 2 * hi, 2)}, {b} "
                    f"offset:{o}", ("T", j, hi)))
    return out


def rc_reads(V, stage, which, dst):
    """-lse' (which 0) / -delta (1) of the tile's 32 query rows: register 4 g + e = row
    8 g + 4 hh + e."""
    return [(f"ds_read_b128 {V.r(dst, 4 * g, 4)}, {V.r('rcoff')} offset:"
             f"{stage * RC + 256 * which + 32 * g}", ("C", g)) for g in range(4)]


def dma_ops(V, stage, half, _unused, rc_rs):
    """The wave's 9 DMA ops of one tile: its 8 row pieces of the Q (half 0) / dO (1) tile
    into `stage`, then its row-constant piece (rc_slot 0 lse', 1 delta, 2 junk)."""
    ops = []
    for i in range(8):
        ops.append((f"s_add_u32 m0, {S_M0}, {stage * STAGE + half * OOFF + i * 1024}",
                    f"buffer_load_dwordx4 {V.r('dma', i)}, {R_DMA}, 0 offen lds"))
    ops.append((f"s_add_u32 m0, {S_RCM0}, {RC_BASE + stage * RC}",
                f"buffer_load_dword {V.r('rcv')}, {rc_rs}, 0 offen lds"))
    tb = "s48" if half == 0 else "s49"
    adv = [f"v_add_u32 {V.r('dma', i)}, {tb}, {V.r('dma', i)}" for i in range(8)]
    adv.append(f"v_add_u32 {V.r('rcv')}, 0x80, {V.r('rcv')}")
    return ops, adv


# ------------------------------------------------------------------ prologue
def prologue_common(st: Stream, V):
    e, r = st.emit, st.raw
    r(f"s_load_dwordx16 s[16:31], {S_KARG}, 0x0")
    r(f"s_load_dwordx16 s[32:47], {S_KARG}, 0x40")
    r(f"s_load_dwordx8 s[48:55], {S_KARG}, 0x80")
    r(f"s_load_dwordx4 s[56:59], {S_KARG}, 0xa0")
    e(f"v_and_b32 {V.r('lane')}, 63, {V.r('tid')}")
    r(f"v_readfirstlane_b32 {S_WAVE}, {V.r('tid')}")
    r("s_nop 1")
    r(f"s_lshr_b32 {S_WAVE}, {S_WAVE}, 6")
    r(f"s_and_b32 {S_PAIR}, {S_WAVE}, 1")
    r(f"s_getpc_b64 {S_TAB}")
    r("s_add_u32 s90, s90, vd_attn_d256dk_lanes@rel32@lo+4")
    r("s_addc_u32 s91, s91, vd_attn_d256dk_lanes@rel32@hi+12")
    r("s_waitcnt lgkmcnt(0)")
    r(f"s_lshl_b32 {S_X}, 1, s55")
    r(f"s_sub_u32 {S_X}, {S_X}, 1")
    r(f"s_and_b32 {S_SPLIT}, {S_WGZ}, {S_X}")
    r(f"s_lshr_b32 {S_ZS}, {S_WGZ}, s55")
    r(f"s_mul_i32 {S_SEQ}, {S_ZS}, s35")
    r(f"s_add_u32 {S_SEQ}, {S_SEQ}, {S_WGY}")
    # k0 = wgx * 64 + pair * 32; M0 base of the wave's row pieces: pair * 8 KiB
    r(f"s_lshl_b32 {S_K0}, {S_WGX}, 6")
    r(f"s_lshl_b32 {S_X}, {S_PAIR}, 5")
    r(f"s_add_u32 {S_K0}, {S_K0}, {S_X}")
    r(f"s_lshl_b32 {S_M0}, {S_PAIR}, 13")
    r(f"s_mov_b32 {S_ITER}, s50")
    t0 = V.r("tmp", 0)
    e(f"v_lshlrev_b32 {t0}, 7, {V.r('tid')}")
    r(f"global_load_dwordx4 {V.r('rowoff', 0, 4)}, {t0}, {S_TAB}")
    r(f"global_load_dwordx4 {V.r('rowoff', 4, 4)}, {t0}, {S_TAB} offset:16")
    r(f"global_load_dwordx4 {V.r('troff', 0, 4)}, {t0}, {S_TAB} offset:32")
    r(f"global_load_dwordx4 {V.r('troff', 4, 4)}, {t0}, {S_TAB} offset:48")
    r(f"global_load_dwordx4 {V.r('dma', 0, 4)}, {t0}, {S_TAB} offset:64")
    r(f"global_load_dwordx4 {V.r('dma', 4, 4)}, {t0}, {S_TAB} offset:80")
    r(f"global_load_dwordx4 {V.r('rowhi', 0, 4)}, {t0}, {S_TAB} offset:96")   # chunks
    r(f"global_load_dwordx4 {V.r('rowhi', 4, 4)}, {t0}, {S_TAB} offset:112")
    # per-lane constant offsets: row constants (16 hh), P exchange (pair slot, lane * 16)
    e(f"v_lshrrev_b32 {V.r('rcoff')}, 5, {V.r('lane')}")
    e(f"v_lshlrev_b32 {V.r('rcoff')}, 4, {V.r('rcoff')}")
    e(f"v_lshlrev_b32 {V.r('pxoff')}, 4, {V.r('lane')}")
    r(f"s_lshl_b32 {S_X}, {S_PAIR}, 12")
    r(f"s_add_u32 {S_X}, {S_X}, {PX_BASE}")
    e(f"v_add_u32 {V.r('pxoff')}, {S_X}, {V.r('pxoff')}")
    e(f"v_lshlrev_b32 {V.r('rcv')}, 2, {V.r('lane')}")


def seq_bases(st: Stream, half):
    """S_T0:T1 = the byte offset of this sequence's (and query split's) Q (half 0) / dO (1)
    rows; S_X = the row range of the split (queries - 1) * stride + 512."""
    r = st.raw
    bsl, bsh, gsl, gsh, ts = (("s36", "s37", "s38", "s39", "s33") if half == 0 else
                              ("s40", "s41", "s42", "s43", "s34"))
    r(f"s_mul_i32 {S_T0}, {S_ZS}, {bsl}")
    r(f"s_mul_hi_u32 {S_T1}, {S_ZS}, {bsl}")
    r(f"s_mul_i32 {S_X}, {S_ZS}, {bsh}")
    r(f"s_add_u32 {S_T1}, {S_T1}, {S_X}")
    r(f"s_mul_i32 {S_T2}, {S_WGY}, {gsl}")
    r(f"s_mul_hi_u32 {S_T3}, {S_WGY}, {gsl}")
    r(f"s_mul_i32 {S_X}, {S_WGY}, {gsh}")
    r(f"s_add_u32 {S_T3}, {S_T3}, {S_X}")
    r(f"s_add_u32 {S_T0}, {S_T0}, {S_T2}")
    r(f"s_addc_u32 {S_T1}, {S_T1}, {S_T3}")


def rsrc(st, dst, plo, phi, nrec):
    r = st.raw
    d0 = int(dst[2:].split(":")[0])
    r(f"s_add_u32 s{d0}, {plo}, {S_T0}")
    r(f"s_addc_u32 s{d0 + 1}, {phi}, {S_T1}")
    r(f"s_and_b32 s{d0 + 1}, s{d0 + 1}, 0xffff")
    r(f"s_mov_b32 s{d0 + 2}, {nrec}")
    r(f"s_mov_b32 s{d0 + 3}, 0x20000")


def prologue_role(st: Stream, V, A, role):
    """Role A (0): K' fragments, Q DMA, lse' row constants, dV output; role B (1): V, dO,
    delta, dK.  Ends with tiles 0 and 1 in flight and the zeroed tile -1 published."""
    e, r = st.emit, st.raw
    half = role
    ts = "s33" if role == 0 else "s34"
    # this sequence's K / V rows (the keys are not split)
    seq_bases(st, 0)
    rsrc(st, R_KV, "s18" if role == 0 else "s20", "s19" if role == 0 else "s21", "s46")
    # output rows: bf16 dK / dV of the sequence, or the fp32 partials of the split
    r("s_cmp_eq_u64 s[52:53], 0")
    r(f"s_cbranch_scc0 .Ldk256_{role}_part")
    rsrc(st, R_OUT, "s30" if role == 0 else "s28", "s31" if role == 0 else "s29", "s46")
    r(f"s_branch .Ldk256_{role}_out")
    st.label(f".Ldk256_{role}_part")
    r(f"s_mul_i32 {S_T0}, {S_SPLIT}, s56")
    r(f"s_mul_hi_u32 {S_T1}, {S_SPLIT}, s56")
    r(f"s_mul_i32 {S_X}, {S_SPLIT}, s57")
    r(f"s_add_u32 {S_T1}, {S_T1}, {S_X}")
    r(f"s_mul_i32 {S_T2}, {S_SEQ}, s32")      # seq * nkv rows of 2 KiB
    r(f"s_mul_hi_u32 {S_T3}, {S_SEQ}, s32")
    r("s_lshl_b64 s[88:89], s[88:89], 11")
    r(f"s_add_u32 {S_T0}, {S_T0}, {S_T2}")
    r(f"s_addc_u32 {S_T1}, {S_T1}, {S_T3}")
    rsrc(st, R_OUT, "s52", "s53", "s58")
    st.label(f".Ldk256_{role}_out")
    # the split's Q / dO rows: base + split * qps * stride, range (queries - 1) * stride + 512
    seq_bases(st, half)
    r(f"s_mul_i32 {S_T2}, {S_SPLIT}, s54")       # first query of the split
    r(f"s_sub_u32 {S_T3}, s32, {S_T2}")
    r(f"s_min_u32 {S_T3}, {S_T3}, s54")          # queries of the split (> 0: host)
    r(f"s_mul_i32 {S_T2}, {S_T2}, {ts}")
    r(f"s_add_u32 {S_T0}, {S_T0}, {S_T2}")
    r(f"s_addc_u32 {S_T1}, {S_T1}, 0")
    r(f"s_sub_u32 {S_X}, {S_T3}, 1")
    r(f"s_mul_i32 {S_X}, {S_X}, {ts}")
    r(f"s_add_u32 {S_X}, {S_X}, 512")
    rsrc(st, R_DMA, "s16" if role == 0 else "s22", "s17" if role == 0 else "s23", S_X)
    # row constants of the split: (seq * n + split * qps) * 4, range queries * 4; pair 1
    # waves DMA theirs into the junk slot
    r(f"s_lshl_b32 {S_X}, {S_T3}, 2")
    r(f"s_mul_i32 {S_T0}, {S_SEQ}, s32")
    r(f"s_mul_i32 {S_T2}, {S_SPLIT}, s54")
    r(f"s_add_u32 {S_T0}, {S_T0}, {S_T2}")
    r(f"s_mov_b32 {S_T1}, 0")
    r(f"s_lshl_b64 s[86:87], s[86:87], 2")
    rsrc(st, R_RC, "s24" if role == 0 else "s26", "s25" if role == 0 else "s27", S_X)
    r(f"s_movk_i32 {S_RCM0}, 0x200")
    r(f"s_cmp_eq_u32 {S_PAIR}, 0")
    r(f"s_cselect_b32 {S_RCM0}, {256 * role}, {S_RCM0}")
    # K' (scaled) / V fragments of the lane's key
    krow, hh16, vk, h8 = (V.r("tmp", k) for k in range(4))
    e(f"v_and_b32 {krow}, 31, {V.r('lane')}")
    e(f"v_add_u32 {krow}, {S_K0}, {krow}")
    e(f"v_lshrrev_b32 {hh16}, 5, {V.r('lane')}")
    e(f"v_lshlrev_b32 {hh16}, 4, {hh16}")
    e(f"v_mul_lo_u32 {vk}, {krow}, s33")
    e(f"v_add_u32 {vk}, {vk}, {hh16}")
    frag = "kf" if role == 0 else "vf"
    # staged in VGPRs above the common block (scaled for K'), then moved to the AGPRs
    stage0 = V["kst"] if role == 0 else None
    if role == 0:
        for s in range(16):
            r(f"buffer_load_dwordx4 v[{stage0 + 4 * s}:{stage0 + 4 * s + 3}], {vk}, {R_KV}, 0 "
              f"offen offset:{32 * s}")
    else:
        for s in range(16):
            r(f"buffer_load_dwordx4 {A.r(frag, 4 * s, 4)}, {vk}, {R_KV}, 0 offen "
              f"offset:{32 * s}")
    # store offsets: bf16 row key * ts + 8 hh, or partial row key * 2048 (+1024 for dV) + 16 hh
    e(f"v_lshrrev_b32 {h8}, 1, {hh16}")
    r("s_cmp_eq_u64 s[52:53], 0")
    r(f"s_cbranch_scc1 .Ldk256_{role}_bst")
    e(f"v_lshlrev_b32 {V.r('stk')}, 11, {krow}")
    e(f"v_add_u32 {V.r('stk')}, {V.r('stk')}, {hh16}")
    if role == 0:
        e(f"v_add_u32 {V.r('stk')}, 0x400, {V.r('stk')}")
    r(f"s_branch .Ldk256_{role}_sdone")
    st.label(f".Ldk256_{role}_bst")
    e(f"v_mul_lo_u32 {V.r('stk')}, {krow}, s33")
    e(f"v_add_u32 {V.r('stk')}, {V.r('stk')}, {h8}")
    st.label(f".Ldk256_{role}_sdone")
    r("s_waitcnt vmcnt(0)")
    if role == 0:
        t0, t1 = V.r("tmp", 0), V.r("tmp", 1)
        for w in range(64):
            x = f"v{stage0 + w}"
            e(f"v_lshlrev_b32 {t0}, 16, {x}")
            e(f"v_and_b32 {t1}, 0xffff0000, {x}")
            e(f"v_mul_f32 {t0}, s45, {t0}")
            e(f"v_mul_f32 {t1}, s45, {t1}")
            e(f"v_cvt_pk_bf16_f32 {x}, {t0}, {t1}")
            e(f"v_accvgpr_write_b32 {A.r('kf', w)}, {x}")
    # DMA source offsets of tile 0 (rows * stride + chunk), the +64 KiB offset copies
    for i in range(8):
        e(f"v_mul_lo_u32 {V.r('dma', i)}, {V.r('dma', i)}, {ts}")
        e(f"v_add_u32 {V.r('dma', i)}, {V.r('dma', i)}, {V.r('rowhi', i)}")
    for k in range(8):
        e(f"v_add_u32 {V.r('rowhi', k)}, {HI:#x}, {V.r('rowoff', k)}")
        e(f"v_add_u32 {V.r('trhi', k)}, {HI:#x}, {V.r('troff', k)}")
    e(f"v_add_u32 {V.r('rcoff')}, {RC_BASE:#x}, {V.r('rcoff')}")
    # zero the accumulators and the G operands of tile -1 (pbf / dsb), then put tiles 0 and 1
    # in flight
    acc = "adv" if role == 0 else "adk"
    for k in range(128):
        e(f"v_accvgpr_write_b32 {A.r(acc, k)}, 0")
    if role == 0:
        for k in range(16):
            e(f"v_mov_b32 {V.r('pbf', k)}, 0")
            e(f"v_mov_b32 {V.r('sacc', k)}, 0")
    else:
        for k in range(32):
            e(f"v_mov_b32 {V.r('dpacc', k)}, 0")
        for k in range(8):
            e(f"v_mov_b32 {V.r('dsb', k)}, 0")
    for t in range(2):
        ops, adv = dma_ops(V, t, half, None, R_RC)
        for m0, ld in ops:
            r(m0)
            r("s_nop 0")
            e(ld)
        for a in adv:
            e(a)


def zero_lds(st: Stream, V):
    """Zero ring stage 3 (tile -1: the transposed operands of the first G products, 32 KiB)
    and the P exchange (16 KiB; the first B body reads "P(-1)"): 8 + 4 ds_write_b128 per
    lane.  Runs before the role split, before the first barrier."""
    e = st.emit
    for k in range(4):
        e(f"v_mov_b32 {V.r('tmp', k)}, 0")
    b = V.r("stk")   # scratch here; the store offset is set later
    e(f"v_lshlrev_b32 {b}, 7, {V.r('tid')}")
    e(f"v_add_u32 {b}, {3 * STAGE:#x}, {b}")
    for k in range(8):
        e(f"ds_write_b128 {b}, {V.r('tmp', 0, 4)} offset:{16 * k}")
    e(f"v_lshlrev_b32 {b}, 6, {V.r('tid')}")
    e(f"v_add_u32 {b}, {PX_BASE:#x}, {b}")
    for k in range(4):
        e(f"ds_write_b128 {b}, {V.r('tmp', 0, 4)} offset:{16 * k}")


def emit_body_a(st: Stream, V, A, stage):
    """A, tile t in `stage` (par = stage & 1): S(t) | dV(t-1)."""
    par, prev = stage & 1, (stage + 3) % NST
    st.comment(f"---- A: query tile, ring stage {stage}")
    st.raw("s_waitcnt vmcnt(9) lgkmcnt(0)")
    st.raw("s_barrier")
    st.flush_lds()
    if stage == 0:  # loop back edge: the last MFMAs of the previous stage-3 body
        st.raw("s_nop 12", ws=13)
    mf = []
    for s in range(16):
        c = V.r("il", 0, 16) if s == 0 else V.r("sacc", 0, 16)
        mf.append((f"{MFMA} {V.r('sacc', 0, 16)}, {A.r('rr', 4 * (s % RING), 4)}, "
                   f"{A.r('kf', 4 * s, 4)}, {c}",
                   (("R", s),) + (tuple(("C", g) for g in range(4)) if s == 0 else ())))
    for j in range(16):
        i, s2 = j // 2, j % 2
        mf.append((f"{MFMA} {A.r('adv', 16 * i, 16)}, {A.r('tr', 4 * (j % TRING), 4)}, "
                   f"{V.r('pbf', 8 * (1 - par) + 4 * s2, 4)}, {A.r('adv', 16 * i, 16)}",
                   (("T", j, 0), ("T", j, 1))))
    slots = {}

    def at(g, item):
        slots.setdefault(g, []).append(item)

    for item in rc_reads(V, stage, 0, "il"):
        at(0, item)
    for s in range(16):
        at(max(0, s - RD_AHEAD), row_read(V, A, stage, s, 0))
    for j in range(16):
        for item in tr_read_pair(V, A, prev, j, 1):
            at(16 + j - TR_AHEAD, item)
    # exp2, the bf16 pack of P(t), then P(t) (fp32) to the exchange slot [par][pair]
    vl = []
    for k in range(8):
        a, b = 2 * k, 2 * k + 1
        vl += [(f"v_exp_f32 v{V['sacc'] + a}, v{V['sacc'] + a}", None),
               (f"v_exp_f32 v{V['sacc'] + b}, v{V['sacc'] + b}", None),
               (f"v_cvt_pk_bf16_f32 {V.r('pbf', 8 * par + k)}, v{V['sacc'] + a}, "
                f"v{V['sacc'] + b}", None)]
    for g in range(4):
        vl.append((f"ds_write_b128 {V.r('pxoff')}, {V.r('sacc', 4 * g, 4)} "
                   f"offset:{par * 2 * PX + g * 1024}", None))
    for k, item in enumerate(vl):
        at(17 + (k * 14) // len(vl), item)
    ops, adv = dma_ops(V, (stage + 2) % NST, 0, None, R_RC)
    emit_slots(st, mf, slots, ops, adv)


def emit_body_b(st: Stream, V, A, stage):
    """B, tile t in `stage` (par = stage & 1): dP(t) | dK(t-1); dS(t-1) in the dP gaps."""
    par, prev = stage & 1, (stage + 3) % NST
    st.comment(f"---- B: query tile, ring stage {stage}")
    st.raw("s_waitcnt vmcnt(9) lgkmcnt(0)")
    st.raw("s_barrier")
    st.flush_lds()
    if stage == 0:
        st.raw("s_nop 12", ws=13)
    mf = []
    dcur = V.r("dpacc", 16 * par, 16)
    for s in range(16):
        c = V.r("id", 0, 16) if s == 0 else dcur
        mf.append((f"{MFMA} {dcur}, {A.r('rr', 4 * (s % RING), 4)}, "
                   f"{A.r('vf', 4 * s, 4)}, {c}",
                   (("R", s),) + (tuple(("C", g) for g in range(4)) if s == 0 else ())))
    for j in range(16):
        i, s2 = j // 2, j % 2
        mf.append((f"{MFMA} {A.r('adk', 16 * i, 16)}, {A.r('tr', 4 * (j % TRING), 4)}, "
                   f"{V.r('dsb', 4 * s2, 4)}, {A.r('adk', 16 * i, 16)}",
                   (("T", j, 0), ("T", j, 1))))
    slots = {}

    def at(g, item):
        slots.setdefault(g, []).append(item)

    # P(t-1) from the exchange slot [1 - par][pair] first, then the row constants and rows
    for g in range(4):
        at(0, (f"ds_read_b128 {V.r('pf', 4 * g, 4)}, {V.r('pxoff')} "
               f"offset:{(1 - par) * 2 * PX + g * 1024}", ("P", g)))
    for item in rc_reads(V, stage, 1, "id"):
        at(0, item)
    for s in range(16):
        at(max(0, s - RD_AHEAD), row_read(V, A, stage, s, 1))
    for j in range(16):
        for item in tr_read_pair(V, A, prev, j, 0):
            at(16 + j - TR_AHEAD, item)
    # dS(t-1) = P(t-1) * dP(t-1), packed to bf16, in gaps 2..14
    dprev = V["dpacc"] + 16 * (1 - par)
    vl = []
    for k in range(8):
        a, b = 2 * k, 2 * k + 1
        vl += [(f"v_mul_f32 v{dprev + a}, v{dprev + a}, v{V['pf'] + a}", ("P", a // 4)),
               (f"v_mul_f32 v{dprev + b}, v{dprev + b}, v{V['pf'] + b}", ("P", b // 4)),
               (f"v_cvt_pk_bf16_f32 {V.r('dsb', k)}, v{dprev + a}, v{dprev + b}", None)]
    for k, item in enumerate(vl):
        at(2 + (k * 12) // len(vl), item)
    ops, adv = dma_ops(V, (stage + 2) % NST, 1, None, R_RC)
    emit_slots(st, mf, slots, ops, adv)


def emit_slots(st: Stream, mf, slots, ops, adv):
    for g in range(len(mf)):
        if g in DMA_AT:
            m0, ld = ops[DMA_AT.index(g)]
            st.raw(m0)
            st.raw("s_nop 0")
            st.emit(ld)
            if g == DMA_AT[-1]:
                for a in adv:
                    st.emit(a)
        for text, rid in slots.get(g, []):
            if rid is not None and rid[0] in ("R", "T", "C") or (rid is not None and rid[0] == "P"
                                                                   and text.startswith("ds_read")):
                st.emit(text, lds_id=rid)
            elif rid is not None:      # a VALU consumer of an LDS read
                st.emit(text, wait_lds=(rid,))
            else:
                st.emit(text)
        text, deps = mf[g]
        st.emit(text, wait_lds=deps)


def emit_tail(st: Stream, V, A, role):
    """After the last tile T-1 (stage 3, parity 1): A runs dV(T-1); B waits for A's P(T-1)
    (the barrier pairs with A's), forms dS(T-1) and runs dK(T-1)."""
    st.comment(f"---- tail ({'A' if role == 0 else 'B'})")
    st.raw("s_waitcnt lgkmcnt(0)")
    st.raw("s_barrier")
    st.flush_lds()
    items = []
    for j in range(16):
        items += tr_read_pair(V, A, 3, j, 1 - role)
    if role == 0:
        for j in range(16):
            for text, rid in tr_read_pair(V, A, 3, j, 1):
                st.emit(text, lds_id=rid)
            i, s2 = j // 2, j % 2
            st.emit(f"{MFMA} {A.r('adv', 16 * i, 16)}, {A.r('tr', 4 * (j % TRING), 4)}, "
                    f"{V.r('pbf', 8 + 4 * s2, 4)}, {A.r('adv', 16 * i, 16)}",
                    wait_lds=(("T", j, 0), ("T", j, 1)))
        return
    for g in range(4):
        st.emit(f"ds_read_b128 {V.r('pf', 4 * g, 4)}, {V.r('pxoff')} offset:{2 * PX + g * 1024}",
                lds_id=("P", g))
    dprev = V["dpacc"] + 16
    for k in range(8):
        a, b = 2 * k, 2 * k + 1
        st.emit(f"v_mul_f32 v{dprev + a}, v{dprev + a}, v{V['pf'] + a}", wait_lds=(("P", a // 4),))
        st.emit(f"v_mul_f32 v{dprev + b}, v{dprev + b}, v{V['pf'] + b}", wait_lds=(("P", b // 4),))
        st.emit(f"v_cvt_pk_bf16_f32 {V.r('dsb', k)}, v{dprev + a}, v{dprev + b}")
    for j in range(16):
        for text, rid in tr_read_pair(V, A, 3, j, 0):
            st.emit(text, lds_id=rid)
        i, s2 = j // 2, j % 2
        st.emit(f"{MFMA} {A.r('adk', 16 * i, 16)}, {A.r('tr', 4 * (j % TRING), 4)}, "
                f"{V.r('dsb', 4 * s2, 4)}, {A.r('adk', 16 * i, 16)}",
                wait_lds=(("T", j, 0), ("T", j, 1)))


def epilogue(st: Stream, V, A, role):
    """dV (A) / dK * scale (B) of the lane's key: bf16 rows, or fp32 partial rows."""
    st.raw("s_waitcnt vmcnt(0)")
    acc = "adv" if role == 0 else "adk"
    t = [V["tmp"] + k for k in range(4)] + [V["rcv"], V["rcoff"]]
    st.raw("s_cmp_eq_u64 s[52:53], 0")
    st.raw(f"s_cbranch_scc1 .Ldk256_{role}_ebf")
    for i in range(8):
        for g in range(4):
            for k in range(4):
                st.emit(f"v_accvgpr_read_b32 v{t[k]}, {A.r(acc, 16 * i + 4 * g + k)}")
            if role == 1:
                for k in range(4):
                    st.emit(f"v_mul_f32 v{t[k]}, s44, v{t[k]}")
            st.emit(f"buffer_store_dwordx4 v[{t[0]}:{t[3]}], {V.r('stk')}, {R_OUT}, 0 offen "
                    f"offset:{128 * i + 32 * g}")
    st.raw(f"s_branch .Ldk256_{role}_edone")
    st.label(f".Ldk256_{role}_ebf")
    for i in range(8):
        for g in range(4):
            for k in range(4):
                st.emit(f"v_accvgpr_read_b32 v{t[k]}, {A.r(acc, 16 * i + 4 * g + k)}")
            if role == 1:
                for k in range(4):
                    st.emit(f"v_mul_f32 v{t[k]}, s44, v{t[k]}")
            st.emit(f"v_cvt_pk_bf16_f32 v{t[4]}, v{t[0]}, v{t[1]}")
            st.emit(f"v_cvt_pk_bf16_f32 v{t[5]}, v{t[2]}, v{t[3]}")
            st.emit(f"buffer_store_dwordx2 v[{t[4]}:{t[5]}], {V.r('stk')}, {R_OUT}, 0 offen "
                    f"offset:{64 * i + 16 * g}")
    st.label(f".Ldk256_{role}_edone")


def gen_dkdv256():
    VA, AA = regs_a()
    VB, AB = regs_b()
    st = Stream()
    prologue_common(st, VA)
    zero_lds(st, VA)
    st.raw(f"s_cmp_ge_u32 {S_WAVE}, 2")
    st.raw("s_cbranch_scc1 .Ldk256_role_b")
    for role, (V, A, body) in enumerate(((VA, AA, emit_body_a), (VB, AB, emit_body_b))):
        if role == 1:
            st.label(".Ldk256_role_b")
            st.flush_lds()
        prologue_role(st, V, A, role)
        st.label(f".Ldk256_{role}_loop")
        for stage in range(NST):
            body(st, V, A, stage)
        st.raw(f"s_sub_u32 {S_ITER}, {S_ITER}, 1")
        st.raw(f"s_cmp_lg_u32 {S_ITER}, 0")
        st.raw(f"s_cbranch_scc1 .Ldk256_{role}_loop")
        emit_tail(st, V, A, role)
        epilogue(st, V, A, role)
        if role == 0:
            st.raw("s_endpgm")
    vg = max(VA.next, VB.next)
    ag = max(AA.next, AB.next)
    k = kernel_text("vd_attn_bwd_dkdv_d256", st.text(), vgprs=vg, agprs=ag, sgprs=92,
                    lds_bytes=LDS_BYTES, kernarg_bytes=KARG, wg_size=64 * NW)
    data = "\n.rodata\n.p2align 8\nvd_attn_d256dk_lanes:\n"
    for row in lane_table():
        data += "\t.long " + ", ".join(str(x) for x in row) + "\n"
    return k, data, st
