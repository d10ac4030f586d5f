"""vd_attn_fwd_d256: hand-scheduled gfx950 forward of the head_dim-256 attention (reference
QKVAttentionLegacy.forward, unet.py:349-366 at C = 256: softmax(Q K^T / sqrt(D)) V), the
head_dim-64/128 forwards' algorithm (gen_fwd.py, gen_fwd128.py: lagged max, rare path) on the
head_dim-256 dQ kernel's data plan (gen_d256.py): 4 waves x 32 queries, ONE wave per SIMD,
32-key tiles, K tiles at u * 16 KiB and V tiles at 64 KiB + u * 16 KiB of a 4-stage ring
filled by LDS-DMA (tile t + 2 issued in body t, 4 K + 4 V pieces per wave), one barrier per
body.  At D = 256 a wave cannot hold its tile's K / V fragments: they stream just in time
through 8-slot rings (K rows two products ahead, V^T transposed fragments TR_AHEAD ahead).

Body t (ring stage u = t mod 4, score set par = u & 1):
    S(t) [16: S^T = K Q'^T - m over 16 head-dim k-steps, into set par] |
    check of tile t-1 | G(t-1) [16: O^T += V^T P^T over 8 output-dim blocks x 2 key k-steps]
with the softmax of tile t-1 (16 v_exp_f32, 2 row-sum chains, 8 v_cvt_pk_bf16_f32 into P^T,
keys >= the split's end masked to -inf in the last 128-key iteration) in the 16 gaps of the
S group, so its lagged-max check sits between the groups: a tile whose row sum reaches 2^16
(or inf, as the first tile does) calls the rare path (s_swappc, 4 variants by parity x
masking): recompute S(t-1) from the resident K tile, take the true max over both lane halves,
rescale O and l, redo tile t-1's softmax, and recompute S(t) against the new max -- before
G(t-1) reads P^T(t-1).  m starts at -inf (the -m splat at +inf), so tile 0 always takes it.

Key split (grid.z = sequences x 2^lsplit): split z takes keys [z kps, min(n, (z + 1) kps)),
its own iteration count and last-iteration mask, and with part != 0 writes its unnormalised
O (fp32) and (m, l) in attention.hip's FwdSplit layout for attn_fwd_combine_kernel
(part[z][seq][n][256], then ml[z][seq][n][2] at part + ml_off); at N = 16384 the query grid
alone is 128 workgroups, half the chip.
"""
from __future__ import annotations

from asmgen import Regs, Stream, kernel_text
from gen_d256 import KTILE, VBASE, swz, toff_bytes  # noqa: F401  (lane table: gen_d256)

MFMA = "v_mfma_f32_32x32x16_bf16"
NW = 4
D = 256
KT = 32
NST = 4
HI = 65536
KARG = 160               # AsmFwd256Args (vd_asm.h)
RING = 8                 # K row-fragment ring slots
TRING = 8                # V^T fragment ring slots (lo 2 + hi 2)
RD_AHEAD = 2             # K row fragments this many products ahead
TR_AHEAD = 5             # V^T fragments this many G products ahead
CHAINS = 2
DMA_AT = tuple(range(17, 32, 2))
NINF, PINF = "0xff800000", "0x7f800000"
CHECK_NOP = 3

# kernel arguments (AsmFwd256Args), s[16:55]:
#  0 q 8 k 16 v 24 o 32 lse                                   (u64)  s16..s25
#  40 n 44 ts_bytes 48 ots_bytes 52 groups                     (u32)  s26..s29
#  56 bs_bytes 64 gs_bytes 72 obs_bytes 80 ogs_bytes           (u64)  s30..s37
#  88 qscale 92 kv_bytes 96 o_bytes 100 tile_bytes 104 niter 108 klim0   s38..s43
#  112 part (u64) s44:45  120 kps s46  124 lsplit s47  128 split_bytes (u64) s48:49
#  136 ml_off (u64) s50:51  144 ml_split_bytes s52  148.. pad
S_KARG = "s[0:1]"
S_WGX, S_WGY, S_WGZ = "s2", "s3", "s4"
S_TAB = "s[6:7]"
S_Y0, S_Y1 = "s8", "s9"          # split key count, iterations
RQ, RK, RV, RO, RL = "s[56:59]", "s[60:63]", "s[64:67]", "s[68:71]", "s[72:75]"
S_WAVE, S_Q0, S_M0, S_ITER, S_SEQ, S_SPLIT, S_ZS, S_X = ("s76", "s77", "s78", "s79", "s80",
                                                          "s81", "s82", "s83")
S_ST, S_ST1, S_KB = "s84", "s85", "s86"
S_RET = "s[88:89]"
S_TGT = 90                        # s90..s97: the 4 rare-path entry points
S_T0, S_T1, S_T2, S_T3 = "s98", "s99", "s100", "s101"


def regs():
    V, A = Regs("v"), Regs("a")
    for name, n in (("tid", 1), ("lane", 1), ("rowoff", 8), ("troff", 8), ("rowhi", 8),
                    ("trhi", 8), ("dma", 4), ("sto", 1), ("stl", 1), ("klim", 1), ("ps", 1),
                    ("l", 1), ("m", 1), ("ninf", 1), ("tc", 2), ("c", CHAINS)):
        V.alloc(name, n)
    V.alloc("tmp", 4, 4)     # (64-bit aligned tuples)
    V.alloc("rt", 8, 4)
    V.alloc("sacc", 32, 16)  # S'^T [parity] x 16
    V.alloc("p", 8, 4)       # P^T as bf16 B operands [s2] x 4
    V.alloc("negm", 16, 4)   # -m splat (srcC of the first S MFMA)
    V.alloc("tr", 4 * TRING, 4)  # V^T fragment ring (lo 2 + hi 2)
    V.alloc("kr", 4 * RING, 4)   # K row-fragment ring
    A.alloc("qf", 64)        # Q' fragments [s]
    A.alloc("acc", 128)      # O^T accumulators [i]
    assert V.next <= 256 and A.next <= 256, (V.next, A.next)
    return V, A


def k_read(V, stage, s):
    """ds_read_b128 of K row fragment k-step s of the tile in `stage` into ring slot s % 8."""
    off = stage * KTILE + (256 if s >= 8 else 0)
    return (f"ds_read_b128 {V.r('kr', 4 * (s % RING), 4)}, {V.r('rowoff', s % 8)} offset:{off}",
            ("K", s))


def tr_read_pair(V, stage, j):
    """The lo / hi transposed reads of G product j = 2 i + s2 (output-dim block i, key k-step
    s2) of the V tile in `stage` (at +64 KiB: through the trhi copies) into ring slot j % 8."""
    i, s2 = j // 2, j % 2
    out = []
    for hi in range(2):
        off = stage * KTILE + (256 if i >= 4 else 0) + 8192 * s2
        assert off + 7934 < HI
        out.append((f"ds_read_b64_tr_b16 {V.r('tr', 4 * (j % TRING) + 2 * hi, 2)}, "
                    f"{V.r('trhi', 2 * (i % 4) + hi)} offset:{off}", ("T", j, hi)))
    return out


def s_mfmas(V, A, par, zero_c=False):
    out = []
    sv = V.r("sacc", 16 * par, 16)
    for s in range(16):
        c = ("0" if zero_c else V.r("negm", 0, 16)) if s == 0 else sv
        out.append((f"{MFMA} {sv}, {V.r('kr', 4 * (s % RING), 4)}, {A.r('qf', 4 * s, 4)}, {c}",
                    (("K", s),)))
    return out


def g_mfmas(V, A, deps=True):
    out = []
    for j in range(16):
        i, s2 = j // 2, j % 2
        acc = A.r("acc", 16 * i, 16)
        out.append((f"{MFMA} {acc}, {V.r('tr', 4 * (j % TRING), 4)}, {V.r('p', 4 * s2, 4)}, "
                    f"{acc}", (("T", j, 0), ("T", j, 1)) if deps else ()))
    return out


# ------------------------------------------------------------------ softmax stream
COST = {"exp": 8.0, "add": 4.0, "cvt": 4.5, "cmp": 4.0, "cnd": 4.0}


def mask_list(V, S, u):
    """Keys >= the split's end to -inf in the score block S of the tile in stage u of the last
    iteration (klim = keys in the last iteration - 4 hh)."""
    out = []
    for r in range(16):
        c = KT * u + (r & 3) + 8 * (r >> 2)
        out.append((f"v_cmp_lt_i32 vcc, {c}, {V.r('klim')}", COST["cmp"]))
        out.append((f"v_cndmask_b32 v{S + r}, {V.r('ninf')}, v{S + r}, vcc", COST["cnd"]))
    return out


def softmax_list(V, par, masked_u):
    """VALU of the softmax of the tile in score set `par`: exp2, CHAINS row-sum chains (4
    scores behind), cvt pairs into P^T, then the chains into ps.  masked_u: the tile's stage
    within the masked last iteration, or None."""
    S = V["sacc"] + 16 * par
    out = []
    if masked_u is not None:
        out += mask_list(V, S, masked_u)
    lag = 4
    for i in range(16 + lag):
        if i < 16:
            out.append((f"v_exp_f32 v{S + i}, v{S + i}", COST["exp"]))
        if i >= lag:
            r = i - lag
            c = V.r("c", r % CHAINS)
            if r < CHAINS:
                out.append((f"v_mov_b32 {c}, v{S + r}", COST["add"]))
            else:
                out.append((f"v_add_f32 {c}, {c}, v{S + r}", COST["add"]))
            if r % 2:
                out.append((f"v_cvt_pk_bf16_f32 {V.r('p', r // 2)}, v{S + r - 1}, v{S + r}",
                            COST["cvt"]))
    if CHAINS == 1:
        out.append((f"v_mov_b32 {V.r('ps')}, {V.r('c', 0)}", COST["add"]))
    else:
        out.append((f"v_add_f32 {V.r('ps')}, {V.r('c', 0)}, {V.r('c', 1)}", COST["add"]))
    return out


def place(items, ngaps):
    """Greedy list schedule by cost over ngaps gaps (gen_fwd.place without earliest gaps)."""
    total = sum(c for _, c in items)
    per = total / ngaps
    slots = [[] for _ in range(ngaps)]
    k = 0
    budget = 0.0
    for g in range(ngaps):
        budget += per
        while k < len(items) and (g == ngaps - 1 or items[k][1] <= budget + 1e-9):
            slots[g].append(items[k][0])
            budget -= items[k][1]
            k += 1
    assert k == len(items)
    return slots


# ------------------------------------------------------------------ prologue
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
    r("s_add_u32 s6, s6, vd_attn_d256_lanes@rel32@lo+4")
    r("s_addc_u32 s7, s7, vd_attn_d256_lanes@rel32@hi+12")
    r(f"s_getpc_b64 s[{S_TGT}:{S_TGT + 1}]")
    st.label(".Lfwd256_pc")
    for v in (3, 2, 1, 0):
        r(f"s_add_u32 s{S_TGT + 2 * v}, s{S_TGT}, .Lfwd256_rare{v}-.Lfwd256_pc")
        r(f"s_addc_u32 s{S_TGT + 2 * v + 1}, s{S_TGT + 1}, 0")
    r("s_waitcnt lgkmcnt(0)")
    # grid.z = (sequence group z') << lsplit | split
    r(f"s_lshl_b32 {S_X}, 1, s47")
    r(f"s_sub_u32 {S_X}, {S_X}, 1")
    r(f"s_and_b32 {S_SPLIT}, {S_WGZ}, {S_X}")
    r(f"s_lshr_b32 {S_ZS}, {S_WGZ}, s47")
    r(f"s_mul_i32 {S_SEQ}, {S_ZS}, s29")
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

    # q sequence base
    mad64(S_T0, S_T1, S_ZS, "s30", "s31")
    mad64(S_T2, S_T3, S_WGY, "s32", "s33")
    add64()
    rsrc(RQ, "s16", "s17", "s39")
    # K / V: the split's keys [split * kps, +keys): base += split * kps * ts_bytes, range
    # (keys - 1) * ts_bytes + 512; S_Y0 = keys of the split (> 0: host)
    r(f"s_mul_i32 {S_T2}, {S_SPLIT}, s46")
    r(f"s_sub_u32 {S_Y0}, s26, {S_T2}")
    r(f"s_min_u32 {S_Y0}, {S_Y0}, s46")
    r(f"s_sub_u32 {S_T3}, {S_Y0}, 1")
    r(f"s_mul_i32 {S_T3}, {S_T3}, s27")
    r(f"s_add_u32 {S_X}, {S_T3}, 512")
    r(f"s_mul_i32 {S_T2}, {S_T2}, s27")
    r(f"s_add_u32 {S_T0}, {S_T0}, {S_T2}")
    r(f"s_addc_u32 {S_T1}, {S_T1}, 0")
    r(f"s_mov_b32 {S_T3}, {S_X}")
    rsrc(RK, "s18", "s19", S_T3)
    rsrc(RV, "s20", "s21", S_T3)
    # iterations of 128 keys: S_Y1 = ceil(keys / 128); the loop runs S_Y1 - 1 of them, the
    # masked copy the last one (keys in it: keys - 128 (S_Y1 - 1))
    r(f"s_add_u32 {S_Y1}, {S_Y0}, 127")
    r(f"s_lshr_b32 {S_Y1}, {S_Y1}, 7")
    r(f"s_sub_u32 {S_ITER}, {S_Y1}, 1")
    r(f"s_lshl_b32 {S_X}, {S_ITER}, 7")
    r(f"s_sub_u32 {S_Y0}, {S_Y0}, {S_X}")     # keys in the last iteration
    # output: part != 0: fp32 O rows of the split (part + split * split_bytes + seq * n * 1024,
    # range n * 1024) and (m, l) rows (part + ml_off + split * ml_split_bytes + seq * n * 8);
    # else the bf16 O rows and the lse row of the sequence
    r("s_cmp_eq_u64 s[44:45], 0")
    r("s_cbranch_scc1 .Lfwd256_out_bf16")
    mad64(S_T0, S_T1, S_SPLIT, "s48", "s49")
    r(f"s_mul_i32 {S_T2}, {S_SEQ}, s26")
    r(f"s_mul_hi_u32 {S_T3}, {S_SEQ}, s26")
    r("s_lshl_b64 s[100:101], s[100:101], 10")
    add64()
    r(f"s_lshl_b32 {S_X}, s26, 10")
    rsrc(RO, "s44", "s45", S_X)
    r(f"s_mul_i32 {S_T0}, {S_SPLIT}, s52")
    r(f"s_mov_b32 {S_T1}, 0")
    r(f"s_add_u32 {S_T0}, {S_T0}, s50")
    r(f"s_addc_u32 {S_T1}, {S_T1}, s51")
    r(f"s_mul_i32 {S_T2}, {S_SEQ}, s26")
    r(f"s_mul_hi_u32 {S_T3}, {S_SEQ}, s26")
    r("s_lshl_b64 s[100:101], s[100:101], 3")
    add64()
    r(f"s_lshl_b32 {S_X}, s26, 3")
    rsrc(RL, "s44", "s45", S_X)
    r("s_branch .Lfwd256_out_done")
    st.label(".Lfwd256_out_bf16")
    mad64(S_T0, S_T1, S_ZS, "s34", "s35")
    mad64(S_T2, S_T3, S_WGY, "s36", "s37")
    add64()
    rsrc(RO, "s22", "s23", "s40")
    r(f"s_mul_i32 {S_T0}, {S_SEQ}, s26")
    r(f"s_mul_hi_u32 {S_T1}, {S_SEQ}, s26")
    r("s_lshl_b64 s[98:99], s[98:99], 2")
    r(f"s_lshl_b32 {S_X}, s26, 2")
    rsrc(RL, "s24", "s25", S_X)
    st.label(".Lfwd256_out_done")
    # q0 = wgx * 128 + wave * 32 ; M0 base of this wave's DMA pieces = wave * 4096
    r(f"s_lshl_b32 {S_Q0}, {S_WGX}, 7")
    r(f"s_lshl_b32 {S_X}, {S_WAVE}, 5")
    r(f"s_add_u32 {S_Q0}, {S_Q0}, {S_X}")
    r(f"s_lshl_b32 {S_M0}, {S_WAVE}, 12")
    t0, t1 = V.r("tmp", 0), V.r("tmp", 1)
    e(f"v_lshlrev_b32 {t0}, 7, {V.r('tid')}")
    r(f"global_load_dwordx4 {V.r('rowoff', 0, 4)}, {t0}, {S_TAB}")
    r(f"global_load_dwordx4 {V.r('rowoff', 4, 4)}, {t0}, {S_TAB} offset:16")
    r(f"global_load_dwordx4 {V.r('troff', 0, 4)}, {t0}, {S_TAB} offset:32")
    r(f"global_load_dwordx4 {V.r('troff', 4, 4)}, {t0}, {S_TAB} offset:48")
    r(f"global_load_dwordx4 {V.r('dma', 0, 4)}, {t0}, {S_TAB} offset:64")
    r(f"global_load_dwordx4 {V.r('rowhi', 0, 4)}, {t0}, {S_TAB} offset:80")  # chunks
    # the lane's query row (staging registers in rt)
    qrow, hh16, vq, h8 = (V.r("rt", k) for k in range(4))
    e(f"v_and_b32 {qrow}, 31, {V.r('lane')}")
    e(f"v_add_u32 {qrow}, {S_Q0}, {qrow}")
    e(f"v_lshrrev_b32 {hh16}, 5, {V.r('lane')}")
    e(f"v_lshlrev_b32 {hh16}, 4, {hh16}")
    e(f"v_lshrrev_b32 {h8}, 1, {hh16}")
    e(f"v_mul_lo_u32 {vq}, {qrow}, s27")
    e(f"v_add_u32 {vq}, {vq}, {hh16}")
    qv = V["tr"]   # Q staged in the V^T and K rings (64 contiguous VGPRs)
    assert V["kr"] == qv + 4 * TRING
    for s in range(16):
        r(f"buffer_load_dwordx4 v[{qv + 4 * s}:{qv + 4 * s + 3}], {vq}, {RQ}, 0 offen "
          f"offset:{32 * s}")
    # store offsets: part: O row qrow * 1024 + 16 hh, (m, l) at qrow * 8; bf16: O row
    # qrow * ots + 8 hh, lse at qrow * 4
    r("s_cmp_eq_u64 s[44:45], 0")
    r("s_cbranch_scc1 .Lfwd256_st_bf16")
    e(f"v_lshlrev_b32 {V.r('sto')}, 10, {qrow}")
    e(f"v_add_u32 {V.r('sto')}, {V.r('sto')}, {hh16}")
    e(f"v_lshlrev_b32 {V.r('stl')}, 3, {qrow}")
    r("s_branch .Lfwd256_st_done")
    st.label(".Lfwd256_st_bf16")
    e(f"v_mul_lo_u32 {V.r('sto')}, {qrow}, s28")
    e(f"v_add_u32 {V.r('sto')}, {V.r('sto')}, {h8}")
    e(f"v_lshlrev_b32 {V.r('stl')}, 2, {qrow}")
    st.label(".Lfwd256_st_done")
    # klim = keys in the last iteration - 4 hh
    e(f"v_lshrrev_b32 {t1}, 2, {hh16}")
    e(f"v_sub_u32 {V.r('klim')}, {S_Y0}, {t1}")
    r("s_waitcnt vmcnt(0)")
    # Q' = bf16(Q * scale * log2 e)
    for w in range(64):
        x = f"v{qv + w}"
        e(f"v_lshlrev_b32 {t0}, 16, {x}")
        e(f"v_and_b32 {t1}, 0xffff0000, {x}")
        e(f"v_mul_f32 {t0}, s38, {t0}")
        e(f"v_mul_f32 {t1}, s38, {t1}")
        e(f"v_cvt_pk_bf16_f32 {x}, {t0}, {t1}")
        e(f"v_accvgpr_write_b32 {A.r('qf', w)}, {x}")
    # DMA source offsets of tile 0: row * ts_bytes + chunk * 16
    for i in range(4):
        e(f"v_mul_lo_u32 {V.r('dma', i)}, {V.r('dma', i)}, s27")
        e(f"v_add_u32 {V.r('dma', i)}, {V.r('dma', i)}, {V.r('rowhi', i)}")
    for k in range(8):
        e(f"v_add_u32 {V.r('rowhi', k)}, {HI:#x}, {V.r('rowoff', k)}")
        e(f"v_add_u32 {V.r('trhi', k)}, {HI:#x}, {V.r('troff', k)}")
    # state: O = 0, l = 0, m = -inf (-m splat +inf); the first body's softmax (of "tile -1",
    # score set 1) sees -inf and yields P = 0 and a row sum 0, and its G reads stage 3's V
    # tile -- zeroed here, so no NaN bit pattern meets the zero P
    for k in range(128):
        e(f"v_accvgpr_write_b32 {A.r('acc', k)}, 0")
    for k in range(4):
        e(f"v_mov_b32 {V.r('tmp', k)}, 0")
    e(f"v_lshlrev_b32 {V.r('rt', 4)}, 6, {V.r('tid')}")
    e(f"v_add_u32 {V.r('rt', 5)}, {VBASE:#x}, {V.r('rt', 4)}")
    for k in range(4):   # stage 3's V tile (at +64 KiB): 256 lanes x 64 B
        e(f"ds_write_b128 {V.r('rt', 5)}, {V.r('tmp', 0, 4)} offset:{3 * KTILE + 16 * k}")
    for k in range(8):
        e(f"v_mov_b32 {V.r('p', k)}, 0")
    for k in range(16):
        e(f"v_mov_b32 {V.r('negm', k)}, {PINF}")
        e(f"v_mov_b32 {V.r('sacc', 16 + k)}, {NINF}")
    e(f"v_mov_b32 {V.r('m')}, {NINF}")
    e(f"v_mov_b32 {V.r('l')}, 0")
    e(f"v_mov_b32 {V.r('ninf')}, {NINF}")
    for t in range(2):
        ops, adv = dma_ops(V, t)
        for m0, ld in ops:
            r(m0)
            r("s_nop 0")
            e(ld)
        for a in adv:
            e(a)


def dma_ops(V, stage):
    ops = []
    for x, rs in ((0, RK), (VBASE, RV)):
        for i in range(4):
            ops.append((f"s_add_u32 m0, {S_M0}, {x + stage * KTILE + i * 1024}",
                        f"buffer_load_dwordx4 {V.r('dma', i)}, {rs}, 0 offen lds"))
    adv = [f"v_add_u32 {V.r('dma', i)}, s41, {V.r('dma', i)}" for i in range(4)]
    return ops, adv


# ------------------------------------------------------------------ one body
def emit_check(st: Stream, V, u, masked, tag):
    """Lagged-max check of tile t-1 (its row sums in ps): any lane >= 2^16 (or inf / NaN) ->
    the rare path; then l += ps."""
    par = u & 1
    st.emit(f"v_cmp_ngt_f32 vcc, 0x47800000, {V.r('ps')}")
    st.raw(f"s_nop {CHECK_NOP}")
    st.raw(f"s_cbranch_vccz .Lfwd256_ok{tag}")
    st.raw(f"s_mov_b32 {S_ST}, {((u + 3) % NST) * KTILE}")
    st.raw(f"s_mov_b32 {S_ST1}, {u * KTILE}")
    st.raw(f"s_mov_b32 {S_KB}, {KT * ((u + 3) % NST)}")
    v = 2 * int(masked) + par
    st.raw(f"s_swappc_b64 {S_RET}, s[{S_TGT + 2 * v}:{S_TGT + 2 * v + 1}]")
    st.label(f".Lfwd256_ok{tag}")
    st.emit(f"v_add_f32 {V.r('l')}, {V.r('l')}, {V.r('ps')}")


def emit_body(st: Stream, V, A, u, masked_soft, tag, dma=True):
    """Body t in ring stage u: S(t) | check(t-1) | G(t-1); masked_soft: the softmax of tile
    t-1 (stage u-1 of the last iteration) masks keys past the split's end."""
    par, prev = u & 1, (u + 3) % NST
    st.comment(f"---- key tile, ring stage {u}{' (softmax masked)' if masked_soft else ''}")
    st.raw("s_waitcnt vmcnt(8) lgkmcnt(0)")
    st.raw("s_barrier")
    st.flush_lds()
    mf_s = s_mfmas(V, A, par)
    mf_g = g_mfmas(V, A)
    slots = {}

    def at(g, item):
        slots.setdefault(g, []).append(item)

    for s in range(16):
        at(max(0, s - RD_AHEAD), k_read(V, u, s))
    for j in range(16):
        for item in tr_read_pair(V, prev, j):
            at(16 + j - TR_AHEAD, item)
    valu = place(softmax_list(V, 1 - par, prev if masked_soft else None), 16)
    ops, adv = dma_ops(V, (u + 2) % NST)
    mf = mf_s + mf_g
    for g in range(32):
        if g == 16:
            emit_check(st, V, u, masked_soft, tag)
        if dma and g in DMA_AT:
            m0, ld = ops[DMA_AT.index(g)]
            st.raw(m0)
            st.raw("s_nop 0")
            st.emit(ld)
            if g == DMA_AT[-1]:
                for a in adv:
                    st.emit(a)
        for text, rid in slots.get(g, []):
            st.emit(text, lds_id=rid)
        if g < 16:
            for text in valu[g]:
                st.emit(text)
        text, deps = mf[g]
        st.emit(text, wait_lds=deps)


def emit_tail(st: Stream, V, A):
    """After the last tile T-1 (stage 3, score set 1, masked): its softmax, check and G."""
    st.comment("---- tail: softmax, check and PV products of the last tile")
    st.raw("s_waitcnt lgkmcnt(0)")
    st.flush_lds()
    for text, _ in softmax_list(V, 1, 3):
        st.emit(text)
    # the rare path's S(t) recompute reads stage 0 (junk, unused); its parity is 0 here
    emit_check(st, V, 0, True, "tail")
    g = g_mfmas(V, A)
    for j in range(16):
        for text, rid in tr_read_pair(V, 3, j):
            st.emit(text, lds_id=rid)
        text, deps = g[j]
        st.emit(text, wait_lds=deps)


def epilogue(st: Stream, V, A):
    e = st.emit
    st.raw("s_waitcnt vmcnt(0)")
    t = [V["sacc"] + k for k in range(8)]
    ad, lx, inv, lg = V["sacc"] + 8, V["sacc"] + 9, V["sacc"] + 10, V["sacc"] + 11
    # each lane half summed its own 16 keys of every tile
    e(f"v_xor_b32 v{ad}, 32, {V.r('lane')}")
    e(f"v_lshlrev_b32 v{ad}, 2, v{ad}")
    e(f"ds_bpermute_b32 v{lx}, v{ad}, {V.r('l')}")
    st.raw("s_waitcnt lgkmcnt(0)")
    e(f"v_add_f32 {V.r('l')}, {V.r('l')}, v{lx}")
    st.raw("s_cmp_eq_u64 s[44:45], 0")
    st.raw("s_cbranch_scc1 .Lfwd256_ep_bf16")
    # split: unnormalised fp32 O rows, then (m, l) -- both lane halves store the same pair
    for i in range(8):
        for g in range(4):
            for k in range(4):
                e(f"v_accvgpr_read_b32 v{t[k]}, {A.r('acc', 16 * i + 4 * g + k)}")
            e(f"buffer_store_dwordx4 v[{t[0]}:{t[3]}], {V.r('sto')}, {RO}, 0 offen "
              f"offset:{128 * i + 32 * g}")
    e(f"v_mov_b32 v{t[4]}, {V.r('m')}")
    e(f"v_mov_b32 v{t[5]}, {V.r('l')}")
    e(f"buffer_store_dwordx2 v[{t[4]}:{t[5]}], {V.r('stl')}, {RL}, 0 offen")
    st.raw("s_branch .Lfwd256_ep_done")
    st.label(".Lfwd256_ep_bf16")
    e(f"v_rcp_f32 v{inv}, {V.r('l')}")
    for i in range(8):
        for g in range(4):
            for k in range(4):
                e(f"v_accvgpr_read_b32 v{t[k]}, {A.r('acc', 16 * i + 4 * g + k)}")
            for k in range(4):
                e(f"v_mul_f32 v{t[k]}, v{inv}, v{t[k]}")
            e(f"v_cvt_pk_bf16_f32 v{t[4]}, v{t[0]}, v{t[1]}")
            e(f"v_cvt_pk_bf16_f32 v{t[5]}, v{t[2]}, v{t[3]}")
            e(f"buffer_store_dwordx2 v[{t[4]}:{t[5]}], {V.r('sto')}, {RO}, 0 offen "
              f"offset:{64 * i + 16 * g}")
    # lse = (m + log2 l) * ln 2
    e(f"v_log_f32 v{lg}, {V.r('l')}")
    e(f"v_add_f32 v{lg}, {V.r('m')}, v{lg}")
    e(f"v_mul_f32 v{lg}, 0x3f317218, v{lg}")
    e(f"buffer_store_dword v{lg}, {V.r('stl')}, {RL}, 0 offen")
    st.label(".Lfwd256_ep_done")


# ------------------------------------------------------------------ the rare path
def rare_path(V, A, par, masked):
    """Subroutine .Lfwd256_rare{2 masked + par} for tile t-1 (score set 1 - par) inside body t
    (score set par): S_ST / S_ST1 = ring offsets of the K tiles of t-1 / t, S_KB = tile t-1's
    first key within the last iteration; returns through S_RET."""
    st = Stream()
    e, r = st.emit, st.raw
    q = 1 - par
    st.label(f".Lfwd256_rare{2 * int(masked) + par}")
    r("s_nop 15")
    r("s_nop 15")
    r("s_waitcnt lgkmcnt(0)")

    def reads_from(sreg):
        ta = [V.r("rt", k) for k in range(8)]
        for k in range(8):
            e(f"v_add_u32 {ta[k]}, {sreg}, {V.r('rowoff', k)}")
        out = []
        for s in range(16):
            out.append((f"ds_read_b128 {V.r('kr', 4 * (s % RING), 4)}, {ta[s % 8]} "
                        f"offset:{256 if s >= 8 else 0}", ("K", s)))
        return out

    def s_group(sreg, set_, zero_c):
        reads = reads_from(sreg)
        mf = s_mfmas(V, A, set_, zero_c=zero_c)
        for s in range(16):
            if s == 0:
                for k in range(min(RING, 16)):
                    e(reads[k][0], lds_id=reads[k][1])
            elif s + RING - 1 < 16:
                e(reads[s + RING - 1][0], lds_id=reads[s + RING - 1][1])
            text, deps = mf[s]
            e(text, wait_lds=deps)
        st.flush_lds()
        r("s_nop 15")
        r("s_nop 15")

    s_group(S_ST, q, True)  # S(t-1) without -m
    S = V["sacc"] + 16 * q
    if masked:
        vl = V.r("tc", 1)
        e(f"v_subrev_u32 {vl}, {S_KB}, {V.r('klim')}")
        for rr in range(16):
            c = (rr & 3) + 8 * (rr >> 2)
            e(f"v_cmp_lt_i32 vcc, {c}, {vl}")
            e(f"v_cndmask_b32 v{S + rr}, {V.r('ninf')}, v{S + rr}, vcc")
    mx, oth, ad, alpha = (V.r("tmp", k) for k in range(4))
    e(f"v_max3_f32 {mx}, v{S}, v{S + 1}, v{S + 2}")
    for k in range(3, 15, 2):
        e(f"v_max3_f32 {mx}, {mx}, v{S + k}, v{S + k + 1}")
    e(f"v_max_f32 {mx}, {mx}, v{S + 15}")
    e(f"v_xor_b32 {ad}, 32, {V.r('lane')}")
    e(f"v_lshlrev_b32 {ad}, 2, {ad}")
    e(f"ds_bpermute_b32 {oth}, {ad}, {mx}")
    r("s_waitcnt lgkmcnt(0)")
    m, l = V.r("m"), V.r("l")
    e(f"v_max_f32 {mx}, {mx}, {oth}")
    e(f"v_max_f32 {mx}, {m}, {mx}")                  # m_new
    e(f"v_sub_f32 {alpha}, {m}, {mx}")
    e(f"v_exp_f32 {alpha}, {alpha}")                 # exp2(m - m_new)
    e(f"v_cmp_eq_f32 vcc, {m}, {mx}")                # equal (also -inf == -inf)
    e(f"v_cndmask_b32 {alpha}, {alpha}, 1.0, vcc")
    e(f"v_mov_b32 {m}, {mx}")
    e(f"v_mul_f32 {l}, {alpha}, {l}")
    e(f"v_xor_b32 {oth}, 0x80000000, {mx}")
    for k in range(16):
        e(f"v_mov_b32 {V.r('negm', k)}, {oth}")
    tmp = [V.r("rt", k) for k in range(4)]
    for i in range(8):
        for g in range(4):
            base = 16 * i + 4 * g
            for k in range(4):
                e(f"v_accvgpr_read_b32 {tmp[k]}, {A.r('acc', base + k)}")
            for k in range(4):
                e(f"v_mul_f32 {tmp[k]}, {alpha}, {tmp[k]}")
            for k in range(4):
                e(f"v_accvgpr_write_b32 {A.r('acc', base + k)}, {tmp[k]}")
    # tile t-1's softmax against m_new (one row-sum chain)
    for k in range(16):
        e(f"v_sub_f32 v{S + k}, v{S + k}, {mx}")
    ps = V.r("ps")
    for k in range(8):
        a, b = S + 2 * k, S + 2 * k + 1
        e(f"v_exp_f32 v{a}, v{a}")
        e(f"v_exp_f32 v{b}, v{b}")
        if k == 0:
            e(f"v_add_f32 {ps}, v{a}, v{b}")
        else:
            e(f"v_add_f32 {ps}, {ps}, v{a}")
            e(f"v_add_f32 {ps}, {ps}, v{b}")
        e(f"v_cvt_pk_bf16_f32 {V.r('p', k)}, v{a}, v{b}")
    # S(t) against m_new
    s_group(S_ST1, par, False)
    r(f"s_setpc_b64 {S_RET}")
    return st


def gen_fwd256():
    V, A = regs()
    st = Stream()
    prologue(st, V, A)
    st.raw(f"s_cmp_eq_u32 {S_ITER}, 0")
    st.raw("s_cbranch_scc1 .Lfwd256_last")
    st.label(".Lfwd256_loop")
    for u in range(NST):
        emit_body(st, V, A, u, False, f"{u}")
    st.raw(f"s_sub_u32 {S_ITER}, {S_ITER}, 1")
    st.raw(f"s_cmp_lg_u32 {S_ITER}, 0")
    st.raw("s_cbranch_scc1 .Lfwd256_loop")
    st.label(".Lfwd256_last")
    for u in range(NST):
        emit_body(st, V, A, u, u > 0, f"m{u}")
    emit_tail(st, V, A)
    epilogue(st, V, A)
    body = st.text() + "\ts_endpgm\n"
    for masked in (False, True):
        for par in range(2):
            body += rare_path(V, A, par, masked).text()
    k = kernel_text("vd_attn_fwd_d256", body, vgprs=V.next, agprs=A.next, sgprs=102,
                    lds_bytes=VBASE + NST * KTILE, kernarg_bytes=KARG, wg_size=64 * NW)
    return k, st
