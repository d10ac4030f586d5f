"""Generate attn_asm.s: hand-scheduled gfx950 kernels for the head_dim-64 attention
backward (reference QKVAttentionLegacy.forward, unet.py:349-366, and its autograd backward).

    python gen_attn_asm.py OUT.s [--report]

vd_attn_bwd_dq_d64 -- dQ of one sequence block: the same arithmetic as
attn_bwd_dq_pipe_kernel<bf16, 64> in attention.hip (S'^T = K Q'^T - lse', dP^T = V dO^T -
delta, dS^T = exp2(S'^T) * dP^T, dQ^T += K^T dS^T, Q' = Q * scale * log2 e in bf16), laid
out for ONE wave per SIMD instead of two: 4 waves x 64 queries per workgroup, 256 queries
per workgroup, the whole 512-entry register file per wave (VGPRs hold what the VALU
touches, AGPRs the MFMA-only operands and the dQ accumulators).

Per 64-key tile a wave runs 48 v_mfma_f32_32x32x16_bf16 (S and dP for 2 key blocks x 2
query blocks, and the dQ products of the PREVIOUS tile) and 160 VALU instructions (64
v_exp_f32, 64 v_mul_f32, 32 v_cvt_pk_bf16_f32).  The generator fixes the MFMA order and
places the VALU stream at a constant rate (10 instructions per 3 MFMA gaps, about 19 of
the 24 issue cycles a gap leaves free) starting START gaps after the tile's first score
block completes; LDS fragment reads go 2 per gap ahead of their MFMAs with counted
lgkmcnt waits; the 4 LDS-DMA pieces per tile are spread over 4 gaps.  The VALU stream of
tile t runs into the first gaps of tile t+1 (the registers are per score-block slot, so
the loop body is the same every iteration).

Ring: 4 stages x (K tile 8 KiB | V tile 8 KiB) = 64 KiB of LDS, filled by
buffer_load ... lds (tile t + 2 issued after the barrier of tile t), one s_barrier per
tile behind s_waitcnt vmcnt(4).  The loop is unrolled by the 4 stages, so every LDS
address is a per-lane constant (a table in .rodata, computed here with the formulas of
attention.hip's toff / mma_rows / mma_tr / dma_tile) plus an immediate.
"""
from __future__ import annotations

import sys

from asmgen import Regs, Stream, code_object_text, kernel_text

MFMA = "v_mfma_f32_32x32x16_bf16"
NW = 4            # waves per workgroup
QPW = 64          # queries per wave (2 blocks of 32)
STAGE = 16384     # bytes per ring stage: K tile | V tile (64 x 64 bf16 each)
VOFF = 8192       # V tile offset in a stage
START = 18        # first VALU gap of a tile's score blocks (after MFMA START)


# ------------------------------------------------------------------ lane tables
def swz(r):
    """attention.hip swz_row<64>."""
    return (((r >> 1) & 1) << 2) | ((r >> 2) & 3)


def toff_bytes(r, c):
    """attention.hip toff<bf16, 64>(r, c) in bytes."""
    return 2 * (r * 64 + (((c >> 3) ^ swz(r)) << 3) + (c & 7))


def lane_table():
    """tab[wave][lane][16] u32: 0-3 mma_rows offsets (s = 0..3, block row 0), 4-7 mma_tr
    offsets (i * 2 + hi; col0 = 32 i, sum0 = 0, s2 = 0), 8-9 DMA row in the tile and 10-11
    its source chunk * 16 (pieces i = 0, 1 of dma_tile<64, 4>)."""
    out = []
    for w in range(NW):
        for lane in range(64):
            r, hh = lane & 31, lane >> 5
            row = [toff_bytes(r, 16 * s + 8 * hh) for s in range(4)]
            g, fr = lane >> 4, lane & 15
            q4, p4 = fr >> 2, fr & 3
            tr = []
            for i in range(2):
                col = 32 * i + 16 * (g & 1) + 4 * p4
                kr = 4 * (g >> 1) + q4
                tr += [toff_bytes(kr, col), toff_bytes(kr + 8, col)]
            dma_row, dma_c = [], []
            for i in range(2):
                gi = w * 2 + i
                rr = gi * 8 + lane // 8
                dma_row.append(rr)
                dma_c.append(((lane % 8) ^ swz(rr)) * 16)
            out.append(row + tr + dma_row + dma_c + [0, 0, 0, 0])
    return out


# ------------------------------------------------------------------ register plan
def regs_dq():
    V, A = Regs("v"), Regs("a")
    V.alloc("tid", 1)
    V.alloc("lane", 1)
    V.alloc("rowoff", 4)
    V.alloc("troff", 4)
    V.alloc("dma", 2)       # DMA voffsets of the next tile to issue (pieces 0, 1)
    V.alloc("dmac", 2)      # (prologue) the pieces' source chunk * 16
    V.alloc("tmp", 4)
    V.alloc("stq", 2)       # per query block: qrow * ts_bytes + 8 hh (dQ stores)
    V.alloc("tmp2", 2)
    V.alloc("sacc", 64, 16)  # S' blocks, 4 slots p = 2 kb + j
    V.alloc("dpacc", 64)     # dP blocks
    V.alloc("ds", 32)        # dS^T as bf16 B operands, 8 per slot
    V.alloc("il", 32)        # -lse' splats (srcC of the first S MFMA), per query block
    V.alloc("id", 32)        # -delta splats
    A.alloc("qf", 32)        # Q' fragments [j][s]
    A.alloc("of", 32)        # dO fragments [j][s]
    A.alloc("acc", 64)       # dQ^T accumulators [i][j]
    A.alloc("kf", 32)        # K row fragments [buf = kb][s]
    A.alloc("vf", 32)        # V row fragments [kb][s]
    A.alloc("trf", 32)       # K^T fragments [kb][i][s2] (lo 2 + hi 2)
    return V, A


def sacc(V, p):
    return V.r("sacc", 16 * p, 16)


def dpacc(V, p):
    return V.r("dpacc", 16 * p, 16)


# SGPR map
S_KARG = "s[0:1]"
S_WGX, S_WGY, S_WGZ = "s2", "s3", "s4"
# kernel arguments (s_load into s[16:47]), byte offsets in the 128-B kernarg block:
#  0 q  8 k  16 v  24 dout  32 nlse2  40 ndelta  48 dq   (u64)
#  56 n  60 ts_bytes  64 ots_bytes  68 groups            (u32)
#  72 bs_bytes  80 gs_bytes  88 obs_bytes  96 ogs_bytes  (u64)
#  104 scale  108 qscale (= scale * log2 e)              (f32)
#  112 kv_bytes  116 o_bytes  120 tile_bytes  124 niter  (u32)
KARG_BYTES = 128
RQ, RK, RV, RO, RL, RD, RDQ = "s[56:59]", "s[60:63]", "s[64:67]", "s[68:71]", "s[72:75]", \
    "s[76:79]", "s[80:83]"
S_WAVE, S_Q0, S_M0, S_ITER, S_TAB = "s84", "s85", "s86", "s87", "s[88:89]"


def prologue_dq(st: Stream, V, A):
    e, r = st.emit, st.raw
    r(f"s_load_dwordx16 s[16:31], {S_KARG}, 0x0")
    r(f"s_load_dwordx16 s[32:47], {S_KARG}, 0x40")
    e(f"v_and_b32 {V.r('lane')}, 63, {V.r('tid')}")
    r(f"v_readfirstlane_b32 {S_WAVE}, {V.r('tid')}")  # first lane's id = 64 * wave
    r("s_nop 1")
    r(f"s_lshr_b32 {S_WAVE}, {S_WAVE}, 6")
    r("s_getpc_b64 s[88:89]")
    r("s_add_u32 s88, s88, vd_attn_dq_lanes@rel32@lo+4")
    r("s_addc_u32 s89, s89, vd_attn_dq_lanes@rel32@hi+12")
    r("s_waitcnt lgkmcnt(0)")
    # seq = wgz * groups + wgy ; base = wgz * bs + wgy * gs ; obase likewise (bytes, 64-bit)
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

    rsrc(RQ, "s16", "s17", "s50", "s51", "s44")
    rsrc(RK, "s18", "s19", "s50", "s51", "s44")
    rsrc(RV, "s20", "s21", "s50", "s51", "s44")
    rsrc(RO, "s22", "s23", "s52", "s53", "s45")
    rsrc(RDQ, "s28", "s29", "s50", "s51", "s44")
    # row constants: seq * n * 4 bytes into nlse2 / ndelta
    r("s_mul_i32 s92, s48, s30")
    r("s_mul_hi_u32 s93, s48, s30")
    r("s_lshl_b64 s[92:93], s[92:93], 2")
    r("s_lshl_b32 s94, s30, 2")
    rsrc(RL, "s24", "s25", "s92", "s93", "s94")
    rsrc(RD, "s26", "s27", "s92", "s93", "s94")
    # q0 = wgx * 256 + wave * 64 ; M0 base of this wave's DMA pieces = wave * 2048
    r(f"s_lshl_b32 {S_Q0}, {S_WGX}, 8")
    r(f"s_lshl_b32 s90, {S_WAVE}, 6")
    r(f"s_add_u32 {S_Q0}, {S_Q0}, s90")
    r(f"s_lshl_b32 {S_M0}, {S_WAVE}, 11")
    r(f"s_mov_b32 {S_ITER}, s47")
    # lane table: tid * 64 bytes
    t0, t1, t2, t3 = (V.r("tmp", i) for i in range(4))
    e(f"v_lshlrev_b32 {t0}, 6, {V.r('tid')}")
    r(f"global_load_dwordx4 {V.r('rowoff', 0, 4)}, {t0}, {S_TAB}")
    r(f"global_load_dwordx4 {V.r('troff', 0, 4)}, {t0}, {S_TAB} offset:16")
    r(f"global_load_dwordx4 v[{V['dma']}:{V['dma'] + 3}], {t0}, {S_TAB} offset:32")
    # per query block j: qrow = q0 + 32 j + (lane & 31); hh = lane >> 5
    qrow = [V.r("sacc", 60), V.r("sacc", 61)]
    hh16 = V.r("sacc", 62)
    e(f"v_and_b32 {qrow[0]}, 31, {V.r('lane')}")
    e(f"v_add_u32 {qrow[0]}, {S_Q0}, {qrow[0]}")
    e(f"v_add_u32 {qrow[1]}, 32, {qrow[0]}")
    e(f"v_lshrrev_b32 {hh16}, 5, {V.r('lane')}")
    e(f"v_lshlrev_b32 {hh16}, 4, {hh16}")
    # Q and dO fragments: [j][s] = row qrow_j, elements 16 s + 8 hh (bytes: 32 s + 16 hh)
    qv = V["sacc"]  # Q fragments staged in VGPRs v[sacc .. +31] for scaling
    for j in range(2):
        vq = V.r("dpacc", 60 + j)
        e(f"v_mul_lo_u32 {vq}, {qrow[j]}, s31")
        e(f"v_add_u32 {vq}, {vq}, {hh16}")
        for s in range(4):
            r(f"buffer_load_dwordx4 v[{qv + 16 * j + 4 * s}:{qv + 16 * j + 4 * s + 3}], {vq}, "
              f"{RQ}, 0 offen offset:{32 * s}")
        vo = V.r("dpacc", 62 + j)
        e(f"v_mul_lo_u32 {vo}, {qrow[j]}, s32")
        e(f"v_add_u32 {vo}, {vo}, {hh16}")
        for s in range(4):
            r(f"buffer_load_dwordx4 {A.r('of', 16 * j + 4 * s, 4)}, {vo}, {RO}, 0 offen "
              f"offset:{32 * s}")
        # row constants of the lane's query
        vl = V.r("dpacc", 58 + j)
        e(f"v_lshlrev_b32 {vl}, 2, {qrow[j]}")
        r(f"buffer_load_dword {V.r('tmp2', j)}, {vl}, {RL}, 0 offen")
        r(f"buffer_load_dword {V.r('dpacc', 56 + j)}, {vl}, {RD}, 0 offen")
        # dQ store offsets: qrow * ts_bytes + 8 hh
        e(f"v_lshrrev_b32 {V.r('dpacc', 54)}, 1, {hh16}")
        e(f"v_mul_lo_u32 {V.r('stq', j)}, {qrow[j]}, s31")
        e(f"v_add_u32 {V.r('stq', j)}, {V.r('stq', j)}, {V.r('dpacc', 54)}")
    r("s_waitcnt vmcnt(0)")
    # Q' = bf16(Q * scale * log2 e), per bf16 element (attention.hip RowFrag::scale)
    for w in range(32):
        x = f"v{qv + w}"
        e(f"v_lshlrev_b32 {t0}, 16, {x}")
        e(f"v_and_b32 {t1}, 0xffff0000, {x}")
        e(f"v_mul_f32 {t0}, s43, {t0}")
        e(f"v_mul_f32 {t1}, s43, {t1}")
        e(f"v_cvt_pk_bf16_f32 {x}, {t0}, {t1}")
        e(f"v_accvgpr_write_b32 {A.r('qf', w)}, {x}")
    # srcC splats: il[j] = -lse' (nlse2), id[j] = -delta (ndelta)
    for j in range(2):
        for k in range(16):
            e(f"v_mov_b32 {V.r('il', 16 * j + k)}, {V.r('tmp2', j)}")
            e(f"v_mov_b32 {V.r('id', 16 * j + k)}, {V.r('dpacc', 56 + j)}")
    # DMA source offsets of tile 0: row * ts_bytes + chunk * 16
    d0, d1 = V["dma"], V["dma"] + 1
    for i in range(2):
        e(f"v_mul_lo_u32 v{d0 + i}, v{d0 + i}, s31")
        e(f"v_add_u32 v{d0 + i}, v{d0 + i}, v{d0 + 2 + i}")
    # zero: accumulators, dS operands, score blocks (the first tile's VALU of "tile -1"
    # then produces exact zeros), and ring stage 3 (tile -1 of the first dQ products)
    for k in range(64):
        e(f"v_accvgpr_write_b32 {A.r('acc', k)}, 0")
    for k in range(32):  # K^T fragments of "tile -1" (the first tile's dQ products)
        e(f"v_accvgpr_write_b32 {A.r('trf', k)}, 0")
    for k in range(32):
        e(f"v_mov_b32 {V.r('ds', k)}, 0")
    for k in range(64):
        e(f"v_mov_b32 {V.r('sacc', k)}, 0")
        e(f"v_mov_b32 {V.r('dpacc', k)}, 0")
    for k in range(4):
        e(f"v_mov_b32 {V.r('tmp', k)}, 0")
    e(f"v_lshlrev_b32 {V.r('tmp2', 0)}, 6, {V.r('tid')}")
    for k in range(4):
        e(f"ds_write_b128 {V.r('tmp2', 0)}, {V.r('tmp', 0, 4)} offset:{3 * STAGE + 16 * k}")
    r("s_waitcnt lgkmcnt(0)")
    # ring fill: tiles 0 and 1
    for t in range(2):
        dma_issue(st, V, t)


def dma_issue(st: Stream, V, stage):
    """The wave's 4 LDS-DMA pieces of the next tile into `stage`, then advance the offsets."""
    d0 = V["dma"]
    for x, rs in ((0, RK), (1, RV)):
        for i in range(2):
            st.raw(f"s_add_u32 m0, {S_M0}, {stage * STAGE + x * VOFF + i * 1024}")
            st.raw("s_nop 0")
            st.emit(f"buffer_load_dwordx4 v{d0 + i}, {rs}, 0 offen lds")
    for i in range(2):
        st.emit(f"v_add_u32 v{d0 + i}, s46, v{d0 + i}")


# ------------------------------------------------------------------ the tile body
def valu_stream(V):
    """The 160 VALU instructions of one tile: per score-block slot p, 16 x (exp2 of S',
    multiply into dP), 8 x pack to bf16 (attention.hip: s = exp2(s) * dp; ds = XOp(s))."""
    out = []
    for p in range(4):
        S, D = V["sacc"] + 16 * p, V["dpacc"] + 16 * p
        dsr = V["ds"] + 8 * p
        for k in range(8):
            a, b = 2 * k, 2 * k + 1
            out += [f"v_exp_f32 v{S + a}, v{S + a}", f"v_exp_f32 v{S + b}, v{S + b}",
                    f"v_mul_f32 v{D + a}, v{S + a}, v{D + a}",
                    f"v_mul_f32 v{D + b}, v{S + b}, v{D + b}",
                    f"v_cvt_pk_bf16_f32 v{dsr + k}, v{D + a}, v{D + b}"]
    return out


def tile_mfmas(V, A, stage):
    """48 MFMAs in program order, each (text, LDS read ids it consumes)."""
    out = []

    def g_block(kb):
        for i in range(2):
            for s2 in range(2):
                tr = A.r("trf", 16 * kb + 8 * i + 4 * s2, 4)
                for j in range(2):
                    p = 2 * kb + j
                    acc = A.r("acc", 16 * (2 * i + j), 16)
                    ds = V.r("ds", 8 * p + 4 * s2, 4)
                    out.append((f"{MFMA} {acc}, {tr}, {ds}, {acc}", ()))

    def pair(kb, j):
        p = 2 * kb + j
        for s in range(4):
            kf, vf = A.r("kf", 16 * kb + 4 * s, 4), A.r("vf", 16 * kb + 4 * s, 4)
            qf, of = A.r("qf", 16 * j + 4 * s, 4), A.r("of", 16 * j + 4 * s, 4)
            cs = V.r("il", 16 * j, 16) if s == 0 else sacc(V, p)
            cd = V.r("id", 16 * j, 16) if s == 0 else dpacc(V, p)
            out.append((f"{MFMA} {sacc(V, p)}, {kf}, {qf}, {cs}", (("K", kb, s),)))
            out.append((f"{MFMA} {dpacc(V, p)}, {vf}, {of}, {cd}", (("V", kb, s),)))

    g_block(0)
    pair(0, 0)
    pair(0, 1)
    g_block(1)
    pair(1, 0)
    pair(1, 1)
    return out


def tile_reads(V, A, stage):
    """slot -> [(ds_read text, id)]: slot g is issued before MFMA g."""
    prev = (stage + 3) % 4
    reads = {}

    def add(slot, text, rid):
        reads.setdefault(slot, []).append((text, rid))

    # score-block fragments of this tile: kb 0 at slots 0-3, kb 1 at slots 10-13 (at most 15
    # LDS reads in flight: lgkmcnt is 4 bits)
    for kb in range(2):
        k = 0
        for s in range(4):
            for x, name, off in (("K", "kf", 0), ("V", "vf", VOFF)):
                text = (f"ds_read_b128 {A.r(name, 16 * kb + 4 * s, 4)}, {V.r('rowoff', s)} "
                        f"offset:{stage * STAGE + off + kb * 4096}")
                add((0, 10)[kb] + k // 2, text, (x, kb, s))
                k += 1
    # K^T fragments of THIS tile for the next iteration's dQ products (kb 0 after MFMA 7
    # has read the previous ones, kb 1 after MFMA 31)
    for kb, slot0 in ((0, 16), (1, 36)):
        k = 0
        for i in range(2):
            for s2 in range(2):
                for hi in range(2):
                    text = (f"ds_read_b64_tr_b16 {A.r('trf', 16 * kb + 8 * i + 4 * s2 + 2 * hi, 2)}, "
                            f"{V.r('troff', 2 * i + hi)} offset:{stage * STAGE + kb * 4096 + s2 * 2048}")
                    add(slot0 + k // 2, text, ("T", kb, i, s2, hi))
                    k += 1
    del prev
    return reads


def emit_tile(st: Stream, V, A, stage, valu):
    """One tile of the unrolled loop (ring stage `stage`)."""
    st.comment(f"---- tile, ring stage {stage}")
    st.raw("s_waitcnt vmcnt(4) lgkmcnt(0)")
    st.raw("s_barrier")
    st.flush_lds()
    mf = tile_mfmas(V, A, stage)
    reads = tile_reads(V, A, stage)
    nm = len(mf)
    slots = {}
    for i, text in enumerate(valu):
        slots.setdefault((START + 1 + (i * nm) // len(valu)) % nm, []).append(text)
    dma_slots = {2: (0, 0), 5: (0, 1), 8: (1, 0), 11: (1, 1)}  # (tensor, piece)
    nxt = (stage + 2) % 4
    d0 = V["dma"]
    for g in range(nm):
        if g in dma_slots:
            x, i = dma_slots[g]
            st.raw(f"s_add_u32 m0, {S_M0}, {nxt * STAGE + x * VOFF + i * 1024}")
            st.raw("s_nop 0")
            st.emit(f"buffer_load_dwordx4 v{d0 + i}, {RK if x == 0 else RV}, 0 offen lds")
            if (x, i) == (1, 1):
                for k in range(2):
                    st.emit(f"v_add_u32 v{d0 + k}, s46, v{d0 + k}")
        for text, rid in reads.get(g, []):
            st.emit(text, lds_id=rid)
        for text in slots.get(g, []):
            st.emit(text)
        text, deps = mf[g]
        st.emit(text, wait_lds=deps)


def emit_tail(st: Stream, V, A, valu):
    """After the last tile: the rest of its VALU stream and its dQ products."""
    nm = 48
    st.comment("---- tail: last tile's dQ products")
    st.raw("s_waitcnt lgkmcnt(0)")
    st.flush_lds()
    rest = [t for i, t in enumerate(valu) if (START + 1 + (i * nm) // len(valu)) >= nm]
    mf = tile_mfmas(V, A, 0)
    g0 = mf[0:8]
    g1 = mf[24:32]
    per = -(-len(rest) // 8)
    for k, (text, _) in enumerate(g0):
        for t in rest[k * per:(k + 1) * per]:
            st.emit(t)
        st.emit(text)
    for text, _ in g1:
        st.emit(text)


def epilogue_dq(st: Stream, V, A):
    st.raw("s_waitcnt vmcnt(0)")
    t = [V["sacc"] + k for k in range(8)]
    for j in range(2):
        for i in range(2):
            for g in range(4):
                base = 16 * (2 * i + j) + 4 * g
                for k in range(4):
                    st.emit(f"v_accvgpr_read_b32 v{t[k]}, {A.r('acc', base + k)}")
                for k in range(4):
                    st.emit(f"v_mul_f32 v{t[k]}, s42, v{t[k]}")
                st.emit(f"v_cvt_pk_bf16_f32 v{t[4]}, v{t[0]}, v{t[1]}")
                st.emit(f"v_cvt_pk_bf16_f32 v{t[5]}, v{t[2]}, v{t[3]}")
                st.emit(f"buffer_store_dwordx2 v[{t[4]}:{t[5]}], {V.r('stq', j)}, {RDQ}, 0 offen "
                        f"offset:{64 * i + 16 * g}")


def emit_probe(st: Stream, regs, karg_off, tmp=("v14", "v15")):
    """Diagnostic builds only (tools/asm_probe.py): store `regs` of every lane of workgroup 0
    to the debug buffer whose address follows the kernel's arguments, then end the wave."""
    t0, t1 = tmp
    st.raw(f"s_load_dwordx2 s[90:91], {S_KARG}, {karg_off}")
    st.raw("s_waitcnt vmcnt(0) lgkmcnt(0)")
    st.raw("s_nop 15")
    st.raw(f"v_mul_u32_u24 {t1}, {4 * len(regs)}, v0")
    for k, r in enumerate(regs):
        src = r
        if r.startswith("a"):
            st.raw(f"v_accvgpr_read_b32 {t0}, {r}")
            st.raw("s_nop 1")
            src = t0
        elif r.startswith("s"):
            st.raw(f"v_mov_b32 {t0}, {r}")
            src = t0
        st.raw(f"global_store_dword {t1}, {src}, s[90:91] offset:{4 * k}")
        st.raw("s_waitcnt vmcnt(0)")
    st.raw("s_endpgm")


def gen_dq(probe=None):
    """probe: (point, [registers]) -- a diagnostic build that dumps the registers at point
    'prologue', 'tile0' (after the first tile) or 'loop' (after the loop)."""
    V, A = regs_dq()
    st = Stream()
    prologue_dq(st, V, A)
    if probe and probe[0] == "prologue":
        emit_probe(st, probe[1], KARG_BYTES)
    valu = valu_stream(V)
    st.label(".Ldq_loop")
    for stage in range(4):
        emit_tile(st, V, A, stage, valu)
        if probe and probe[0] == "tile0" and stage == 0:
            emit_probe(st, probe[1], KARG_BYTES)
    st.raw(f"s_sub_u32 {S_ITER}, {S_ITER}, 1")
    st.raw(f"s_cmp_lg_u32 {S_ITER}, 0")
    st.raw("s_cbranch_scc1 .Ldq_loop")
    emit_tail(st, V, A, valu)
    if probe and probe[0] == "loop":
        emit_probe(st, probe[1], KARG_BYTES)
    epilogue_dq(st, V, A)
    k = kernel_text("vd_attn_bwd_dq_d64", st.text(), vgprs=V.next, agprs=A.next, sgprs=96,
                    lds_bytes=4 * STAGE, kernarg_bytes=KARG_BYTES + (8 if probe else 0),
                    wg_size=64 * NW)
    data = "\n.rodata\n.p2align 8\nvd_attn_dq_lanes:\n"
    for row in lane_table():
        data += "\t.long " + ", ".join(str(x) for x in row) + "\n"
    return k, data, st


def main():
    out = sys.argv[1]
    for arg in sys.argv[2:]:  # A/B builds only (tools/build_asm_phase.sh, build_asm_knobs.sh)
        if arg.startswith("--phase="):
            import asmgen
            asmgen.PHASE_FLIP = arg[len("--phase="):]
        elif arg.startswith("--knob="):  # --knob=module.NAME=int, e.g. gen_fwd.CHAINS=4
            import importlib
            target, val = arg[len("--knob="):].split("=")
            mod, name = target.split(".")
            m = sys.modules[__name__] if mod == "gen_attn_asm" else importlib.import_module(mod)
            assert hasattr(m, name), target
            setattr(m, name, int(val))
    from gen_d128 import gen_dkdv128, gen_dq128
    from gen_fwd128 import gen_fwd128
    from gen_fwd import gen_fwd
    from gen_d256 import gen_dq256
    from gen_d256dk import gen_dkdv256
    from gen_fwd256 import gen_fwd256
    kdq, ddq, sdq = gen_dq()
    kdk, ddk, sdk = gen_dkdv()
    kfw, sfw = gen_fwd()
    kdk2, ddk2, sdk2 = gen_dkdv128()
    kdq2, sdq2 = gen_dq128()
    kfw2, dfw2, sfw2 = gen_fwd128()
    kdq4, ddq4, sdq4 = gen_dq256()
    kdk4, ddk4, sdk4 = gen_dkdv256()
    kfw4, sfw4 = gen_fwd256()
    with open(out, "w") as f:
        f.write("// generated by gen_attn_asm.py -- do not edit\n")
        f.write(code_object_text([kdq, kdk, kfw, kdk2, kdq2, kfw2, kdq4, kdk4, kfw4],
                                 ddq + ddk + ddk2 + dfw2 + ddq4 + ddk4))
    if "--report" in sys.argv:
        for name, st in (("dq", sdq), ("dkdv", sdk), ("fwd", sfw), ("dkdv128", sdk2),
                         ("dq128", sdq2), ("fwd128", sfw2), ("dq256", sdq4),
                         ("dkdv256", sdk4), ("fwd256", sfw4)):
            print(f"{name}: {len(st.lines)} lines, {st.nops} nop wait states, {st.waits} lgkm "
                  f"waits, {st.forced} forced by the 15-read limit ({st.young} on young reads)")




# ================================================================== dK / dV
# vd_attn_bwd_dkdv_d64: the arithmetic of attn_bwd_dkdv_pipe_kernel<bf16, 64> (S' = Q K'^T -
# lse', dP = dO V^T - delta with the query on the accumulator rows and the key on the lane,
# dV^T += dO^T P, dK^T += Q^T dS, K' = K * scale * log2 e) at one wave per SIMD: 4 waves x
# 64 keys (2 key blocks kj) per workgroup.  Per 64-query tile (2 query blocks qb) a wave runs
# 64 MFMAs and 192 VALU instructions.  MFMA order of iteration t:
#   S/dP(t, qb0) [16] | dQ-less G(t-1, qb1) [16] | S/dP(t, qb1) [16] | barrier | G(t, qb0) [16]
# The barrier that publishes tile t+1 sits before the last group, so the fragment reads of
# (t+1, qb0) -- rows of Q and dO, the row constants -- are issued under G(t, qb0).  The VALU
# stream runs at 3 instructions per gap: the softmax of (t, qb0) in gaps 17..48, of (t, qb1)
# in gaps 49..16 of the next iteration, each finishing just before its G group.
DK_STAGE = 16384          # Q tile | dO tile
DK_RC = 768               # per stage: lse' (256 B) | delta (256 B) | junk (256 B)
DK_RC_BYTES = 4 * DK_RC   # the row-constant region at LDS offset 0
DK_KARG = 144
DK_START = 17
RQ2, RK2, RV2, RO2, RL2, RD2, RDK2, RDV2 = ("s[60:63]", "s[64:67]", "s[68:71]", "s[72:75]",
                                            "s[76:79]", "s[80:83]", "s[84:87]", "s[88:91]")
S2_WAVE, S2_K0, S2_M0, S2_ITER, S2_RCM0 = "s92", "s93", "s94", "s95", "s98"
RRC2 = "s[56:59]"  # this wave's row-constant DMA source (lse', delta, or lse' into junk)


def regs_dkdv():
    V, A = Regs("v"), Regs("a")
    for name, n in (("tid", 1), ("lane", 1), ("rowoff", 4), ("troff", 4), ("dmaq", 2),
                    ("dmao", 2), ("dmac", 2), ("rcv", 1), ("rcoff", 1), ("tmp", 4),
                    ("stk", 2), ("tmp2", 2)):
        V.alloc(name, n)
    V.alloc("s", 64, 16)     # S' blocks [qb][kj]
    V.alloc("dp", 64)        # dP blocks [qb][kj]
    V.alloc("pp", 32)        # P as bf16 B operands [qb][kj] x 8
    V.alloc("ds", 32)        # dS as bf16 B operands
    V.alloc("il", 16)        # -lse' of the current query block's rows (srcC of S)
    V.alloc("id", 16)        # -delta of those rows (srcC of dP)
    A.alloc("kf", 32)        # K' fragments [kj][s]
    A.alloc("vf", 32)        # V fragments [kj][s]
    A.alloc("adk", 64)       # dK^T accumulators [i][kj]
    A.alloc("adv", 64)       # dV^T accumulators [i][kj]
    A.alloc("qrow", 16)      # Q row fragments of the current query block [s]
    A.alloc("orow", 16)      # dO row fragments [s]
    A.alloc("otr", 16)       # dO^T fragments of the G block [i][s2]
    A.alloc("qtr", 16)       # Q^T fragments [i][s2]
    return V, A


def dk_lane_table():
    base = lane_table()
    for w in range(NW):
        for lane in range(64):
            base[w * 64 + lane][12] = 16 * (lane >> 5)  # row-constant read base (16 hh)
    return base


def blk(qb, kj):
    return 2 * qb + kj


def prologue_dkdv(st: Stream, V, A):
    e, r = st.emit, st.raw
    r(f"s_load_dwordx16 s[16:31], {S_KARG}, 0x0")
    r(f"s_load_dwordx16 s[32:47], {S_KARG}, 0x40")
    r(f"s_load_dwordx4 s[48:51], {S_KARG}, 0x80")
    e(f"v_and_b32 {V.r('lane')}, 63, {V.r('tid')}")
    r(f"v_readfirstlane_b32 {S2_WAVE}, {V.r('tid')}")  # first lane's id = 64 * wave
    r("s_nop 1")
    r(f"s_lshr_b32 {S2_WAVE}, {S2_WAVE}, 6")
    r("s_getpc_b64 s[96:97]")
    r("s_add_u32 s96, s96, vd_attn_dkdv_lanes@rel32@lo+4")
    r("s_addc_u32 s97, s97, vd_attn_dkdv_lanes@rel32@hi+12")
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

    rsrc(RQ2, "s16", "s17", "s54", "s55", "s46")
    rsrc(RK2, "s18", "s19", "s54", "s55", "s46")
    rsrc(RV2, "s20", "s21", "s54", "s55", "s46")
    rsrc(RO2, "s22", "s23", "s56", "s57", "s47")
    rsrc(RDK2, "s28", "s29", "s54", "s55", "s46")
    rsrc(RDV2, "s30", "s31", "s54", "s55", "s46")
    r("s_mul_i32 s58, s52, s32")
    r("s_mul_hi_u32 s59, s52, s32")
    r("s_lshl_b64 s[58:59], s[58:59], 2")
    r("s_lshl_b32 s99, s32, 2")
    rsrc(RL2, "s24", "s25", "s58", "s59", "s99")
    rsrc(RD2, "s26", "s27", "s58", "s59", "s99")
    # wave 1 stages delta, the others lse' (waves 2, 3 into the junk slot)
    r(f"s_cmp_eq_u32 {S2_WAVE}, 1")
    r("s_cselect_b64 s[56:57], s[80:81], s[76:77]")
    r("s_cselect_b64 s[58:59], s[82:83], s[78:79]")
    r(f"s_min_u32 s99, {S2_WAVE}, 2")
    r(f"s_lshl_b32 {S2_RCM0}, s99, 8")
    # k0 = wgx * 256 + wave * 64 ; DMA M0 base = wave * 2048 (+ the tile region)
    r(f"s_lshl_b32 {S2_K0}, {S_WGX}, 8")
    r(f"s_lshl_b32 s99, {S2_WAVE}, 6")
    r(f"s_add_u32 {S2_K0}, {S2_K0}, s99")
    r(f"s_lshl_b32 {S2_M0}, {S2_WAVE}, 11")
    r(f"s_add_u32 {S2_M0}, {S2_M0}, {DK_RC_BYTES}")
    r(f"s_mov_b32 {S2_ITER}, s50")
    t0, t1 = V.r("tmp", 0), V.r("tmp", 1)
    e(f"v_lshlrev_b32 {t0}, 6, {V.r('tid')}")
    r(f"global_load_dwordx4 {V.r('rowoff', 0, 4)}, {t0}, s[96:97]")
    r(f"global_load_dwordx4 {V.r('troff', 0, 4)}, {t0}, s[96:97] offset:16")
    r(f"global_load_dwordx2 {V.r('dmaq', 0, 2)}, {t0}, s[96:97] offset:32")
    r(f"global_load_dwordx2 {V.r('dmac', 0, 2)}, {t0}, s[96:97] offset:40")
    r(f"global_load_dword {V.r('rcoff')}, {t0}, s[96:97] offset:48")
    # key rows of the wave: krow_kj = k0 + 32 kj + (lane & 31)
    krow = [V.r("s", 60), V.r("s", 61)]
    hh16 = V.r("s", 62)
    e(f"v_and_b32 {krow[0]}, 31, {V.r('lane')}")
    e(f"v_add_u32 {krow[0]}, {S2_K0}, {krow[0]}")
    e(f"v_add_u32 {krow[1]}, 32, {krow[0]}")
    e(f"v_lshrrev_b32 {hh16}, 5, {V.r('lane')}")
    e(f"v_lshlrev_b32 {hh16}, 4, {hh16}")
    kv = V["s"]  # K fragments staged in v[s .. s+31] for scaling
    for kj in range(2):
        vk = V.r("dp", 60 + kj)
        e(f"v_mul_lo_u32 {vk}, {krow[kj]}, s33")
        e(f"v_add_u32 {vk}, {vk}, {hh16}")
        for s in range(4):
            r(f"buffer_load_dwordx4 v[{kv + 16 * kj + 4 * s}:{kv + 16 * kj + 4 * s + 3}], {vk}, "
              f"{RK2}, 0 offen offset:{32 * s}")
            r(f"buffer_load_dwordx4 {A.r('vf', 16 * kj + 4 * s, 4)}, {vk}, {RV2}, 0 offen "
              f"offset:{32 * s}")
        e(f"v_lshrrev_b32 {V.r('dp', 54)}, 1, {hh16}")
        e(f"v_mul_lo_u32 {V.r('stk', kj)}, {krow[kj]}, s33")
        e(f"v_add_u32 {V.r('stk', kj)}, {V.r('stk', kj)}, {V.r('dp', 54)}")
    r("s_waitcnt vmcnt(0)")
    for w in range(32):
        x = f"v{kv + w}"
        e(f"v_lshlrev_b32 {t0}, 16, {x}")
        e(f"v_and_b32 {t1}, 0xffff0000, {x}")
        e(f"v_mul_f32 {t0}, s45, {t0}")
        e(f"v_mul_f32 {t1}, s45, {t1}")
        e(f"v_cvt_pk_bf16_f32 {x}, {t0}, {t1}")
        e(f"v_accvgpr_write_b32 {A.r('kf', w)}, {x}")
    # DMA source offsets: Q / dO pieces row * stride + chunk * 16 ; row constants 4 lane
    for i in range(2):
        e(f"v_mul_lo_u32 {V.r('dmao', i)}, {V.r('dmaq', i)}, s34")
        e(f"v_add_u32 {V.r('dmao', i)}, {V.r('dmao', i)}, {V.r('dmac', i)}")
        e(f"v_mul_lo_u32 {V.r('dmaq', i)}, {V.r('dmaq', i)}, s33")
        e(f"v_add_u32 {V.r('dmaq', i)}, {V.r('dmaq', i)}, {V.r('dmac', i)}")
    e(f"v_lshlrev_b32 {V.r('rcv')}, 2, {V.r('lane')}")
    for k in range(128):
        e(f"v_accvgpr_write_b32 a{A['adk'] + k}, 0")
    for name in ("pp", "ds"):
        for k in range(32):
            e(f"v_mov_b32 {V.r(name, k)}, 0")
    for k in range(64):
        e(f"v_mov_b32 {V.r('s', k)}, 0")
        e(f"v_mov_b32 {V.r('dp', k)}, 0")
    for k in range(4):
        e(f"v_mov_b32 {V.r('tmp', k)}, 0")
    # zero ring stage 3 (tile -1: the A operands of the first G group) and its constants
    e(f"v_lshlrev_b32 {V.r('tmp2', 0)}, 6, {V.r('tid')}")
    for k in range(4):
        e(f"ds_write_b128 {V.r('tmp2', 0)}, {V.r('tmp', 0, 4)} "
          f"offset:{DK_RC_BYTES + 3 * DK_STAGE + 16 * k}")
    e(f"v_lshlrev_b32 {V.r('tmp2', 1)}, 2, {V.r('tid')}")
    r(f"s_cmp_lt_u32 {S2_WAVE}, 3")
    r("s_cbranch_scc0 .Ldk_nozero")
    e(f"ds_write_b32 {V.r('tmp2', 1)}, {V.r('tmp', 0)} offset:{3 * DK_RC}")
    st.label(".Ldk_nozero")
    r("s_waitcnt lgkmcnt(0)")
    for k in range(4):  # the loop's +32 KiB copies of the K^T / Q^T fragment offsets
        e(f"v_add_u32 {V.r('tmp', k)}, 0x8000, {V.r('troff', k)}")
    for t in range(3):
        dk_dma(st, V, t, slots=None)
    r("s_waitcnt vmcnt(10)")
    r("s_barrier")
    st.flush_lds()
    for text, rid in dk_row_reads(V, A, 0, 0):
        st.emit(text, lds_id=rid)


def dk_dma(st: Stream, V, stage, slots):
    """The wave's 5 DMA ops of one tile into `stage` (Q pieces, dO pieces, its row-constant
    piece), then advance the source offsets.  slots=None: emit now."""
    ops = []
    for x, (rs, nm) in enumerate(((RQ2, "dmaq"), (RO2, "dmao"))):
        for i in range(2):
            ops.append((f"s_add_u32 m0, {S2_M0}, {stage * DK_STAGE + x * 8192 + i * 1024}",
                        f"buffer_load_dwordx4 {V.r(nm, i)}, {rs}, 0 offen lds"))
    ops.append((f"s_add_u32 m0, {S2_RCM0}, {stage * DK_RC}",
                f"buffer_load_dword {V.r('rcv')}, {RRC2}, 0 offen lds"))
    adv = [f"v_add_u32 {V.r('dmaq', 0)}, s48, {V.r('dmaq', 0)}",
           f"v_add_u32 {V.r('dmaq', 1)}, s48, {V.r('dmaq', 1)}",
           f"v_add_u32 {V.r('dmao', 0)}, s49, {V.r('dmao', 0)}",
           f"v_add_u32 {V.r('dmao', 1)}, s49, {V.r('dmao', 1)}",
           f"v_add_u32 {V.r('rcv')}, 0x100, {V.r('rcv')}"]
    if slots is None:
        for m0, ld in ops:
            st.raw(m0)
            st.raw("s_nop 0")
            st.emit(ld)
        for a in adv:
            st.emit(a)
        return None
    return ops, adv


def dk_row_reads(V, A, stage, qb):
    """Fragment reads of query block qb of the tile in `stage`: Q rows, dO rows, -lse' and
    -delta of the block's rows (register 4g + e = row 8 g + 4 hh + e)."""
    out = []
    tq = DK_RC_BYTES + stage * DK_STAGE + qb * 4096
    for s in range(4):
        out.append((f"ds_read_b128 {A.r('qrow', 4 * s, 4)}, {V.r('rowoff', s)} offset:{tq}",
                    ("Q", s)))
        out.append((f"ds_read_b128 {A.r('orow', 4 * s, 4)}, {V.r('rowoff', s)} "
                    f"offset:{tq + 8192}", ("O", s)))
    for g in range(4):
        rc = stage * DK_RC + qb * 128 + 32 * g
        out.append((f"ds_read_b128 {V.r('il', 4 * g, 4)}, {V.r('rcoff')} offset:{rc}", ("L", g)))
        out.append((f"ds_read_b128 {V.r('id', 4 * g, 4)}, {V.r('rcoff')} offset:{rc + 256}",
                    ("D", g)))
    return out


def dk_tr_reads(V, A, stage, qb):
    out = []
    tq = DK_RC_BYTES + stage * DK_STAGE + qb * 4096
    for i in range(2):
        for s2 in range(2):
            for hi in range(2):
                for x, name in ((8192, "otr"), (0, "qtr")):
                    off, base = tq + x + s2 * 2048, V.r("troff", 2 * i + hi)
                    if off > 65535:  # past the 16-bit immediate: the +32 KiB base copy
                        off, base = off - 32768, V.r("tmp", 2 * i + hi)
                    out.append((f"ds_read_b64_tr_b16 {A.r(name, 8 * i + 4 * s2 + 2 * hi, 2)}, "
                                f"{base} offset:{off}", (name, i, s2, hi)))
    return out


def dk_valu(V):
    out = []
    for qb in range(2):
        for kj in range(2):
            b = blk(qb, kj)
            S, D = V["s"] + 16 * b, V["dp"] + 16 * b
            P, G = V["pp"] + 8 * b, V["ds"] + 8 * b
            for k in range(8):
                a, c = 2 * k, 2 * k + 1
                out += [f"v_exp_f32 v{S + a}, v{S + a}", f"v_exp_f32 v{S + c}, v{S + c}",
                        f"v_mul_f32 v{D + a}, v{D + a}, v{S + a}",
                        f"v_mul_f32 v{D + c}, v{D + c}, v{S + c}",
                        f"v_cvt_pk_bf16_f32 v{P + k}, v{S + a}, v{S + c}",
                        f"v_cvt_pk_bf16_f32 v{G + k}, v{D + a}, v{D + c}"]
    return out


def dk_sdp(V, A, qb):
    out = []
    for s in range(4):
        for kj in range(2):
            b = blk(qb, kj)
            sv, dv = V.r("s", 16 * b, 16), V.r("dp", 16 * b, 16)
            cs = V.r("il", 0, 16) if s == 0 else sv
            cd = V.r("id", 0, 16) if s == 0 else dv
            out.append((f"{MFMA} {sv}, {A.r('qrow', 4 * s, 4)}, {A.r('kf', 16 * kj + 4 * s, 4)}, "
                        f"{cs}", (("Q", s),) + ((("L", 0), ("L", 1), ("L", 2), ("L", 3))
                                                  if s == 0 else ())))
            out.append((f"{MFMA} {dv}, {A.r('orow', 4 * s, 4)}, {A.r('vf', 16 * kj + 4 * s, 4)}, "
                        f"{cd}", (("O", s),) + ((("D", 0), ("D", 1), ("D", 2), ("D", 3))
                                                  if s == 0 else ())))
    return out


def dk_g(V, A, qb):
    out = []
    for i in range(2):
        for s2 in range(2):
            for kj in range(2):
                b = blk(qb, kj)
                acc = A.r("adv", 16 * (2 * i + kj), 16)
                out.append((f"{MFMA} {acc}, {A.r('otr', 8 * i + 4 * s2, 4)}, "
                            f"{V.r('pp', 8 * b + 4 * s2, 4)}, {acc}",
                            tuple(("otr", i, s2, h) for h in range(2))))
        for s2 in range(2):
            for kj in range(2):
                b = blk(qb, kj)
                acc = A.r("adk", 16 * (2 * i + kj), 16)
                out.append((f"{MFMA} {acc}, {A.r('qtr', 8 * i + 4 * s2, 4)}, "
                            f"{V.r('ds', 8 * b + 4 * s2, 4)}, {acc}",
                            tuple(("qtr", i, s2, h) for h in range(2))))
    return out


def emit_dk_iter(st: Stream, V, A, stage, valu):
    """Iteration t (tile t in `stage`): S/dP(t, qb0), G(t-1, qb1), S/dP(t, qb1), barrier for
    tile t+1, G(t, qb0); reads for (t+1, qb0) after the barrier."""
    prev, nxt = (stage + 3) % 4, (stage + 1) % 4
    st.comment(f"---- query tile, ring stage {stage}")
    mf = dk_sdp(V, A, 0) + dk_g(V, A, 1) + dk_sdp(V, A, 1) + dk_g(V, A, 0)
    nm = len(mf)
    slots = {}
    for i, text in enumerate(valu):
        slots.setdefault((DK_START + (i * nm) // len(valu)) % nm, []).append((text, None))

    def put(slot0, lst, per=2):
        for k, (text, rid) in enumerate(lst):
            slots.setdefault(slot0 + k // per, []).insert(0, (text, rid))

    put(2, dk_tr_reads(V, A, prev, 1))          # G(t-1, qb1) operands, tile t-1
    put(18, dk_row_reads(V, A, stage, 1))       # (t, qb1) fragments
    put(34, dk_tr_reads(V, A, stage, 0))        # G(t, qb0) operands
    ops, adv = dk_dma(st, V, (stage + 3) % 4, slots=True)
    dma_at = [49, 51, 53, 55, 57]
    for g in range(nm):
        if g == 48:
            st.raw("s_waitcnt vmcnt(5) lgkmcnt(0)")
            st.raw("s_barrier")
            st.flush_lds()
            for text, rid in dk_row_reads(V, A, nxt, 0):
                slots.setdefault(49 + 0, [])
            for k, (text, rid) in enumerate(dk_row_reads(V, A, nxt, 0)):
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
    del prev


def emit_dk_tail(st: Stream, V, A, valu):
    nm = 64
    st.comment("---- tail: the last tile's second G group")
    st.raw("s_waitcnt lgkmcnt(0)")
    st.flush_lds()
    # the last tile's trailing softmax: the VALU of slots 0..DK_START-1 (they wrapped)
    rest = [t for i, t in enumerate(valu) if DK_START + (i * nm) // len(valu) >= nm]
    stage = 3
    for text, rid in dk_tr_reads(V, A, stage, 1):
        st.emit(text, lds_id=rid)
    for t in rest:
        st.emit(t)
    for text, deps in dk_g(V, A, 1):
        st.emit(text, wait_lds=deps)


def epilogue_dkdv(st: Stream, V, A):
    st.raw("s_waitcnt vmcnt(0)")
    t = [V["s"] + k for k in range(8)]
    for name, rs, scale in (("adk", RDK2, "s44"), ("adv", RDV2, None)):
        for kj in range(2):
            for i in range(2):
                for g in range(4):
                    base = 16 * (2 * i + kj) + 4 * g
                    for k in range(4):
                        st.emit(f"v_accvgpr_read_b32 v{t[k]}, {A.r(name, base + k)}")
                    if scale:
                        for k in range(4):
                            st.emit(f"v_mul_f32 v{t[k]}, {scale}, v{t[k]}")
                    st.emit(f"v_cvt_pk_bf16_f32 v{t[4]}, v{t[0]}, v{t[1]}")
                    st.emit(f"v_cvt_pk_bf16_f32 v{t[5]}, v{t[2]}, v{t[3]}")
                    st.emit(f"buffer_store_dwordx2 v[{t[4]}:{t[5]}], {V.r('stk', kj)}, {rs}, 0 "
                            f"offen offset:{64 * i + 16 * g}")


def gen_dkdv():
    V, A = regs_dkdv()
    st = Stream()
    prologue_dkdv(st, V, A)
    valu = dk_valu(V)
    st.label(".Ldk_loop")
    for stage in range(4):
        emit_dk_iter(st, V, A, stage, valu)
    st.raw(f"s_sub_u32 {S2_ITER}, {S2_ITER}, 1")
    st.raw(f"s_cmp_lg_u32 {S2_ITER}, 0")
    st.raw("s_cbranch_scc1 .Ldk_loop")
    emit_dk_tail(st, V, A, valu)
    epilogue_dkdv(st, V, A)
    k = kernel_text("vd_attn_bwd_dkdv_d64", st.text(), vgprs=V.next, agprs=A.next, sgprs=100,
                    lds_bytes=DK_RC_BYTES + 4 * DK_STAGE, kernarg_bytes=DK_KARG,
                    wg_size=64 * NW)
    data = "\n.rodata\n.p2align 8\nvd_attn_dkdv_lanes:\n"
    for row in dk_lane_table():
        data += "\t.long " + ", ".join(str(x) for x in row) + "\n"
    return k, data, st


if __name__ == "__main__":
    main()
