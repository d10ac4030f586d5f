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

from asmgen import Regs, Stream, kernel_text

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
    e(f"v_lshrrev_b32 {V.r('tmp')}, 6, {V.r('tid')}")
    r(f"v_readfirstlane_b32 {S_WAVE}, {V.r('tmp')}")
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

    # score-block fragments of this tile: kb 0 at slots 0-3, kb 1 at slots 4-7
    for kb in range(2):
        k = 0
        for s in range(4):
            for x, name, off in (("K", "kf", 0), ("V", "vf", VOFF)):
                text = (f"ds_read_b128 {A.r(name, 16 * kb + 4 * s, 4)}, {V.r('rowoff', s)} "
                        f"offset:{stage * STAGE + off + kb * 4096}")
                add(4 * kb + k // 2, text, (x, kb, s))
                k += 1
    # K^T fragments of THIS tile for the next iteration's dQ products (kb 0 after MFMA 7
    # has read the previous ones, kb 1 after MFMA 31)
    for kb, slot0 in ((0, 12), (1, 36)):
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


def gen_dq():
    V, A = regs_dq()
    st = Stream()
    prologue_dq(st, V, A)
    valu = valu_stream(V)
    st.label(".Ldq_loop")
    for stage in range(4):
        emit_tile(st, V, A, stage, valu)
    st.raw(f"s_sub_u32 {S_ITER}, {S_ITER}, 1")
    st.raw(f"s_cmp_lg_u32 {S_ITER}, 0")
    st.raw("s_cbranch_scc1 .Ldq_loop")
    emit_tail(st, V, A, valu)
    epilogue_dq(st, V, A)
    name = "vd_attn_bwd_dq_d64"
    text = kernel_text(name, st.text(), vgprs=V.next, agprs=A.next, sgprs=96,
                       lds_bytes=4 * STAGE, kernarg_bytes=KARG_BYTES, wg_size=64 * NW)
    tab = lane_table()
    text += "\n.rodata\n.p2align 8\nvd_attn_dq_lanes:\n"
    for row in tab:
        text += "\t.long " + ", ".join(str(x) for x in row) + "\n"
    return text, st


def main():
    out = sys.argv[1]
    text, st = gen_dq()
    with open(out, "w") as f:
        f.write("// generated by gen_attn_asm.py -- do not edit\n" + text)
    if "--report" in sys.argv:
        print(f"dq: {len(st.lines)} lines, {st.nops} nop wait states, {st.waits} lgkm waits")


if __name__ == "__main__":
    main()
