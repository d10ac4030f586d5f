"""vd_attn_fwd_d64: hand-scheduled gfx950 forward of the head_dim-64 joint attention
(reference QKVAttentionLegacy.forward, unet.py:349-366: softmax(Q K^T / sqrt(D)) V), the
arithmetic of attn_fwd_defer_kernel<bf16, 64> in attention.hip laid out for ONE wave per
SIMD: 4 waves x 64 queries (2 query blocks j) per workgroup, 256 queries per workgroup.

Per 64-key tile t a wave runs 32 v_mfma_f32_32x32x16_bf16 in body t:
    G(t-1, kb0) [8] | S(t+1, kb0) [8] | G(t-1, kb1) [8] | S(t+1, kb1) [8]
with S^T = K Q'^T - m (the key on the accumulator rows, the query on the lane; srcC = the
-m splat), G: O^T += V^T P^T (P^T as the B operand straight from the accumulators, the key
permutation absorbed into the V^T transposed-read offsets as in the dQ kernel), and the
softmax of tile t (64 v_exp_f32, 62 row-sum adds, 32 v_cvt_pk_bf16_f32) spread over the 32
gaps of the same body by cost (exp 8 cycles, add 4, cvt 4.5).  S is computed one tile
ahead into a second accumulator set, so the softmax stream never waits for its MFMAs.

Lagged max (attention.hip kLagSum): p = exp2(S' - m) with the stale m; after the softmax of
tile t the wave checks that every lane's tile sum is < 2^16 (false for inf / NaN too) and
otherwise calls the rare path (a subroutine, s_swappc): recompute S(t) from the resident K
tile, take the true row max over the tile (both lane halves), rescale O and l by
exp2(m - m_new), redo tile t's softmax, and recompute S(t+1), whose MFMAs ran against the
old m.  m starts at -inf (the -m splat at +inf), so the first tile always takes it.

Ring: 8 stages x (K tile 8 KiB | V tile 8 KiB) = 128 KiB of LDS by LDS-DMA, tile t+4 issued
in body t (4 pieces per wave spread over the body), one barrier per body behind
s_waitcnt vmcnt(8).  The loop is unrolled by the 8 stages; keys past the end of the
sequence (zero-filled by the buffer range check) are masked to -inf only in the last
iteration, which is its own copy of the 8 bodies.
"""
from __future__ import annotations

from asmgen import Regs, Stream, kernel_text

MFMA = "v_mfma_f32_32x32x16_bf16"
NW = 4
NST = 8                # ring stages
PD = 4                 # prefetch distance (tiles)
STAGE = 16384          # K tile | V tile
VOFF = 8192
KARG = 112
HI = 65536             # ds_read immediates are 16 bits: stages >= 4 use the +64 KiB bases
NINF, PINF = "0xff800000", "0x7f800000"
BAR2 = False           # A/B (tools/asm_ab.py): one barrier per two bodies
CHECK_NOP = 3          # wait states between the check's v_cmp and its branch
DROP = 0               # timing experiments only (wrong results): 1 exp, 2 add, 4 cvt, 8 reads,
                       # 16 the loop's LDS-DMA pieces
CHAINS = 1             # row-sum accumulators per query block (1: one dependent add chain;
                       # 14.24 vs 14.42 ms for 4, profiles/r03_ab_fwd_knobs.txt)
NORARE = 0             # timing experiment only: never take the rare path (wrong results)
STAMP = 0              # diagnostic: store loop cycles / realtime per workgroup (karg 112)
GSGS = 0               # MFMA order of a body: 0 G(kb0) G(kb1) S(kb0) S(kb1); 1 G S G S
LAG1 = 0               # CHAINS = 1 through the lagged list (adds 4 scores behind their exps)
DMAS = 0               # LDS-DMA slots of a body: 0 {4,12,20,28} 1 {1,9,17,25} 2 {6,14,22,30}
                       # 3 {0,8,16,24}
MSUM = 0               # row sums on the matrix pipe: 8 MFMAs (ones x P^T) per body replace the
                       # 64 v_add_f32; the tile's lagged-max check moves to the next body's top.
                       # 1: 32x32x16 (ones x P^T); 2: 16x16x32 with a lane-group selector as
                       # the A operand (half the matrix-pipe time, both lane halves summed)

# kernel arguments (AsmFwdArgs in vd_asm.h), loaded into s[16:43]:
#  0 q  8 k  16 v  24 o  32 lse                            (u64)   s16..s25
#  40 n  44 ts_bytes  48 ots_bytes  52 groups              (u32)   s26..s29
#  56 bs_bytes  64 gs_bytes  72 obs_bytes  80 ogs_bytes    (u64)   s30..s37
#  88 qscale (f32)  92 kv_bytes  96 o_bytes  100 tile_bytes         s38..s41
#  104 niter (512-key iterations, the last one masked)  108 klim0 (keys in it)  s42, s43
S_KARG = "s[0:1]"
S_WGX, S_WGY, S_WGZ = "s2", "s3", "s4"
RQ, RK, RV, RO, RL = "s[44:47]", "s[48:51]", "s[52:55]", "s[56:59]", "s[60:63]"
S_WAVE, S_Q0, S_M0, S_ITER, S_TAB = "s64", "s65", "s66", "s67", "s[68:69]"
S_ST, S_ST1, S_KB, S_RET, S_TGT = "s76", "s77", "s78", "s[80:81]", 82


def regs():
    V, A = Regs("v"), Regs("a")
    for name, n in (("tid", 1), ("lane", 1), ("rowoff", 4), ("troff", 4), ("rowhi", 4),
                    ("trhi", 4), ("dma", 2), ("dmac", 2), ("tmp", 4), ("sto", 2), ("klim", 1),
                    ("ps", 2), ("l", 2), ("m", 2), ("ninf", 1), ("tc", 2), ("c", 8)):
        V.alloc(name, n)
    V.alloc("s0", 64, 16)    # S' of the even tiles, 4 slots p = 2 kb + j
    V.alloc("s1", 64, 16)    # ... of the odd tiles
    V.alloc("p", 32)         # P^T as bf16 B operands, 8 per slot
    V.alloc("negm", 32)      # -m splats per query block (srcC of the first S MFMA)
    A.alloc("qf", 32)        # Q' fragments [j][s]
    A.alloc("acc", 64)       # O^T accumulators [i][j]
    A.alloc("kf", 32)        # K row fragments [kb][s]
    A.alloc("trf", 32)       # V^T fragments [kb][i][s2] (lo 2 + hi 2)
    if MSUM == 2:
        A.alloc("lsum", 8)   # tile row sums [j] (all 4 rows of a lane hold its query's sum)
        A.alloc("sel", 4)    # bf16 lane-group selector A operand (sum16_mfmas)
    elif MSUM:
        A.alloc("lsum", 32)  # tile row sums [j] (all 16 rows of a block hold the lane's sum)
        A.alloc("ones", 4)   # bf16 1.0 A operand
    return V, A


def sblk(V, par, p):
    return V.r(f"s{par}", 16 * p, 16)


def lds(V, base, off):
    """(base register, immediate) of an LDS byte offset `off` from a per-lane table entry."""
    if off >= HI:
        return V.r({"rowoff": "rowhi", "troff": "trhi"}[base[0]], base[1]), off - HI
    return V.r(base[0], base[1]), off


def k_reads(V, A, stage, kb):
    out = []
    for s in range(4):
        b, off = lds(V, ("rowoff", s), stage * STAGE + kb * 4096)
        out.append((f"ds_read_b128 {A.r('kf', 16 * kb + 4 * s, 4)}, {b} offset:{off}",
                    ("K", kb, s)))
    return out


def tr_reads(V, A, stage, kb):
    out = []
    for i in range(2):
        for s2 in range(2):
            for hi in range(2):
                b, off = lds(V, ("troff", 2 * i + hi), stage * STAGE + VOFF + kb * 4096 + s2 * 2048)
                out.append((f"ds_read_b64_tr_b16 {A.r('trf', 16 * kb + 8 * i + 4 * s2 + 2 * hi, 2)}"
                            f", {b} offset:{off}", ("T", kb, i, s2, hi)))
    return out


def g_mfmas(V, A, kb):
    out = []
    for i in range(2):
        for s2 in range(2):
            tr = A.r("trf", 16 * kb + 8 * i + 4 * s2, 4)
            for j in range(2):
                acc = A.r("acc", 16 * (2 * i + j), 16)
                pv = V.r("p", 8 * (2 * kb + j) + 4 * s2, 4)
                out.append((f"{MFMA} {acc}, {tr}, {pv}, {acc}", ()))
    return out


def sum_mfmas(V, A):
    """MSUM: lsum[j] = sum over the tile's 64 keys of P^T (bf16, the PV operand) for the
    lane's query -- ones[32 x 16] x P^T[kb][j][s2], both lane halves get the full sum."""
    out = []
    for j in range(2):
        acc = A.r("lsum", 16 * j, 16)
        for n, (kb, s2) in enumerate((kb, s2) for kb in range(2) for s2 in range(2)):
            c = "0" if n == 0 else acc
            out.append((f"{MFMA} {acc}, {A.r('ones', 0, 4)}, "
                        f"{V.r('p', 8 * (2 * kb + j) + 4 * s2, 4)}, {c}", ()))
    return out


def sum16_mfmas(V, A):
    """MSUM 2: lsum[j] = the tile's row sums of P^T (bf16) by v_mfma_f32_16x16x32_bf16.  The
    B operand of lane l = 16 g + n is its P^T quad: 8 keys of query 16 (g & 1) + n, key half
    g >> 1.  The A operand `sel` of lane 16 g + m is 1.0 where (g & 1) == ((m >> 2) & 1), so
    D row m (held by lane group m >> 2) sums the lane groups of the same query parity: every
    lane's 4 result rows are its own query's sum over both key halves of the 16-key chunk.
    The k order within a lane group does not matter (A and B lanes cover the same k)."""
    out = []
    for n, (kb, s2) in enumerate((kb, s2) for kb in range(2) for s2 in range(2)):
        for j in range(2):
            acc = A.r("lsum", 4 * j, 4)
            c = "0" if n == 0 else acc
            out.append((f"v_mfma_f32_16x16x32_bf16 {acc}, {A.r('sel', 0, 4)}, "
                        f"{V.r('p', 8 * (2 * kb + j) + 4 * s2, 4)}, {c}", ()))
    return out


def s_mfmas(V, A, par, kb, zero_c=False):
    """S'(kb) of both query blocks into accumulator set `par` (srcC: -m, or 0)."""
    out = []
    for s in range(4):
        for j in range(2):
            d = sblk(V, par, 2 * kb + j)
            c = ("0" if zero_c else V.r("negm", 16 * j, 16)) if s == 0 else d
            out.append((f"{MFMA} {d}, {A.r('kf', 16 * kb + 4 * s, 4)}, "
                        f"{A.r('qf', 16 * j + 4 * s, 4)}, {c}", (("K", kb, s),)))
    return out


# ------------------------------------------------------------------ softmax stream
COST = {"exp": 8.0, "add": 4.0, "cvt": 4.5, "cmp": 4.0, "cnd": 4.0}


def softmax_list(V, par, masked, u):
    """The VALU of one tile's softmax: [(text, cost, earliest gap)] in issue order.  Per
    score: v_exp_f32, an add into one of CHAINS row-sum accumulators of its query block
    (round robin, 4 scores behind its exp, so neither the exp result nor the accumulator's
    previous add is waited for), half a v_cvt_pk_bf16_f32.  A slot's bf16 P^T is written
    only after G(t-1) of the same key block has read the previous tile's (earliest gap).
    Masked tiles set keys >= n to -inf first (klim = keys left - 4 hh)."""
    kinds = {"v_exp_f32": 1, "v_add_f32": 2, "v_mov_b32": 2, "v_cvt_pk_bf16_f32": 4}
    gk = {0: 9, 1: 25} if GSGS else {0: 9, 1: 17}
    out = []
    if MSUM:
        for kb in range(2):
            for j in range(2):
                p = 2 * kb + j
                S = V[f"s{par}"] + 16 * p
                out += mask_list(V, S, masked, u, kb)
                for k in range(0, 8, 2):  # 4 exps, then their 2 packs (no trans hazard)
                    for x in range(4):
                        out.append((f"v_exp_f32 v{S + 2 * k + x}, v{S + 2 * k + x}",
                                    COST["exp"], 0))
                    for kk in (k, k + 1):
                        out.append((f"v_cvt_pk_bf16_f32 {V.r('p', 8 * p + kk)}, v{S + 2 * kk}, "
                                    f"v{S + 2 * kk + 1}", COST["cvt"], gk[kb]))
        return [it for it in out if not DROP & kinds.get(it[0].split()[0], 0)]
    if CHAINS == 1 and not LAG1:
        for kb in range(2):
            for j in range(2):
                p = 2 * kb + j
                S = V[f"s{par}"] + 16 * p
                ps = V.r("ps", j)
                out += mask_list(V, S, masked, u, kb)
                for k in range(8):
                    a, b = S + 2 * k, S + 2 * k + 1
                    out.append((f"v_exp_f32 v{a}, v{a}", COST["exp"], 0))
                    out.append((f"v_exp_f32 v{b}, v{b}", COST["exp"], 0))
                    if kb == 0 and k == 0:
                        out.append((f"v_add_f32 {ps}, v{a}, v{b}", COST["add"], 0))
                    else:
                        out.append((f"v_add_f32 {ps}, {ps}, v{a}", COST["add"], 0))
                        out.append((f"v_add_f32 {ps}, {ps}, v{b}", COST["add"], 0))
                    out.append((f"v_cvt_pk_bf16_f32 {V.r('p', 8 * p + k)}, v{a}, v{b}",
                                COST["cvt"], gk[kb]))
        return [it for it in out if not DROP & kinds.get(it[0].split()[0], 0)]
    # the tile's 64 scores in slot order; E = exp, A = accumulate (4 scores behind), C = cvt
    seq = []
    for kb in range(2):
        for j in range(2):
            for r in range(16):
                seq.append((kb, j, r))
    lag = 4
    for i in range(len(seq) + lag):
        if i < len(seq):
            kb, j, r = seq[i]
            p = 2 * kb + j
            S = V[f"s{par}"] + 16 * p
            if r == 0:
                out += mask_list(V, S, masked, u, kb)
            out.append((f"v_exp_f32 v{S + r}, v{S + r}", COST["exp"], 0))
        if i >= lag:
            kb, j, r = seq[i - lag]
            p = 2 * kb + j
            S = V[f"s{par}"] + 16 * p
            c = V.r("c", 4 * j + r % CHAINS)
            if kb == 0 and r < CHAINS:
                out.append((f"v_mov_b32 {c}, v{S + r}", COST["add"], 0))
            else:
                out.append((f"v_add_f32 {c}, {c}, v{S + r}", COST["add"], 0))
            if r % 2:
                k = r // 2
                out.append((f"v_cvt_pk_bf16_f32 {V.r('p', 8 * p + k)}, v{S + r - 1}, v{S + r}",
                            COST["cvt"], gk[kb]))
    # combine the accumulators of each query block into ps
    out += combine_list(V)
    return [it for it in out if not DROP & kinds.get(it[0].split()[0], 0)]


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


def mask_list(V, S, masked, u, kb):
    out = []
    if masked:
        for r in range(16):
            c = 64 * u + 32 * kb + (r & 3) + 8 * (r >> 2)
            out.append((f"v_cmp_lt_i32 vcc, {c}, {V.r('klim')}", COST["cmp"], 0))
            out.append((f"v_cndmask_b32 v{S + r}, {V.r('ninf')}, v{S + r}, vcc", COST["cnd"], 0))
    return out


def place(items, ngaps):
    """Greedy list schedule: gap g takes, in list order, the instructions whose earliest gap
    has come, until the gap's share of the total cost is used; an instruction held back by
    its earliest gap lets the later ones pass (only P^T writes are held back)."""
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
    r(f"v_readfirstlane_b32 {S_WAVE}, {V.r('tid')}")  # first lane's id = 64 * wave
    r("s_nop 1")
    r(f"s_lshr_b32 {S_WAVE}, {S_WAVE}, 6")
    r("s_getpc_b64 s[68:69]")
    r("s_add_u32 s68, s68, vd_attn_dq_lanes@rel32@lo+4")  # the dQ kernel's lane table
    r("s_addc_u32 s69, s69, vd_attn_dq_lanes@rel32@hi+12")
    # rare-path entry points: S_TGT + 2 v = .Lfwd_rare{v}
    r(f"s_getpc_b64 s[{S_TGT}:{S_TGT + 1}]")
    st.label(".Lfwd_pc")
    for v in (3, 2, 1, 0):
        r(f"s_add_u32 s{S_TGT + 2 * v}, s{S_TGT}, .Lfwd_rare{v}-.Lfwd_pc")
        r(f"s_addc_u32 s{S_TGT + 2 * v + 1}, s{S_TGT + 1}, 0")
    r("s_waitcnt lgkmcnt(0)")
    # seq = wgz * groups + wgy ; base = wgz * bs + wgy * gs ; obase likewise (bytes, 64-bit)
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
    # lse row: seq * n * 4 bytes, n * 4 bytes long
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
    e(f"v_lshlrev_b32 {t0}, 6, {V.r('tid')}")
    r(f"global_load_dwordx4 {V.r('rowoff', 0, 4)}, {t0}, {S_TAB}")
    r(f"global_load_dwordx4 {V.r('troff', 0, 4)}, {t0}, {S_TAB} offset:16")
    r(f"global_load_dwordx4 v[{V['dma']}:{V['dma'] + 3}], {t0}, {S_TAB} offset:32")
    qrow = [V.r("s1", 60), V.r("s1", 61)]
    hh16 = V.r("s1", 62)
    e(f"v_and_b32 {qrow[0]}, 31, {V.r('lane')}")
    e(f"v_add_u32 {qrow[0]}, {S_Q0}, {qrow[0]}")
    e(f"v_add_u32 {qrow[1]}, 32, {qrow[0]}")
    e(f"v_lshrrev_b32 {hh16}, 5, {V.r('lane')}")
    e(f"v_lshlrev_b32 {hh16}, 4, {hh16}")
    qv = V["s0"]  # Q fragments staged in v[s0 .. +31] for scaling
    for j in range(2):
        vq = V.r("s1", 56 + j)
        e(f"v_mul_lo_u32 {vq}, {qrow[j]}, s27")
        e(f"v_add_u32 {vq}, {vq}, {hh16}")
        for s in range(4):
            r(f"buffer_load_dwordx4 v[{qv + 16 * j + 4 * s}:{qv + 16 * j + 4 * s + 3}], {vq}, "
              f"{RQ}, 0 offen offset:{32 * s}")
        # O store offsets: qrow * ots_bytes + 8 hh
        e(f"v_lshrrev_b32 {V.r('s1', 54)}, 1, {hh16}")
        e(f"v_mul_lo_u32 {V.r('sto', j)}, {qrow[j]}, s28")
        e(f"v_add_u32 {V.r('sto', j)}, {V.r('sto', j)}, {V.r('s1', 54)}")
    # klim = keys in the last iteration - 4 hh
    e(f"v_lshrrev_b32 {t1}, 2, {hh16}")
    e(f"v_sub_u32 {V.r('klim')}, s43, {t1}")
    r("s_waitcnt vmcnt(0)")
    # Q' = bf16(Q * scale * log2 e), per bf16 element (attention.hip RowFrag::scale)
    for w in range(32):
        x = f"v{qv + w}"
        e(f"v_lshlrev_b32 {t0}, 16, {x}")
        e(f"v_and_b32 {t1}, 0xffff0000, {x}")
        e(f"v_mul_f32 {t0}, s38, {t0}")
        e(f"v_mul_f32 {t1}, s38, {t1}")
        e(f"v_cvt_pk_bf16_f32 {x}, {t0}, {t1}")
        e(f"v_accvgpr_write_b32 {A.r('qf', w)}, {x}")
    for k in range(4):
        e(f"v_add_u32 {V.r('rowhi', k)}, {HI:#x}, {V.r('rowoff', k)}")
        e(f"v_add_u32 {V.r('trhi', k)}, {HI:#x}, {V.r('troff', k)}")
    d0 = V["dma"]
    for i in range(2):
        e(f"v_mul_lo_u32 v{d0 + i}, v{d0 + i}, s27")
        e(f"v_add_u32 v{d0 + i}, v{d0 + i}, v{d0 + 2 + i}")
    # state: O = 0, l = 0, m = -inf (-m splat +inf), S'(0) = +inf (the first check fails),
    # G(-1) adds 0 (zero V^T fragments and P^T)
    for k in range(64):
        e(f"v_accvgpr_write_b32 {A.r('acc', k)}, 0")
    for k in range(32):
        e(f"v_accvgpr_write_b32 {A.r('trf', k)}, 0")
        e(f"v_mov_b32 {V.r('p', k)}, 0")
        e(f"v_mov_b32 {V.r('negm', k)}, {PINF}")
    for k in range(64):
        e(f"v_mov_b32 {V.r('s0', k)}, {PINF}")
    for j in range(2):
        e(f"v_mov_b32 {V.r('m', j)}, {NINF}")
        e(f"v_mov_b32 {V.r('l', j)}, 0")
        e(f"v_mov_b32 {V.r('ps', j)}, 0")
    e(f"v_mov_b32 {V.r('ninf')}, {NINF}")
    if MSUM == 2:  # sel (sum16_mfmas); the "tile -1" check of the first body passes (sum 0)
        t0, t1 = V.r("tmp", 0), V.r("tmp", 1)
        e(f"v_lshrrev_b32 {t0}, 2, {V.r('lane')}")
        e(f"v_lshrrev_b32 {t1}, 4, {V.r('lane')}")
        e(f"v_xor_b32 {t0}, {t0}, {t1}")
        e(f"v_and_b32 {t0}, 1, {t0}")
        e(f"v_cmp_eq_u32 vcc, 0, {t0}")
        e(f"v_mov_b32 {t1}, 0x3f803f80")
        e(f"v_cndmask_b32 {t0}, 0, {t1}, vcc")
        for k in range(4):
            e(f"v_accvgpr_write_b32 {A.r('sel', k)}, {t0}")
        for k in range(8):
            e(f"v_accvgpr_write_b32 {A.r('lsum', k)}, 0")
    elif MSUM:  # the "tile -1" check of the first body passes (sum 0)
        e(f"v_mov_b32 {V.r('tmp', 0)}, 0x3f803f80")
        for k in range(4):
            e(f"v_accvgpr_write_b32 {A.r('ones', k)}, {V.r('tmp', 0)}")
        for k in range(32):
            e(f"v_accvgpr_write_b32 {A.r('lsum', k)}, 0")
    for t in range(PD):
        dma_tile(st, V, t)


def dma_ops(V, stage):
    d0 = V["dma"]
    ops = []
    for x, rs in ((0, RK), (VOFF, RV)):
        for i in range(2):
            ops.append((f"s_add_u32 m0, {S_M0}, {stage * STAGE + x + i * 1024}",
                        f"buffer_load_dwordx4 v{d0 + i}, {rs}, 0 offen lds"))
    adv = [f"v_add_u32 v{d0 + i}, s41, v{d0 + i}" for i in range(2)]
    return ops, adv


def dma_tile(st: Stream, V, stage):
    ops, adv = dma_ops(V, stage)
    for m0, ld in ops:
        st.raw(m0)
        st.raw("s_nop 0")
        st.emit(ld)
    for a in adv:
        st.emit(a)


# ------------------------------------------------------------------ one body
def emit_check(st: Stream, V, A, u, masked, tag, msum):
    """Lagged-max check of the tile in stage u: any lane's tile sum >= 2^16 (or inf / NaN)
    -> the rare path; then l += the tile sum.  msum: the sum is read from the lsum MFMA
    accumulators (both lane halves hold the full sum)."""
    par = u % 2
    kst = (u + 1) % NST
    tc = V.r("tc", 0)
    if msum:
        for j in range(2):
            st.emit(f"v_accvgpr_read_b32 {V.r('ps', j)}, {A.r('lsum', (4 if MSUM == 2 else 16) * j)}")
    st.emit(f"v_max_f32 {tc}, {V.r('ps', 0)}, {V.r('ps', 1)}")
    st.emit(f"v_cmp_ngt_f32 vcc, 0x47800000, {tc}")
    if CHECK_NOP:
        st.raw(f"s_nop {CHECK_NOP}")
    st.raw(f"s_cbranch_vccz .Lfwd_ok{tag}")
    if NORARE:
        st.raw(f"s_branch .Lfwd_ok{tag}")
    st.raw(f"s_mov_b32 {S_ST}, {u * STAGE}")
    st.raw(f"s_mov_b32 {S_ST1}, {kst * STAGE}")
    st.raw(f"s_mov_b32 {S_KB}, {64 * u}")
    v = 2 * int(masked) + par
    st.raw(f"s_swappc_b64 {S_RET}, s[{S_TGT + 2 * v}:{S_TGT + 2 * v + 1}]")
    st.label(f".Lfwd_ok{tag}")
    for j in range(2):
        st.emit(f"v_add_f32 {V.r('l', j)}, {V.r('l', j)}, {V.r('ps', j)}")


def emit_body(st: Stream, V, A, u, masked, tag, prev=None):
    """Body of tile t (ring stage u = t mod 8): G(t-1), S(t+1), the softmax of tile t, the
    lagged-max check of tile t (MSUM: of tile t-1 at the top, prev = its (u, masked))."""
    par = u % 2
    st.comment(f"---- body, stage {u}{' (masked)' if masked else ''}")
    if MSUM:
        return emit_body_msum(st, V, A, u, masked, tag, prev)
    if not BAR2:
        st.raw(f"s_waitcnt vmcnt({(PD - 2) * 4}) lgkmcnt(0)")  # tile t+1 landed
        st.raw("s_barrier")
    elif u % 2 == 0:
        st.raw(f"s_waitcnt vmcnt({(PD - 3) * 4}) lgkmcnt(0)")  # tiles t+1, t+2 landed
        st.raw("s_barrier")
    else:
        st.raw("s_waitcnt lgkmcnt(0)")
    st.flush_lds()
    if GSGS:
        mf = (g_mfmas(V, A, 0) + s_mfmas(V, A, 1 - par, 0) + g_mfmas(V, A, 1)
              + s_mfmas(V, A, 1 - par, 1))
        rslots = (0, 8, 16, 24)
    else:
        mf = (g_mfmas(V, A, 0) + g_mfmas(V, A, 1) + s_mfmas(V, A, 1 - par, 0)
              + s_mfmas(V, A, 1 - par, 1))
        rslots = (2, 8, 12, 16)
    nm = len(mf)
    reads = {}

    def put(slot0, lst, per=2):
        for k, item in enumerate(lst):
            reads.setdefault(slot0 + k // per, []).append(item)

    kst = (u + 1) % NST
    if not DROP & 8:
        put(rslots[0], k_reads(V, A, kst, 0))  # K(t+1) rows, key block 0
        put(rslots[1], tr_reads(V, A, u, 0))   # V(t)^T, for G(t) in the next body
        put(rslots[2], k_reads(V, A, kst, 1))
        put(rslots[3], tr_reads(V, A, u, 1))
    ops, adv = dma_ops(V, (u + PD) % NST)
    slots4 = ((4, 12, 20, 28), (1, 9, 17, 25), (6, 14, 22, 30), (0, 8, 16, 24))[DMAS]
    dma_at = {} if DROP & 16 else {g: i for i, g in enumerate(slots4)}
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
    # lagged-max check of tile t: any lane's tile sum >= 2^16 (or inf / NaN) -> rare path
    emit_check(st, V, A, u, masked, tag, False)


def emit_body_msum(st: Stream, V, A, u, masked, tag, prev):
    """MSUM body t: the check of tile t-1 (prev) after the barrier, then
    G(t-1) kb0 | G(t-1) kb1 | S(t+1) kb0 | SUM(t) | S(t+1) kb1 (40 MFMAs) with tile t's
    softmax (exp + cvt only) in gaps 0..23, so P^T(t) is complete before SUM(t)."""
    par = u % 2
    st.raw(f"s_waitcnt vmcnt({(PD - 2) * 4}) lgkmcnt(0)")  # tile t+1 landed
    st.raw("s_barrier")
    st.flush_lds()
    if prev is not None:
        if u == 0 and not masked:
            st.raw("s_nop 7")  # the loop back edge: SUM(t-1) of the last body wrote lsum
        emit_check(st, V, A, prev[0], prev[1], f"c{tag}", True)
    if MSUM == 2:
        # G(t-1) kb0 | G(t-1) kb1 | S(t+1) kb0 | S(t+1) kb1 | SUM(t) (8 x 16x16x32); the
        # softmax over gaps 0..31 as in the adds body
        mf = (g_mfmas(V, A, 0) + g_mfmas(V, A, 1) + s_mfmas(V, A, 1 - par, 0)
              + s_mfmas(V, A, 1 - par, 1) + sum16_mfmas(V, A))
        rslots, dma_at, ngap = (2, 8, 12, 16), {4: 0, 12: 1, 20: 2, 28: 3}, 32
    else:
        mf = (g_mfmas(V, A, 0) + g_mfmas(V, A, 1) + s_mfmas(V, A, 1 - par, 0)
              + sum_mfmas(V, A) + s_mfmas(V, A, 1 - par, 1))
        rslots, dma_at, ngap = (2, 24, 12, 32), {4: 0, 12: 1, 34: 2, 38: 3}, 24
    nm = len(mf)
    reads = {}

    def put(slot0, lst, per=2):
        for k, item in enumerate(lst):
            reads.setdefault(slot0 + k // per, []).append(item)

    kst = (u + 1) % NST
    if not DROP & 8:
        put(rslots[0], k_reads(V, A, kst, 0))   # K(t+1) rows kb0
        put(rslots[2], k_reads(V, A, kst, 1))   # kb1
        put(rslots[1], tr_reads(V, A, u, 0))    # V(t)^T for G(t) in the next body
        put(rslots[3], tr_reads(V, A, u, 1))
    ops, adv = dma_ops(V, (u + PD) % NST)
    valu = place(softmax_list(V, par, masked, u), ngap)
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
        if g < ngap:
            for text in valu[g]:
                st.emit(text)
        text, deps = mf[g]
        st.emit(text, wait_lds=deps)


def emit_tail(st: Stream, V, A):
    st.comment("---- tail: G of the last tile")
    st.raw("s_waitcnt lgkmcnt(0)")
    st.flush_lds()
    for text, _ in g_mfmas(V, A, 0) + g_mfmas(V, A, 1):
        st.emit(text)


def epilogue(st: Stream, V, A):
    e = st.emit
    st.raw("s_waitcnt vmcnt(0)")
    t = [V["s0"] + k for k in range(8)]
    ad, lx, inv = V["s0"] + 8, V["s0"] + 10, V["s0"] + 12
    e(f"v_xor_b32 v{ad}, 32, {V.r('lane')}")
    e(f"v_lshlrev_b32 v{ad}, 2, v{ad}")
    if not MSUM:  # each lane half summed its own 32 keys of every tile
        for j in range(2):
            e(f"ds_bpermute_b32 v{lx + j}, v{ad}, {V.r('l', j)}")
        st.raw("s_waitcnt lgkmcnt(0)")
        for j in range(2):
            e(f"v_add_f32 {V.r('l', j)}, {V.r('l', j)}, v{lx + j}")
    for j in range(2):
        e(f"v_rcp_f32 v{inv + j}, {V.r('l', j)}")
    for j in range(2):
        for i in range(2):
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
    # lse = (m + log2 l) * ln 2 per query (both lane halves store the same value)
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
    """Subroutine .Lfwd_rare{2 masked + par}: S_ST / S_ST1 = ring offsets of tiles t / t+1,
    S_KB = tile t's first key within the masked iteration; returns through S_RET."""
    st = Stream()
    e, r = st.emit, st.raw
    st.label(f".Lfwd_rare{2 * int(masked) + par}")
    r("s_add_u32 s79, s79, 1")  # rare-path count (read by diagnostic probes only)
    r("s_nop 15")
    r("s_nop 15")
    r("s_waitcnt lgkmcnt(0)")
    ta = [V.r("p", k) for k in range(4)]  # P^T is rewritten below: scratch until then

    def reads_from(sreg):
        for s in range(4):
            e(f"v_add_u32 {ta[s]}, {sreg}, {V.r('rowoff', s)}")
        for kb in range(2):
            for s in range(4):
                e(f"ds_read_b128 {A.r('kf', 16 * kb + 4 * s, 4)}, {ta[s]} offset:{kb * 4096}",
                  lds_id=("K", kb, s))

    reads_from(S_ST)
    for kb in range(2):
        for text, deps in s_mfmas(V, A, par, kb, zero_c=True):
            e(text, wait_lds=deps)
    st.flush_lds()
    r("s_nop 15")
    r("s_nop 15")
    if masked:
        vl = V.r("p", 4)
        e(f"v_subrev_u32 {vl}, {S_KB}, {V.r('klim')}")
        for kb in range(2):
            for rr in range(16):
                c = 32 * kb + (rr & 3) + 8 * (rr >> 2)
                e(f"v_cmp_lt_i32 vcc, {c}, {vl}")
                for j in range(2):
                    x = V[f"s{par}"] + 16 * (2 * kb + j) + rr
                    e(f"v_cndmask_b32 v{x}, {V.r('ninf')}, v{x}, vcc")
    # true row max of tile t: 32 keys of the lane, then the other lane half
    mx, oth, ad, alpha = V["p"] + 8, V["p"] + 10, V["p"] + 12, V["p"] + 14
    for j in range(2):
        R = [V[f"s{par}"] + 16 * (2 * kb + j) + k for kb in range(2) for k in range(16)]
        e(f"v_max3_f32 v{mx + j}, v{R[0]}, v{R[1]}, v{R[2]}")
        for k in range(3, 31, 2):
            e(f"v_max3_f32 v{mx + j}, v{mx + j}, v{R[k]}, v{R[k + 1]}")
        e(f"v_max_f32 v{mx + j}, v{mx + j}, v{R[31]}")
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
        e(f"v_cmp_eq_f32 vcc, {m}, v{mx + j}")                    # equal (also -inf == -inf)
        e(f"v_cndmask_b32 v{alpha + j}, v{alpha + j}, 1.0, vcc")
        e(f"v_mov_b32 {m}, v{mx + j}")
        e(f"v_mul_f32 {l}, v{alpha + j}, {l}")
        e(f"v_xor_b32 v{oth + j}, 0x80000000, v{mx + j}")
        for k in range(16):
            e(f"v_mov_b32 {V.r('negm', 16 * j + k)}, v{oth + j}")
        tmp = [V.r("tmp", k) for k in range(4)]
        for i in range(2):
            for g in range(4):
                for k in range(4):
                    e(f"v_accvgpr_read_b32 {tmp[k]}, {A.r('acc', 16 * (2 * i + j) + 4 * g + k)}")
                for k in range(4):
                    e(f"v_mul_f32 {tmp[k]}, v{alpha + j}, {tmp[k]}")
                for k in range(4):
                    e(f"v_accvgpr_write_b32 {A.r('acc', 16 * (2 * i + j) + 4 * g + k)}, {tmp[k]}")
    # tile t's softmax against m_new (the m_new registers live in p[8..9], so slot 1's P^T
    # words 0..1 are written after both query blocks' subtractions)
    for j in range(2):
        for kb in range(2):
            S = V[f"s{par}"] + 16 * (2 * kb + j)
            for k in range(16):
                e(f"v_sub_f32 v{S + k}, v{S + k}, v{mx + j}")
    for kb in range(2):
        for j in range(2):
            p = 2 * kb + j
            S = V[f"s{par}"] + 16 * p
            ps = V.r("ps", j)
            for k in range(8):
                a, b = S + 2 * k, S + 2 * k + 1
                e(f"v_exp_f32 v{a}, v{a}")
                e(f"v_exp_f32 v{b}, v{b}")
                if kb == 0 and k == 0:
                    e(f"v_add_f32 {ps}, v{a}, v{b}")
                else:
                    e(f"v_add_f32 {ps}, {ps}, v{a}")
                    e(f"v_add_f32 {ps}, {ps}, v{b}")
                e(f"v_cvt_pk_bf16_f32 {V.r('p', 8 * p + k)}, v{a}, v{b}")
    if MSUM:  # the check's sums are per lane over both halves: add the partner half's
        t0, t1 = V.r("tmp", 0), V.r("tmp", 1)
        e(f"v_xor_b32 {t0}, 32, {V.r('lane')}")
        e(f"v_lshlrev_b32 {t0}, 2, {t0}")
        for j in range(2):
            e(f"ds_bpermute_b32 {V.r('tmp', 2 + j)}, {t0}, {V.r('ps', j)}")
        r("s_waitcnt lgkmcnt(0)")
        for j in range(2):
            e(f"v_add_f32 {V.r('ps', j)}, {V.r('ps', j)}, {V.r('tmp', 2 + j)}")
        del t1
    # S(t+1) against m_new
    ta = [V.r("tmp", k) for k in range(4)]
    reads_from(S_ST1)
    for kb in range(2):
        for text, deps in s_mfmas(V, A, 1 - par, kb):
            e(text, wait_lds=deps)
    st.flush_lds()
    r("s_nop 15")
    r("s_nop 15")
    r(f"s_setpc_b64 {S_RET}")
    return st


def emit_stamp(st: Stream, V):
    """STAMP builds: lane 0 of each wave stores (loop cycles, loop realtime ticks) at
    dbg[(wgx * 4 + wave) * 2] (dbg pointer at kernarg offset KARG)."""
    r = st.raw
    r("s_memtime s[94:95]")
    r("s_memrealtime s[72:73]")
    r(f"s_load_dwordx2 s[74:75], {S_KARG}, {KARG}")
    r("s_waitcnt lgkmcnt(0)")
    r("s_sub_u32 s94, s94, s90")
    r("s_sub_u32 s72, s72, s92")
    t0, t1, t2 = V.r("tmp", 0), V.r("tmp", 1), V.r("tmp", 2)
    r(f"s_lshl_b32 s70, {S_WGX}, 2")
    r(f"s_add_u32 s70, s70, {S_WAVE}")
    r("s_lshl_b32 s70, s70, 3")
    r(f"v_mov_b32 {t0}, s70")
    r(f"v_mov_b32 {t1}, s94")
    r(f"v_mov_b32 {t2}, s72")
    r("s_mov_b64 exec, 1")
    r(f"global_store_dword {t0}, {t1}, s[74:75]")
    r(f"global_store_dword {t0}, {t2}, s[74:75] offset:4")
    r("s_mov_b64 exec, -1")
    r("s_waitcnt vmcnt(0)")


def gen_fwd(probe=None):
    V, A = regs()
    assert V.next <= 256 and A.next <= 256, (V.next, A.next)
    st = Stream()
    prologue(st, V, A)
    if probe and probe[0] == "prologue":
        from gen_attn_asm import emit_probe
        emit_probe(st, probe[1], KARG, tmp=(V.r("tmp", 0), V.r("tmp", 1)))
    if STAMP:
        st.raw("s_memtime s[90:91]")
        st.raw("s_memrealtime s[92:93]")
    st.label(".Lfwd_loop")
    for u in range(NST):
        emit_body(st, V, A, u, False, f"{u}", prev=((u - 1) % NST, False))
    st.raw(f"s_sub_u32 {S_ITER}, {S_ITER}, 1")
    st.raw(f"s_cmp_lg_u32 {S_ITER}, 0")
    st.raw("s_cbranch_scc1 .Lfwd_loop")
    for u in range(NST):
        emit_body(st, V, A, u, True, f"m{u}", prev=((u - 1) % NST, u > 0))
    if MSUM:  # the last tile's check
        st.raw("s_waitcnt lgkmcnt(0)")
        emit_check(st, V, A, NST - 1, True, "last", True)
    emit_tail(st, V, A)
    if STAMP:
        emit_stamp(st, V)
    if probe and probe[0] == "loop":
        from gen_attn_asm import emit_probe
        emit_probe(st, probe[1], KARG, tmp=(V.r("tmp", 0), V.r("tmp", 1)))
    epilogue(st, V, A)
    body = st.text() + "\ts_endpgm\n"
    for masked in (False, True):
        for par in range(2):
            body += rare_path(V, A, par, masked).text()
    k = kernel_text("vd_attn_fwd_d64", body, vgprs=V.next, agprs=A.next, sgprs=96,
                    lds_bytes=NST * STAGE, kernarg_bytes=KARG + (8 if probe or STAMP else 0),
                    wg_size=64 * NW)
    return k, st
