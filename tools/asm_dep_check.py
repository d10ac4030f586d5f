"""Dependence check of a generator knob (CPU only): builds a hand-scheduled kernel twice, with
the knob off and on, walks each straight-line text in program order and compares
  * for every MFMA (by ordinal): the registers it reads and, per register, the lineage of
    the value: the ordinal of the MFMA it derives from through VALU work;
  * for every VALU read of an MFMA result: (register, section, producing MFMA ordinal).
A VALU rewrite (packed adds / multiplies, reordering inside a slot) that keeps both equal
reads the same generation of every value the old schedule read.

    python tools/asm_dep_check.py fwd LAG1       # gen_fwd knob LAG1 0 vs 1: same dependences
    python tools/asm_dep_check.py fwd GSGS       # a different MFMA order: reports differences
(kernels: fwd, dq, dkdv, fwd128, dq128, dkdv128).  Used in round 5 for the packed-f32 softmax
variants (v_pk_add_f32 row sums, v_pk_mul_f32 P * dP; rejected).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lipreading-video-generation_amd", "csrc", "asm"))

from asmgen import Ins  # noqa: E402


def build(which, knob, val):
    import gen_attn_asm as G
    import gen_d128 as G128
    import gen_fwd as F
    import gen_fwd128 as F128
    mod, fn = {"fwd": (F, lambda: F.gen_fwd()[-1]), "dq": (G, lambda: G.gen_dq()[-1]),
               "dkdv": (G, lambda: G.gen_dkdv()[-1]),
               "fwd128": (F128, lambda: F128.gen_fwd128()[-1]),
               "dq128": (G128, lambda: G128.gen_dq128()[-1]),
               "dkdv128": (G128, lambda: G128.gen_dkdv128()[-1])}[which]
    old = getattr(mod, knob)
    setattr(mod, knob, val)
    try:
        return fn().text()  # the Stream
    finally:
        setattr(mod, knob, old)


def walk(text):
    """MFMA reads as (register, lineage): the ordinal of the MFMA whose result the value derives
    from (a VALU result inherits the newest MFMA lineage of its operands), or the section
    of the write for values without one; VALU reads of MFMA results as (register, ordinal)."""
    lin = {}       # reg -> lineage
    direct = {}    # reg -> ordinal of the MFMA that wrote it last (None after a VALU write)
    section = "prologue"
    nm = 0
    mfma_reads, valu_reads = [], set()
    for line in text.splitlines():
        t = line.strip()
        if t.startswith("; ----"):
            section = t[2:]
            continue
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        try:
            ins = Ins(t.split(";")[0])
        except Exception:
            continue
        if ins.kind not in ("mfma", "valu", "trans"):
            continue
        uses = ins.uses | (ins.srcc if ins.kind == "mfma" else set())
        if ins.kind == "mfma":
            mfma_reads.append(tuple(sorted((r, str(lin.get(r))) for r in uses)))
            for r in ins.defs:
                lin[r], direct[r] = nm, nm
            nm += 1
            continue
        for r in uses:
            if direct.get(r) is not None:
                valu_reads.add((r, direct[r]))
        ords = [lin[r] for r in uses if isinstance(lin.get(r), int)]
        for r in ins.defs:
            lin[r] = max(ords) if ords else ("valu", section)
            direct[r] = None
    return mfma_reads, valu_reads


def main():
    which, knob = sys.argv[1], sys.argv[2]
    a = walk(build(which, knob, 0))
    b = walk(build(which, knob, 1))
    bad = 0
    if len(a[0]) != len(b[0]):
        print(f"MFMA count differs: {len(a[0])} vs {len(b[0])}")
        bad += 1
    for i, (x, y) in enumerate(zip(a[0], b[0])):
        if x != y:
            bad += 1
            if bad <= 5:
                dx, dy = set(x) - set(y), set(y) - set(x)
                print(f"MFMA {i}: off-only {sorted(dx)[:4]} on-only {sorted(dy)[:4]}")
    if a[1] != b[1]:
        bad += 1
        print(f"VALU reads of MFMA results differ: off-only {sorted(a[1] - b[1])[:6]} "
              f"on-only {sorted(b[1] - a[1])[:6]}")
    print(f"{which} {knob}: {len(a[0])} MFMAs, {len(a[1])} VALU reads of MFMA results; "
          f"{'SAME dependences' if not bad else f'{bad} DIFFERENCES'}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
