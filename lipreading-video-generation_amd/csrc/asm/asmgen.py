"""Small assembler-text toolkit for the hand-scheduled gfx950 kernels (attn_asm.s).

The hot loops of the head_dim-64 attention kernels are emitted as explicit instruction
streams: MFMAs in a fixed order, with the softmax VALU work and the LDS fragment reads
placed into the gaps between them by position (MI355X_MICROARCH.md: per
v_mfma_f32_32x32x16_bf16 gap one wave can hide about 24 cycles of vector issue).  This
module provides
  * `Regs`  -- named register ranges (VGPR / AGPR / SGPR);
  * `Stream` -- an instruction list that tracks the wait-state hazards gfx950 does not
    interlock and pads them with s_nop, and derives the counted lgkmcnt waits of every
    consumer of an LDS read;
  * `kernel_text` -- the code object wrapper (.amdhsa_kernel descriptor + metadata).

Hazard distances (gfx950; measured from hipcc's own padding of the same instruction pairs, the
store-data rule from LLVM's hazard recognizer -- a VALU write of the data VGPRs of a VMEM store
wider than 64 bits needs 2 wait states between them on gfx940+):
MFMA 32x32x16 write -> VALU / VMEM / DS / MFMA-A/B read 12 wait states (16x16x32: 8); VALU write -> MFMA
read 2; transcendental write -> VALU read 2 (one instruction between); an MFMA reading its
own accumulator chain as srcC needs none.  Wait states are counted as issued instructions
(s_nop n = n + 1), which under-counts the cycles an MFMA occupies, so the padding is
conservative.
"""
from __future__ import annotations

import re


class Regs:
    """Named register ranges in one file ('v', 'a' or 's')."""

    def __init__(self, kind: str, start: int = 0):
        self.kind, self.next, self.names = kind, start, {}

    def alloc(self, name: str, n: int, align: int = 1) -> int:
        if self.next % align:
            self.next += align - self.next % align
        base = self.next
        self.names[name] = (base, n)
        self.next += n
        return base

    def __getitem__(self, name):
        return self.names[name][0]

    def r(self, name, off=0, n=1) -> str:
        b, size = self.names[name]
        assert off + n <= size, (name, off, n, size)
        return reg(self.kind, b + off, n)


def reg(kind: str, i: int, n: int = 1) -> str:
    return f"{kind}{i}" if n == 1 else f"{kind}[{i}:{i + n - 1}]"


_RANGE = re.compile(r"\b([vas])\[(\d+):(\d+)\]|\b([vas])(\d+)\b")


def regs_of(text: str) -> set:
    """Physical registers named in an operand string: {('v', 12), ('a', 3), ...}."""
    out = set()
    for m in _RANGE.finditer(text):
        if m.group(1):
            k, lo, hi = m.group(1), int(m.group(2)), int(m.group(3))
            out.update((k, i) for i in range(lo, hi + 1))
        else:
            out.add((m.group(4), int(m.group(5))))
    return out


def classify(op: str) -> str:
    if op.startswith("v_mfma"):
        return "mfma"
    if op in ("v_exp_f32", "v_log_f32", "v_rcp_f32", "v_rsq_f32", "v_sqrt_f32"):
        return "trans"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "ds"
    if op.startswith(("buffer_", "global_")):
        return "vmem"
    return "salu"


class Ins:
    __slots__ = ("text", "op", "kind", "defs", "uses", "srcc", "lds_id", "wait_lds", "sdata")

    def __init__(self, text, lds_id=None, wait_lds=()):
        self.text = text.strip()
        self.op = self.text.split()[0]
        self.kind = classify(self.op)
        ops = self.text[len(self.op):].split(",")
        ops = [o.strip() for o in ops]
        self.srcc = set()
        self.sdata = set()   # data VGPRs of a store wider than 64 bits
        if self.kind in ("mfma", "trans", "valu"):
            self.defs = regs_of(ops[0]) if ops and ops[0] else set()
            self.uses = set().union(*[regs_of(o) for o in ops[1:]]) if len(ops) > 1 else set()
            if self.kind == "mfma" and len(ops) >= 4:
                self.srcc = regs_of(ops[3])
        elif self.kind == "ds":
            if self.op.startswith("ds_read"):
                self.defs, self.uses = regs_of(ops[0]), regs_of(ops[1].split()[0])
            else:
                self.defs, self.uses = set(), set().union(*[regs_of(o.split()[0]) for o in ops])
        elif self.kind == "vmem":
            if "lds" in self.text.split() or self.op.startswith(("buffer_store", "global_store")):
                self.defs, self.uses = set(), set().union(*[regs_of(o.split()[0]) for o in ops])
                if self.op.endswith(("_dwordx3", "_dwordx4", "_b96", "_b128")) and \
                        "lds" not in self.text.split():
                    self.sdata = regs_of(ops[0].split()[0])
            else:
                self.defs = regs_of(ops[0])
                self.uses = set().union(*[regs_of(o.split()[0]) for o in ops[1:]])
        else:
            self.defs, self.uses = set(), set()
        self.lds_id = lds_id          # id of this LDS read (for counted waits)
        self.wait_lds = tuple(wait_lds)  # LDS read ids this instruction consumes


class Stream:
    """Straight-line instruction stream with hazard padding and counted lgkmcnt waits.

    Every ds_read must carry an lds_id; an instruction that consumes LDS-read results names
    them in wait_lds and gets the weakest `s_waitcnt lgkmcnt(k)` that covers them (reads
    complete in issue order).  Call `flush_lds()` to forget outstanding reads (after an
    explicit lgkmcnt(0))."""

    MFMA_RAW = 12      # MFMA write -> VALU / VMEM / DS / MFMA A-B read (and write)
    MFMA16_RAW = 8     # ... of a 16x16 (4-pass) MFMA (hipcc: s_nop 7 before the VALU read)
    VALU_TO_MFMA = 2   # VALU write -> MFMA read
    TRANS_RAW = 2      # transcendental write -> VALU read
    MFMA_WAR = 12      # VALU write of an in-flight MFMA's source
    STORE_DATA = 3     # VALU write of the data VGPRs of a VMEM store wider than 64 bits:
                       # 2 wait states between them (gfx940+, LLVM GCNHazardRecognizer; the
                       # distances here count the producing instruction itself)

    def __init__(self):
        self.lines = []
        self.hist = []        # (position, Ins) of the hazard-relevant recent instructions
        self.pos = 0          # wait states issued so far
        self.pending = []     # outstanding LDS read ids, issue order
        self.nops = 0
        self.waits = 0
        self.forced = 0   # waits forced by the 15-read limit
        self.young = 0    # ... of which waited on a read issued < 4 MFMAs earlier (a stall)
        self.nmfma = 0
        self.issued_at = {}

    def comment(self, text):
        self.lines.append(f"\t; {text}")

    def label(self, name):
        self.lines.append(f"{name}:")

    def raw(self, text, ws=1):
        """An instruction outside the hazard model (branches, barriers, SALU)."""
        self.lines.append("\t" + text)
        self.pos += ws

    def _need(self, ins: Ins) -> int:
        need = 0
        for p, h in reversed(self.hist):
            d = self.pos - p
            if d >= 13:
                break
            if h.kind == "mfma":
                raw = self.MFMA16_RAW if "_16x16x" in h.op else self.MFMA_RAW
                if ins.kind == "mfma":
                    # chained accumulator (srcC == the producer's dst) needs no padding
                    touched = (ins.uses - ins.srcc) & h.defs
                    if touched:
                        need = max(need, raw - d)
                elif (ins.uses | ins.defs) & h.defs:
                    need = max(need, raw - d)
                if ins.kind in ("valu", "trans", "ds", "vmem") and ins.defs & (h.uses | h.srcc):
                    need = max(need, self.MFMA_WAR - d)
            elif h.kind == "vmem":
                if ins.kind in ("valu", "trans") and ins.defs & h.sdata:
                    need = max(need, self.STORE_DATA - d)
            elif h.kind in ("valu", "trans"):
                if ins.kind == "mfma" and (ins.uses | ins.defs) & h.defs:
                    need = max(need, self.VALU_TO_MFMA - d)
                if h.kind == "trans" and ins.kind in ("valu", "trans", "vmem", "ds") \
                        and ins.uses & h.defs:
                    need = max(need, self.TRANS_RAW - d)
        return need

    def emit(self, text, lds_id=None, wait_lds=()):
        ins = Ins(text, lds_id, wait_lds)
        if ins.lds_id is not None and len(self.pending) >= 15:
            # lgkmcnt is a 4-bit counter: keep at most 15 LDS reads outstanding
            k = 14
            young = self.nmfma - self.issued_at.get(self.pending[0], -99) < 4
            self.young += young
            self.lines.append(f"\ts_waitcnt lgkmcnt({k})  ; forced: 15 reads in flight"
                              + (" (young)" if young else ""))
            self.pending = self.pending[len(self.pending) - k:]
            self.pos += 1
            self.waits += 1
            self.forced += 1
        if ins.wait_lds:
            idx = [self.pending.index(i) for i in ins.wait_lds if i in self.pending]
            if idx:
                k = len(self.pending) - 1 - max(idx)
                self.lines.append(f"\ts_waitcnt lgkmcnt({min(k, 15)})")
                self.pending = self.pending[max(idx) + 1:]
                self.pos += 1
                self.waits += 1
        need = self._need(ins)
        while need > 0:
            n = min(need, 16)
            self.lines.append(f"\ts_nop {n - 1}")
            self.pos += n
            self.nops += n
            need -= n
        self.lines.append("\t" + ins.text)
        if ins.lds_id is not None:
            self.pending.append(ins.lds_id)
            self.issued_at[ins.lds_id] = self.nmfma
        if ins.kind == "mfma":
            self.nmfma += 1
        if ins.kind in ("mfma", "valu", "trans") or ins.sdata:
            self.hist.append((self.pos, ins))
            if len(self.hist) > 64:
                self.hist = self.hist[-64:]
        self.pos += 1
        return ins

    def flush_lds(self):
        self.pending = []

    def text(self):
        return "\n".join(self.lines) + "\n"


# Code placement (MI355X_MICROARCH.md "Two waves per SIMD" item 8: a hand-written stream can
# lose ~13 % under a uniform 4-byte shift): kernels named here start with one s_nop 0, which
# shifts their whole instruction stream by 4 bytes.  PHASE_FLIP (A/B builds only:
# gen_attn_asm.py --phase=..., tools/build_asm_phase.sh): "all", or a comma list of kernel
# names, flips the phase of those kernels relative to this table.  The product build (make)
# never sets it, and nothing here reads the environment, so a leftover variable cannot
# shift the shipped code (advisor r04).
PHASE4 = set()
PHASE_FLIP = ""


def _phase4(name):
    flip = PHASE_FLIP == "all" or name in PHASE_FLIP.split(",")
    return (name in PHASE4) != flip


def kernel_text(name, body, *, vgprs, agprs, sgprs, lds_bytes, kernarg_bytes, wg_size,
                wg_ids=(1, 1, 1)):
    """(code + descriptor text, metadata entry) of one kernel (code object v5)."""
    accum = (vgprs + 3) // 4 * 4
    total = accum + agprs
    assert total <= 512, total
    pad = "\ts_nop 0\n" if _phase4(name) else ""
    code = f""".text
.globl {name}
.p2align 8
.type {name},@function
{name}:
{pad}{body}
\ts_endpgm
.Lfunc_end_{name}:
.size {name}, .Lfunc_end_{name}-{name}

.rodata
.p2align 6
.amdhsa_kernel {name}
  .amdhsa_group_segment_fixed_size {lds_bytes}
  .amdhsa_private_segment_fixed_size 0
  .amdhsa_kernarg_size {kernarg_bytes}
  .amdhsa_user_sgpr_count 2
  .amdhsa_user_sgpr_kernarg_segment_ptr 1
  .amdhsa_system_sgpr_workgroup_id_x {wg_ids[0]}
  .amdhsa_system_sgpr_workgroup_id_y {wg_ids[1]}
  .amdhsa_system_sgpr_workgroup_id_z {wg_ids[2]}
  .amdhsa_system_vgpr_workitem_id 0
  .amdhsa_next_free_vgpr {total}
  .amdhsa_next_free_sgpr {sgprs}
  .amdhsa_accum_offset {accum}
  .amdhsa_reserve_vcc 1
  .amdhsa_float_denorm_mode_32 3
  .amdhsa_float_denorm_mode_16_64 3
  .amdhsa_ieee_mode 1
  .amdhsa_dx10_clamp 1
.end_amdhsa_kernel
"""
    meta = f"""  - .name: {name}
    .symbol: {name}.kd
    .kernarg_segment_size: {kernarg_bytes}
    .group_segment_fixed_size: {lds_bytes}
    .private_segment_fixed_size: 0
    .kernarg_segment_align: 8
    .wavefront_size: 64
    .sgpr_count: {sgprs + 6}
    .vgpr_count: {total}
    .agpr_count: {agprs}
    .max_flat_workgroup_size: {wg_size}
    .args:
      - {{ .offset: 0, .size: {kernarg_bytes}, .value_kind: by_value }}
"""
    return code, meta


def code_object_text(kernels, data=""):
    """One .s holding several kernels: kernels = [(code, meta)], data = extra .rodata."""
    out = '.amdgcn_target "amdgcn-amd-amdhsa--gfx950"\n.amdhsa_code_object_version 5\n'
    out += "".join(c for c, _ in kernels)
    out += data
    out += "\n.amdgpu_metadata\n---\namdhsa.version: [ 1, 2 ]\namdhsa.kernels:\n"
    out += "".join(m for _, m in kernels)
    out += "...\n.end_amdgpu_metadata\n"
    return out
