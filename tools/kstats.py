"""Per-kernel instruction counts from a device assembly file (hipcc -S --cuda-device-only):
MFMAs, v_exp, packed-f32 VALU (an anti-lever beside MFMAs, MI355X_MICROARCH.md), scratch
traffic and branches.  python tools/kstats.py /tmp/attn.s [filter]"""
import re
import sys

s = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
KEYS = ["v_mfma", "v_exp_f32", "v_pk_mul_f32", "v_pk_add_f32", "v_pk_fma_f32",
        "scratch_load", "scratch_store", "s_cbranch", "s_barrier"]
for m in re.finditer(r"^(_Z\S+):[^\n]*\n(.*?)\ts_endpgm", s, re.S | re.M):
    name, body = m.group(1), m.group(2)
    if flt not in name:
        continue
    short = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", name)
    short = re.sub(r"EEEvP.*", "", short)
    c = " ".join(f"{k.replace('v_', '').replace('_f32', '')}={len(re.findall(k, body))}" for k in KEYS)
    print(f"{short:46s} {c}")
