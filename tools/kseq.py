"""Compact instruction-class sequence of one kernel's loops from a device assembly file:
M mfma, E v_exp, C v_cvt_pk, V other VALU, R ds_read, T ds_read_tr, D LDS-DMA, W s_waitcnt,
B s_barrier, S scalar, J branch.  python tools/kseq.py /tmp/attn.s kernel_substring"""
import re
import sys

s = open(sys.argv[1]).read()
flt = sys.argv[2]
for m in re.finditer(r"^(_Z\S+):[^\n]*\n(.*?)\ts_endpgm", s, re.S | re.M):
    name, body = m.group(1), m.group(2)
    if flt not in name:
        continue
    out = []
    for ln in body.split("\n"):
        ln = ln.strip()
        if not ln or ln.startswith(";") or ln.startswith("."):
            if ln.startswith(".LBB"):
                out.append("\n" + ln.split(":")[0] + ": ")
            continue
        op = ln.split()[0]
        if op.startswith("v_mfma"): c = "M"
        elif op.startswith("v_exp"): c = "E"
        elif op.startswith("v_cvt_pk"): c = "C"
        elif op.startswith("ds_read_b64_tr") or op.startswith("ds_read_tr"): c = "T"
        elif op.startswith("ds_read"): c = "R"
        elif op.startswith("buffer_load") and "lds" in ln: c = "D"
        elif op.startswith("s_waitcnt"): c = "W"
        elif op.startswith("s_barrier"): c = "B"
        elif op.startswith("s_cbranch") or op.startswith("s_branch"): c = "J"
        elif op.startswith("v_"): c = "V"
        elif op.startswith("s_"): c = "S"
        else: c = "?"
        out.append(c)
    print(name[:60])
    print("".join(out))
    break
