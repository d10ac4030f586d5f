"""Print VGPR / AGPR / scratch per kernel from a device assembly file (hipcc -S
--cuda-device-only), e.g. python tools/kregs.py /tmp/attn.s [filter]."""
import re
import sys

s = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for blk in re.finditer(r"\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", s, re.S):
    name, body = blk.group(1), blk.group(2)
    if flt not in name:
        continue
    g = lambda k: re.search(r"amdhsa_%s (\d+)" % k, body).group(1)
    short = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", name)
    short = re.sub(r"EEEvP.*", "", short)
    print(f"{short:50s} vgpr {g('next_free_vgpr'):>4s} accum_off {g('accum_offset'):>4s} "
          f"scratch {g('private_segment_fixed_size')}")
