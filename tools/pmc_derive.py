"""Derived per-kernel figures from a tools/pmc_attn.sh table: MFMA-busy (SQ_VALU_MFMA_BUSY_CYCLES
/ 1024 / (GRBM_GUI_ACTIVE / 8)), cycles, instruction mix per wave, LDS waits.
    python tools/pmc_derive.py gpurun_out/pmc_X/pmc_attn.md"""
import sys


def table(path):
    lines = open(path).read().splitlines()
    i = next(k for k, l in enumerate(lines) if l.startswith("| kernel"))
    hdr = [h.strip() for h in lines[i].split("|")[1:-1]]
    out = {}
    for l in lines[i + 2:]:
        c = [x.strip() for x in l.split("|")[1:-1]]
        if len(c) == len(hdr) and c[0]:
            out[c[0]] = dict(zip(hdr[1:], map(float, c[1:])))
    return out


def main():
    t = table(sys.argv[1])
    for k, r in sorted(t.items()):
        if not k.startswith("attn_"):
            continue
        cyc = r["GRBM_GUI_ACTIVE"] / 8
        w = r["SQ_WAVES"]
        print(f"{k:20s} MFMA-busy {100 * r['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / cyc:5.1f} %  "
              f"cycles {cyc:.3e}  per wave: VALU {r['SQ_INSTS_VALU'] / w:.3e} MFMA "
              f"{r['SQ_INSTS_MFMA'] / w:.3e} LDS {r['SQ_INSTS_LDS'] / w:.3e} SALU "
              f"{r['SQ_INSTS_SALU'] / w:.3e}  WAIT_INST_LDS/wave {r['SQ_WAIT_INST_LDS'] / w:.3e} "
              f"WAIT_ANY/wave {r['SQ_WAIT_ANY'] / w:.3e} WAVE_CYCLES/wave {r['SQ_WAVE_CYCLES'] / w:.3e}")


if __name__ == "__main__":
    main()
