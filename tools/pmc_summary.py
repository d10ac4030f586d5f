"""Per-kernel derived PMC figures from a tools/pmc_conv.sh output tree:
   python tools/pmc_summary.py gpurun_out/r06e_pmc [kernel substring] [kernel us]
MFMA-busy = SQ_VALU_MFMA_BUSY_CYCLES / 1024 / (GRBM_GUI_ACTIVE / 8); per-wave instruction
counts; SQ_*_CYCLES / WAIT counters are quad-cycles (x4); FETCH_SIZE doubled (gfx950)."""
import collections
import csv
import glob
import sys

root, flt = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
us = float(sys.argv[3]) if len(sys.argv) > 3 else None
rows = collections.defaultdict(lambda: collections.defaultdict(list))
for p in glob.glob(f"{root}/p*/pmc_counter_collection.csv"):
    per, names = collections.defaultdict(dict), {}
    for r in csv.DictReader(open(p)):
        k = r["Dispatch_Id"]
        names[k] = r["Kernel_Name"]
        per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
    for k, cs in per.items():
        if flt not in names[k]:
            continue
        for c, v in cs.items():
            rows[names[k].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:70]][c].append(v)
for k, cs in rows.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    w = m.get("SQ_WAVES", 1)
    print(k)
    cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8
    if cyc:
        print(f"  MFMA-busy {m['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / cyc:.3f}"
              + (f"  clock {cyc / us / 1e3:.2f} GHz" if us else ""))
    print("  per wave: " + "  ".join(f"{c[8:] if c.startswith('SQ_INSTS') else c} {m[c] / w:.0f}"
                                      for c in sorted(m) if c.startswith("SQ_INSTS")))
    print("  per wave cycles: " + "  ".join(f"{c[3:]} {4 * m[c] / w:.0f}" for c in (
        "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
        "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_LDS")
        if c in m))
    if "SQ_LDS_IDX_ACTIVE" in m:
        print(f"  LDS cycles/wave {m['SQ_LDS_IDX_ACTIVE'] / w:.0f}, bank-conflict cycles/wave "
              f"{m.get('SQ_LDS_BANK_CONFLICT', 0) / w:.0f}")
    if "FETCH_SIZE" in m:
        print(f"  HBM fetch {m['FETCH_SIZE'] * 2 * 1024 / 1e6:.1f} MB per launch")
