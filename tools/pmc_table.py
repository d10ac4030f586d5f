"""Per-kernel mean of every PMC counter found under a rocprofv3 output tree (csv):
  python tools/pmc_table.py gpurun_out/pmcf [name substring, default attn_fwd]
  -> markdown table, one row per (run dir, kernel)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else "attn_fwd"
rows = defaultdict(lambda: defaultdict(list))
for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    run = os.path.relpath(path, root).split(os.sep)[0]
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            key = (r["Dispatch_Id"])
            names[key] = r["Kernel_Name"]
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    for key, cs in per.items():
        kn = names[key]
        if flt not in kn:
            continue
        short = kn.split("(")[0].replace("void ", "")[:60]
        for c, v in cs.items():
            rows[(run[:-1], short)][c].append(v)
merged = defaultdict(dict)
for (run, k), cs in rows.items():
    for c, vs in cs.items():
        merged[(run, k)][c] = sum(vs) / len(vs)
cols = sorted({c for d in merged.values() for c in d})
print("| run | kernel | " + " | ".join(cols) + " |")
print("|---|---|" + "---|" * len(cols))
for (run, k), d in sorted(merged.items()):
    print(f"| {run} | `{k}` | " + " | ".join(f"{d.get(c, float('nan')):.4g}" for c in cols) + " |")
