"""Effective shader clock per kernel from a rocprofv3 GRBM_GUI_ACTIVE pass with
--kernel-trace (csv): GHz = GRBM_GUI_ACTIVE / XCDs / duration.
    python tools/clock_pmc.py <rocprofv3 -d dir> [xcds=8]"""
import csv
import glob
import sys

root = sys.argv[1]
xcds = int(sys.argv[2]) if len(sys.argv) > 2 else 8
pmc = glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)
kt = glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True)
dur = {}
for r in csv.DictReader(open(kt[0])):
    dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
agg = {}
for r in csv.DictReader(open(pmc[0])):
    if r["Counter_Name"] != "GRBM_GUI_ACTIVE" or r["Dispatch_Id"] not in dur:
        continue
    name = r["Kernel_Name"]
    name = name.replace("(anonymous namespace)::", "")
    name = (name[5:] if name.startswith("void ") else name).split("(")[0][:60]
    a = agg.setdefault(name, [0, 0.0, 0])
    a[0] += float(r["Counter_Value"])
    a[1] += dur[r["Dispatch_Id"]]
    a[2] += 1
print(f"{'kernel':60s} {'launches':>8s} {'ms':>9s} {'GHz':>6s}")
for name, (cyc, ns, n) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:12]:
    print(f"{name:60s} {n:8d} {ns / 1e6:9.2f} {cyc / xcds / ns:6.3f}")
