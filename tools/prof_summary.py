"""Summarise a rocprofv3 --kernel-trace database (rocpd sqlite) or kernel_stats.csv into
a per-kernel table: calls, total / average / min / max duration, share of GPU time.

    python tools/prof_summary.py gpurun_out/prof/run_results.db > profiles/rNN_kernel_stats.md
"""
import csv
import re
import sqlite3
import sys


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"\(.*\)$", "", name)  # drop the parameter list
    return name.replace("unsigned short", "bf16").replace("void ", "")


def from_db(path):
    c = sqlite3.connect(path)
    rows = {}
    for name, dur in c.execute("select name, duration from kernels"):
        r = rows.setdefault(short(name), [0, 0, float("inf"), 0])
        r[0] += 1
        r[1] += dur
        r[2] = min(r[2], dur)
        r[3] = max(r[3], dur)
    return rows


def from_csv(path):
    rows = {}
    with open(path) as f:
        for rec in csv.DictReader(f):
            rows[short(rec["Name"])] = [int(rec["Calls"]), float(rec["TotalDurationNs"]),
                                       float(rec["MinNs"]), float(rec["MaxNs"])]
    return rows


def main(path):
    rows = from_db(path) if path.endswith(".db") else from_csv(path)
    total = sum(r[1] for r in rows.values())
    print(f"# rocprofv3 kernel summary: {path}\n")
    print("| kernel | calls | total ms | avg us | min us | max us | % GPU time |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for name, (n, tot, mn, mx) in sorted(rows.items(), key=lambda kv: -kv[1][1]):
        print(f"| `{name}` | {n} | {tot / 1e6:.3f} | {tot / n / 1e3:.1f} | {mn / 1e3:.1f} | "
              f"{mx / 1e3:.1f} | {100 * tot / total:.2f} |")
    print(f"\nTotal kernel time: {total / 1e6:.3f} ms over {sum(r[0] for r in rows.values())} "
          f"dispatches")


if __name__ == "__main__":
    main(sys.argv[1])
