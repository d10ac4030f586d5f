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
    # the bench's roofline unit (the head_dim-64 backward pair at N = 262144, one sequence per
    # launch: 8 N^2 D algorithmic FLOP) from these averages, to set beside roofline.frac
    dq, dkdv = rows.get("vd_attn_bwd_dq_d64"), rows.get("vd_attn_bwd_dkdv_d64")
    if dq and dkdv:
        unit_us = dq[1] / dq[0] / 1e3 + dkdv[1] / dkdv[0] / 1e3
        flop = 8.0 * 262144 ** 2 * 64
        print(f"\nD = 64 backward unit from these averages: {unit_us / 1e3:.3f} ms = "
              f"{flop / (unit_us * 1e-6) / 1e12:.1f} TFLOP/s algorithmic = "
              f"frac {flop / (unit_us * 1e-6) / 2.5e15:.4f} of 2.5 PF/s "
              f"(every launch of the process, warm-up and auxiliary legs included)")


if __name__ == "__main__":
    main(sys.argv[1])
