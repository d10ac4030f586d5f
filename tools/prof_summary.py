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


def _grid_cols(c):
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    for cand in (("grid_size_x", "grid_size_y", "grid_size_z"), ("grid_x", "grid_y", "grid_z"),
                 ("grid_size",)):
        if all(x in cols for x in cand):
            return cand
    return ()


def from_db(path, by_grid=False):
    """{kernel: [calls, total ns, min, max]}; by_grid: keyed (kernel, grid) instead."""
    c = sqlite3.connect(path)
    g = _grid_cols(c) if by_grid else ()
    sel = ", ".join(("name", "duration") + g)
    rows = {}
    for rec in c.execute(f"select {sel} from kernels"):
        key = short(rec[0]) if not by_grid else (short(rec[0]), tuple(rec[2:]))
        r = rows.setdefault(key, [0, 0, float("inf"), 0])
        r[0] += 1
        r[1] += rec[1]
        r[2] = min(r[2], rec[1])
        r[3] = max(r[3], rec[1])
    return rows


def unit_line(path):
    """The bench's roofline unit (the head_dim-64 backward pair at N = 262144, one sequence per
    launch: 8 N^2 D algorithmic FLOP) from the launches of that grid only, (262144, 1, 1) in
    threads (the auxiliary spatial_temporal leg runs the same kernels per frame at N = 16384
    on other grids); None when the process ran no such launch."""
    rows = from_db(path, by_grid=True)
    best = {}
    for (name, grid), r in rows.items():
        # one N = 262144 sequence per launch: 1024 workgroups of 256 threads, z = 1
        if name in ("vd_attn_bwd_dq_d64", "vd_attn_bwd_dkdv_d64") and tuple(grid[:3]) == (262144, 1, 1):
            if name not in best or r[1] > best[name][1][1]:
                best[name] = (grid, r)
    if len(best) < 2:
        return None
    (gq, dq), (gk, dkdv) = best["vd_attn_bwd_dq_d64"], best["vd_attn_bwd_dkdv_d64"]
    unit_us = dq[1] / dq[0] / 1e3 + dkdv[1] / dkdv[0] / 1e3
    flop = 8.0 * 262144 ** 2 * 64
    return (f"D = 64 backward unit (grids dq {gq} x{dq[0]}, dk/dv {gk} x{dkdv[0]}): "
            f"{unit_us / 1e3:.3f} ms = {flop / (unit_us * 1e-6) / 1e12:.1f} TFLOP/s algorithmic "
            f"= frac {flop / (unit_us * 1e-6) / 2.5e15:.4f} of 2.5 PF/s (every launch of that "
            f"grid in the process, warm-up steps included)")


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
    if path.endswith(".db"):
        g = from_db(path, by_grid=True)
        print("\nHand-scheduled attention kernels by grid shape (the headline's joint launches "
              "and the auxiliary legs' per-frame / per-clip launches apart):\n")
        print("| kernel | grid | calls | total ms | avg us |")
        print("|---|---|---:|---:|---:|")
        for (name, grid), (n, tot, _, _) in sorted(g.items(), key=lambda kv: -kv[1][1]):
            if name.startswith("vd_attn_"):
                print(f"| `{name}` | {grid} | {n} | {tot / 1e6:.3f} | {tot / n / 1e3:.1f} |")
        line = unit_line(path)
        if line:
            print("\n" + line)


if __name__ == "__main__":
    main(sys.argv[1])
