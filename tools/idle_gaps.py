"""GPU idle time inside a run, from a rocprofv3 kernel trace (csv): the union of kernel
intervals against the span from the first to the last kernel, the idle gaps between
consecutive kernels binned by length, and the largest gaps with the kernels either side.
This is the time a HIP-graph replay of the same work could recover at most.
    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gap -- python3 bench.py --only train ...
    python tools/idle_gaps.py gpurun_out/gap/**/*kernel_trace.csv [--skip-ms 0]
"""
import argparse
import csv
import glob


def load(paths):
    rows = []
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("paths", nargs="+")
    ap.add_argument("--skip-ms", type=float, default=0.0,
                    help="ignore kernels starting in the first SKIP ms (warm-up, init)")
    ap.add_argument("--after", default="spin",
                    help="start after the last kernel whose name contains this (a marker)")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--steps", type=int, default=1, help="divide the per-kernel totals by this")
    a = ap.parse_args()
    paths = [q for p in a.paths for q in (glob.glob(p, recursive=True) or [p])]
    rows = load(paths)
    marks = [i for i, r in enumerate(rows) if a.after and a.after in r[2]]
    if marks:
        rows = rows[marks[-1] + 1:]
    t0 = rows[0][0] + int(a.skip_ms * 1e6)
    rows = [r for r in rows if r[0] >= t0]
    span = rows[-1][1] - rows[0][0]
    busy, end = 0, rows[0][0]
    gaps = []
    prev = None
    for s, e, n in rows:
        if s > end:
            gaps.append((s - end, prev, n))
        busy += max(0, e - max(s, end))
        end = max(end, e)
        prev = n
    idle = span - busy
    print(f"{len(rows)} kernels over {span / 1e6:.2f} ms: busy {busy / 1e6:.2f} ms, "
          f"idle {idle / 1e6:.3f} ms ({100 * idle / span:.2f} %)")
    bins = [(0, 2e3), (2e3, 1e4), (1e4, 5e4), (5e4, 1e12)]
    for lo, hi in bins:
        g = [x[0] for x in gaps if lo <= x[0] < hi]
        print(f"  gaps {lo / 1e3:6.0f}-{min(hi, 1e9) / 1e3:6.0f} us: {len(g):6d}, "
              f"{sum(g) / 1e6:8.3f} ms")
    for d, p, n in sorted(gaps, reverse=True)[:a.top]:
        print(f"  {d / 1e3:9.1f} us  after {(p or '')[:60]}  before {n[:60]}")
    per = {}
    for s, e, n in rows:
        c, t = per.get(n, (0, 0))
        per[n] = (c + 1, t + e - s)
    print(f"kernel time per step ({a.steps} steps in the window):")
    for n, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:3 * a.top]:
        print(f"  {t / 1e6 / a.steps:9.3f} ms  {c / a.steps:7.1f} launches  {n[:90]}")


if __name__ == "__main__":
    main()
