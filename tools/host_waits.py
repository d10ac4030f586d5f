"""Where does the host wait in a train step?  Reads a rocprofv3 --hip-trace --kernel-trace
database (a rocprofv3 --hip-runtime-trace run of bench.py) and prints, for the last complete step (steps cut at the
q_sample kernels), the HIP API calls that took longest on the host (a synchronising call
blocks until the GPU has drained) and the per-name totals of the calls that can block
(…Synchronize, hipMemcpy without Async, hipMalloc / hipFree, hipHostMalloc …).
    python tools/host_waits.py run_results.db"""
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    names = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
    api_src = None
    for cand in ("regions", "region", "hip_api", "api"):
        if cand in names:
            api_src = cand
            break
    if api_src is None:
        print("tables / views:", names)
        for n in names:
            try:
                cols = [d[1] for d in c.execute(f"pragma table_info('{n}')")]
                print(" ", n, cols)
            except sqlite3.Error:
                pass
        return 1
    cols = [d[1] for d in c.execute(f"pragma table_info('{api_src}')")]
    print(f"API source: {api_src} {cols}")
    ks = list(c.execute("select name, start, end from kernels order by start"))
    cuts = [s for n, s, e in ks if "QSample" in n]
    print(f"{len(cuts)} steps (q_sample launches)")
    if len(cuts) < 2:
        return 1
    lo, hi = cuts[-2], cuts[-1]
    api = list(c.execute(f"select name, start, end from {api_src} order by start"))
    step = [(n, s, e) for n, s, e in api if lo <= s < hi]
    tot = sum(e - s for n, s, e in step) / 1e6
    print(f"last complete step: {len(step)} API calls, {tot:.1f} ms inside them, step "
          f"{(hi - lo) / 1e6:.1f} ms")
    agg = {}
    for n, s, e in step:
        a = agg.setdefault(n, [0, 0.0, 0.0])
        a[0] += 1
        a[1] += (e - s) / 1e6
        a[2] = max(a[2], (e - s) / 1e6)
    print("per name (calls, total ms, max ms), by total:")
    for n, (k, t, m) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"   {n[:60]:60s} {k:6d} {t:9.3f} {m:8.3f}")
    print("longest single calls (ms, name, offset in step ms, kernels done before it):")
    kend = [e for n, s, e in ks]
    for n, s, e in sorted(step, key=lambda x: -(x[2] - x[1]))[:25]:
        done = sum(1 for ke in kend if lo <= ke <= s)
        print(f"   {(e - s) / 1e6:8.3f}  {n[:50]:50s} at {(s - lo) / 1e6:8.2f}  ({done} kernels)")
    return 0


if __name__ == "__main__" and len(sys.argv) == 2:
    sys.exit(main(sys.argv[1]))


def lead(path, step_index=2):
    """Launch lead per kernel of one step: kernel start - the start of the API call that
    launched it (joined on the correlation id).  A small lead where the GPU sits idle means
    the host was late; a large one, that the GPU waited on something else."""
    c = sqlite3.connect(path)
    kcols = [d[1] for d in c.execute("pragma table_info('kernels')")]
    cid = next((k for k in ("corr_id", "correlation_id", "kernel_id") if k in kcols), None)
    print("kernel columns:", kcols)
    if cid is None:
        return 1
    ks = list(c.execute(f"select name, start, end, {cid} from kernels order by start"))
    api = {r[0]: (r[1], r[2]) for r in c.execute("select corr_id, name, start from regions")}
    cuts = [s for n, s, e, _ in ks if "QSample" in n]
    lo, hi = cuts[step_index], cuts[step_index + 1]
    step = [(n, s, e, k) for n, s, e, k in ks if lo <= s < hi]
    prev_end = None
    rows = []
    for i, (n, s, e, k) in enumerate(step):
        a = api.get(k)
        ld = (s - a[1]) / 1e3 if a else float("nan")
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        rows.append((i, n[:48], ld, gap, a[0][:28] if a else "?"))
        prev_end = e if prev_end is None else max(prev_end, e)
    print(f"step {step_index}: {len(step)} kernels; the 20 largest idle gaps before a kernel "
          "(gap us, launch lead us = kernel start - its API call start):")
    for i, n, ld, gap, an in sorted(rows, key=lambda r: -r[3])[:20]:
        print(f"   #{i:5d} gap {gap:8.1f}  lead {ld:10.1f}  {n}  ({an})")
    for w0 in range(0, len(rows), 100):
        w = rows[w0:w0 + 100]
        leads = sorted(r[2] for r in w if r[2] == r[2])
        med = leads[len(leads) // 2] if leads else float("nan")
        print(f"   kernels {w0:5d}+: median lead {med:10.1f} us, idle {sum(r[3] for r in w) / 1e3:6.2f} ms")
    return 0


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[2] == "--lead":
    sys.exit(lead(sys.argv[1], int(sys.argv[3]) if len(sys.argv) > 3 else 2))
