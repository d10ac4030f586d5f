"""Per-(kernel, grid) duration table from a rocprofv3 --kernel-trace database: separates
launches of one kernel at different shapes.  python tools/prof_dispatch.py run_results.db [substr]"""
import sqlite3
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import short  # noqa: E402

c = sqlite3.connect(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cur = c.execute("select * from kernels limit 1")
cols = [d[0] for d in cur.description]
grid = [x for x in cols if "grid" in x.lower() or "lds" in x.lower()]
rows = {}
for r in c.execute(f"select name, duration, {', '.join(grid) if grid else 0} from kernels"):
    name = short(r[0])
    if flt and flt not in name:
        continue
    key = (name, tuple(r[2:]))
    e = rows.setdefault(key, [0, 0.0])
    e[0] += 1
    e[1] += r[1]
print(f"| kernel | grid ({', '.join(grid)}) | calls | avg us |")
print("|---|---|---:|---:|")
for (name, g), (n, tot) in sorted(rows.items(), key=lambda kv: -kv[1][1]):
    print(f"| `{name}` | {g} | {n} | {tot / n / 1e3:.1f} |")
